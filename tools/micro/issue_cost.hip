// issue_cost.hip — per-instruction VALU issue cost on gfx950 for the issue model of bench.py
// (MI355X_MICROARCH.md gives fp32 rows; this adds the fp64 / integer / select forms the fp64
// decoder_v2_4 MLP is made of).  One kernel per instruction, 8 independent register chains per
// lane, 2048 workgroups x 256 threads (8 waves per SIMD); prints ns per instruction per SIMD
// (= cycles / 2.4 at the 2.4 GHz clock).  usage: hipcc --offload-arch=gfx950 -O3 -o issue_cost
// issue_cost.hip && ./issue_cost
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x2 __attribute__((ext_vector_type(2)));
template <class T> __device__ __forceinline__ T mk(int t, int j) { return (T)(t * 1e-3 + j + 1); }
template <> __device__ __forceinline__ f32x2 mk<f32x2>(int t, int j) { return f32x2{t * 1e-3f + j + 1, 1.0f}; }
template <class T> __device__ __forceinline__ double tod(T v) { return (double)v; }
template <> __device__ __forceinline__ double tod<f32x2>(f32x2 v) { return (double)v.x + v.y; }
#define K(NAME, T, ASM, CONS)                                                                \
    __global__ void __launch_bounds__(256) k_##NAME(float* out, int n, float a) {           \
        T r[8];                                                                             \
        T b = mk<T>(0, 0) * (T)a;                                                           \
        for (int j = 0; j < 8; ++j) r[j] = mk<T>(threadIdx.x, j);                            \
        for (int i = 0; i < n; ++i) {                                                       \
            _Pragma("unroll") for (int j = 0; j < 8; ++j) asm volatile(ASM : "+v"(r[j]) : CONS(b)); \
        }                                                                                   \
        double s = 0;                                                                       \
        for (int j = 0; j < 8; ++j) s += tod(r[j]);                                         \
        out[blockIdx.x * 256 + threadIdx.x] = (float)s;                                     \
    }
#define V(x) "v"(x)
#define S(x) "s"(x)
#define NONE(x) "v"(x)
K(fma_f32, float, "v_fma_f32 %0, %0, %1, 0.5", V)
K(add_f32, float, "v_add_f32 %0, %0, %1", V)
K(exp_f32, float, "v_exp_f32 %0, %0", V)
K(rcp_f32, float, "v_rcp_f32 %0, %0", V)
K(fma_f64, double, "v_fma_f64 %0, %0, %1, 0.5", V)
K(add_f64, double, "v_add_f64 %0, %0, %1", V)
K(mul_f64, double, "v_mul_f64 %0, %0, %1", V)
K(max_f64, double, "v_max_f64 %0, %0, %1", V)
K(rcp_f64, double, "v_rcp_f64 %0, %0", V)
K(ldexp_f64, double, "v_ldexp_f64 %0, %0, 1", V)
K(add_u32, int, "v_add_u32 %0, %0, %1", V)
K(and_b32, int, "v_and_b32 %0, %0, %1", V)
K(cndmask_b32, int, "v_cndmask_b32 %0, %0, %1, vcc", V)
K(mov_b32, int, "v_mov_b32 %0, %1", V)
K(pk_fma_f32, f32x2, "v_pk_fma_f32 %0, %0, %1, %0", V)
K(pk_add_f32, f32x2, "v_pk_add_f32 %0, %0, %1", V)
K(pk_mul_f32, f32x2, "v_pk_mul_f32 %0, %0, %1", V)
K(fma_f32_sgpr, float, "v_fma_f32 %0, %0, %1, 0.5", S)
K(log_f32, float, "v_log_f32 %0, %0", V)
K(bfe_u32, int, "v_bfe_u32 %0, %0, 3, 7", NONE)
K(lshl_add_u64, long, "v_lshl_add_u64 %0, %0, 2, %1", V)
K(cndmask_sgpr, int, "v_cndmask_b32 %0, %0, %1, s[4:5]", V)

typedef void (*kfn)(float*, int, float);
static void run(const char* name, kfn f, float* d, int ops_per_iter) {
    const int blocks = 256 * 8, n = 2048;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    // clock ramp: ~150 ms of this kernel before the timed repetitions
    for (int rep = 0; rep < 300; ++rep) f<<<blocks, 256>>>(d, n, 0.999f);
    (void)hipDeviceSynchronize();
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
        (void)hipEventRecord(e0);
        f<<<blocks, 256>>>(d, n, 0.999f);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    const double ops = (double)blocks * 4 / 1024.0 * n * 8 * ops_per_iter;   // per SIMD
    printf("%-12s %8.3f ms  %6.3f ns per wave64 instruction per SIMD  (%4.1f cycles at 2.4 GHz)\n",
           name, best, best * 1e6 / ops, best * 1e6 / ops * 2.4);
}
int main() {
    float* d;
    (void)hipMalloc(&d, 256 * 8 * 256 * 4);
    run("fma_f32", k_fma_f32, d, 1);
    run("add_f32", k_add_f32, d, 1);
    run("exp_f32", k_exp_f32, d, 1);
    run("rcp_f32", k_rcp_f32, d, 1);
    run("fma_f64", k_fma_f64, d, 1);
    run("add_f64", k_add_f64, d, 1);
    run("mul_f64", k_mul_f64, d, 1);
    run("max_f64", k_max_f64, d, 1);
    run("rcp_f64", k_rcp_f64, d, 1);
    run("ldexp_f64", k_ldexp_f64, d, 1);
    run("add_u32", k_add_u32, d, 1);
    run("and_b32", k_and_b32, d, 1);
    run("cndmask_b32", k_cndmask_b32, d, 1);
    run("mov_b32", k_mov_b32, d, 1);
    run("pk_fma_f32", k_pk_fma_f32, d, 1);
    run("pk_add_f32", k_pk_add_f32, d, 1);
    run("pk_mul_f32", k_pk_mul_f32, d, 1);
    run("fma_f32_sgpr", k_fma_f32_sgpr, d, 1);
    run("log_f32", k_log_f32, d, 1);
    run("bfe_u32", k_bfe_u32, d, 1);
    run("lshl_add_u64", k_lshl_add_u64, d, 1);
    run("cndmask_sgpr", k_cndmask_sgpr, d, 1);
    return 0;
}
