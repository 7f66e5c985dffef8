// Microbenchmark (tools/micro): issue cost of v_exp_f32 / v_log_f32 vs v_fma_f32 /
// v_pk_fma_f32 on gfx950, and whether transcendentals overlap plain VALU work.
// Each lane runs 8 independent chains per op kind (inline asm: exact instruction mix).
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f32x2 __attribute__((ext_vector_type(2)));

#define EXP(r) asm volatile("v_exp_f32 %0, %0" : "+v"(r))
#define LOG(r) asm volatile("v_log_f32 %0, %0" : "+v"(r))
#define FMA(r) asm volatile("v_fma_f32 %0, %0, %1, 0.5" : "+v"(r) : "v"(a))
#define PKF(r) asm volatile("v_pk_fma_f32 %0, %0, %1, %0" : "+v"(r) : "v"(aa))

template <int NE, int NL, int NF, int NP>
__global__ void __launch_bounds__(256) k(float* out, int n, float a) {
    float v[8], w[8];
    f32x2 p[8];
    const f32x2 aa = {a, a};
    for (int j = 0; j < 8; ++j) { v[j] = threadIdx.x * 1e-3f + j; w[j] = v[j] * 0.5f; p[j] = f32x2{v[j], w[j]}; }
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (j < NE) EXP(v[j]);
            if (j < NL) LOG(v[j]);
            if (j < NF) FMA(w[j]);
            if (j < NP) PKF(p[j]);
            if (NF > 8) FMA(w[j]);
        }
    }
    float s = 0;
    for (int j = 0; j < 8; ++j) s += v[j] + w[j] + p[j].x + p[j].y;
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int NE, int NL, int NF, int NP>
void run(const char* name, float* d, int blocks, int n) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
        (void)hipEventRecord(e0);
        k<NE, NL, NF, NP><<<blocks, 256>>>(d, n, 0.999f);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    // per SIMD: blocks*4 waves / 1024 SIMDs, each n iterations
    const double iters_per_simd = (double)blocks * 4 / 1024.0 * n;
    printf("%-28s %8.3f ms  %7.2f ns per loop-iteration per SIMD-wave  (%.1f cyc@2.4GHz)\n", name,
           best, best * 1e6 / iters_per_simd, best * 1e6 / iters_per_simd * 2.4);
}

int main() {
    const int blocks = 256 * 8, n = 4096;
    float* d;
    (void)hipMalloc(&d, blocks * 256 * 4);
    run<8, 0, 0, 0>("8 exp", d, blocks, n);
    run<0, 8, 0, 0>("8 log", d, blocks, n);
    run<0, 0, 8, 0>("8 fma", d, blocks, n);
    run<0, 0, 0, 8>("8 pk_fma", d, blocks, n);
    run<8, 0, 8, 0>("8 exp + 8 fma", d, blocks, n);
    run<8, 0, 0, 8>("8 exp + 8 pk_fma", d, blocks, n);
    run<8, 0, 16, 0>("8 exp + 16 fma", d, blocks, n);
    run<4, 0, 8, 0>("4 exp + 8 fma", d, blocks, n);
    run<8, 8, 0, 0>("8 exp + 8 log", d, blocks, n);
    return 0;
}
