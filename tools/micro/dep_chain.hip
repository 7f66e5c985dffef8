// Microbenchmark (tools/micro): the fp32 V24 softplus unit as DEPENDENT chains
// (h -> exp -> +1 -> log -> fma|h| -> acc), 8 chains per lane, either emitted chain by
// chain ("serial": dependent ops adjacent) or op by op across chains ("interleaved").
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f32x2 __attribute__((ext_vector_type(2)));

#define L1(h, u, s)  asm volatile("v_pk_fma_f32 %0, %1, %2, %2 op_sel:[0,0,1] op_sel_hi:[1,0,1]" : "=v"(h) : "v"(u), "s"(s))
#define EX(e, h)     asm volatile("v_exp_f32_e64 %0, -|%1|" : "=v"(e) : "v"(h))
#define K1(e)        asm volatile("v_pk_add_f32 %0, %0, 1.0 op_sel_hi:[1,0]" : "+v"(e))
#define LG(l, e)     asm volatile("v_log_f32 %0, %1" : "=v"(l) : "v"(e))
#define AF(t, h, l)  asm volatile("v_fma_f32 %0, |%1|, 0.5, %2" : "=v"(t) : "v"(h), "v"(l))
#define L2(acc, t, s) asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[1,0,1]" : "+v"(acc) : "v"(t), "s"(s))

template <int MODE, int NCH>
__global__ void __launch_bounds__(256) k(float* out, int n, float a) {
    f32x2 u = {threadIdx.x * 1e-3f, threadIdx.x * 2e-3f};
    const f32x2 s = {a, 0.25f};
    f32x2 acc[NCH];
    for (int j = 0; j < NCH; ++j) acc[j] = f32x2{0.f, 0.f};
    for (int i = 0; i < n; ++i) {
        if (MODE == 0) {           // serial
#pragma unroll
            for (int j = 0; j < NCH; ++j) {
                f32x2 h, e, l, t;
                L1(h, u, s);
                EX(e.x, h.x); EX(e.y, h.y);
                K1(e);
                LG(l.x, e.x); LG(l.y, e.y);
                AF(t.x, h.x, l.x); AF(t.y, h.y, l.y);
                L2(acc[j], t, s);
            }
        } else {                   // interleaved
            f32x2 h[NCH], e[NCH], l[NCH], t[NCH];
#pragma unroll
            for (int j = 0; j < NCH; ++j) L1(h[j], u, s);
#pragma unroll
            for (int j = 0; j < NCH; ++j) { EX(e[j].x, h[j].x); EX(e[j].y, h[j].y); }
#pragma unroll
            for (int j = 0; j < NCH; ++j) K1(e[j]);
#pragma unroll
            for (int j = 0; j < NCH; ++j) { LG(l[j].x, e[j].x); LG(l[j].y, e[j].y); }
#pragma unroll
            for (int j = 0; j < NCH; ++j) { AF(t[j].x, h[j].x, l[j].x); AF(t[j].y, h[j].y, l[j].y); }
#pragma unroll
            for (int j = 0; j < NCH; ++j) L2(acc[j], t[j], s);
        }
        u = u + acc[0] * 1e-9f;
    }
    float r = 0;
    for (int j = 0; j < NCH; ++j) r += acc[j].x + acc[j].y;
    out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <int MODE, int NCH>
void run(const char* name, float* d, int blocks, int n) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
        (void)hipEventRecord(e0);
        k<MODE, NCH><<<blocks, 256>>>(d, n, 0.999f);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    const double units = (double)blocks * 4 / 1024.0 * n * NCH;   // unit-pairs per SIMD
    printf("%-16s waves/SIMD %2d  %8.3f ms  %6.2f ns per unit (2 edges) per SIMD-wave\n", name,
           blocks * 4 / 1024, best, best * 1e6 / units);
}

int main() {
    const int n = 1024;
    float* d;
    (void)hipMalloc(&d, 256 * 64 * 256 * 4);
    for (int wps : {1, 2, 3, 4, 8}) {
        const int blocks = 256 * wps;
        run<0, 8>("serial x8", d, blocks, n);
        run<1, 8>("interleaved x8", d, blocks, n);
        run<1, 4>("interleaved x4", d, blocks, n);
        run<1, 16>("interleaved x16", d, blocks, n);
    }
    return 0;
}
