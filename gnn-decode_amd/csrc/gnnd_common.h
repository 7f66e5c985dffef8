// gnnd_common.h — shared device/host helpers for libgnnd (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>
#include "../../include/gnnd.h"

#define GNND_BLOCK 256

// ---------------------------------------------------------------------------------------
// host-side graph (owned by libgnnd, device-resident tables built once per H)
// ---------------------------------------------------------------------------------------
struct GraphView {            // passed by value to kernels
    int V, C, E, N;
    int max_dv, max_dc;
    const uint32_t* edge_vc;  // [E]   v | (c << 16), reference edge order (sorted by v, c)
    const int* var_ptr;       // [V+1] edges of variable v are [var_ptr[v], var_ptr[v+1])
    const int* chk_ptr;       // [C+1]
    const int* chk_edge;      // [E]   edge ids of check c, increasing (= increasing v)
    // check-group slot plan of the fused decoder: check c owns G lanes x R slots,
    // slot (c, lane g, r) = c*G*R + g*R + r holds its edges in increasing order, padded.
    int G, logG, R;
    int padded;               // 1 if some check has fewer than G*R edges (padding slots exist)
    int padr;                 // most padding slots in one lane (trailing: lanes fill in order)
    const uint32_t* slot;     // [C*G*R]  variable of the slot's edge; GNND_SLOT_PAD if padding
    const int* vslot;         // [E]      slot of edge e (reference edge order = var-major)
    const uint32_t* slot_ve;  // [C*G*R]  v | (e << 16); padding = 0 | (E << 16) (dummy edge)
    // variables sorted by (degree, v): {v | dv << 16, first edge}.  Consecutive entries have
    // (nearly) equal degree, so lanes summing them run the same trip count.
    const uint2* var_ord;     // [V]
    // register-resident kernel's LDS message layout (gnnd_graph::rlay): variable-major
    // positions, each variable's edges padded with never-written zero slots to the largest
    // degree among the `vgroup` consecutive var_ord entries one wave sums together, so a
    // wave's variable sums run one uniform trip count with no masks.  vlay[i] = {v | dpad
    // << 16, first position} in var_ord order; slot_ve of the resident plans carries the
    // POSITION (not the edge id) in its high half; `spare` = the position padding slots and
    // idle items write; P1 = per-codeword stride (odd: bank-conflict-free codeword strides).
    // The identity layout (vgroup 1) is var_ord with positions = edge ids, spare = E.
    const uint2* vlay;        // [V]
    int vgroup, spare, P1;
};
#define GNND_SLOT_PAD 0x80000000u   // padding slot: variable 0, flag bit 31

struct gnnd_graph {
    GraphView view;           // slot plan of the streaming kernel (ties -> smaller R)
    GraphView rview;          // slot plan of the register-resident kernel (ties -> larger R)
    GraphView pview;          // ties -> R = 2: paired-edge fp32 V24 streaming at small batch
    GraphView rlay[7];        // rview with the padded message layout for vgroup 2^i (i = 0:
                              // identity); rlay[i].vlay == nullptr if it does not fit 16 bits
    void* dev;                // single device allocation holding every table
    size_t table_bytes;       // bytes of the four CSR/CSC tables (staged to LDS)
};

// int tables staged to LDS in this order: edge_vc[E], var_ptr[V+1], chk_ptr[C+1], chk_edge[E]
__host__ __device__ inline int graph_table_ints(int V, int C, int E) {
    return E + (V + 1) + (C + 1) + E;
}

int set_hip_error(hipError_t e);   // records e, returns GNND_ERR_HIP

#define GNND_HIP_CHECK(call)                                   \
    do {                                                       \
        hipError_t _e = (call);                                \
        if (_e != hipSuccess) return set_hip_error(_e);        \
    } while (0)

#define GNND_LAUNCH_CHECK()                                    \
    do {                                                       \
        hipError_t _e = hipGetLastError();                     \
        if (_e != hipSuccess) return set_hip_error(_e);        \
    } while (0)

// ---------------------------------------------------------------------------------------
// division by a runtime-constant divisor (Granlund-Montgomery, n < 2^31)
// ---------------------------------------------------------------------------------------
struct FastDiv {
    uint32_t d, m, s;
};
inline FastDiv make_fastdiv(uint32_t d) {
    FastDiv f;
    f.d = d;
    uint32_t l = 0;
    while ((1u << l) < d) ++l;
    f.s = l;
    f.m = (uint32_t)((((uint64_t)1 << 32) * (((uint64_t)1 << l) - d)) / d + 1);
    return f;
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
    return (__umulhi(n, f.m) + n) >> f.s;
}

// ---------------------------------------------------------------------------------------
// scalar math with reference (torch CPU) semantics, float and double overloads
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ float g_tanh(float x) { return tanhf(x); }
__device__ __forceinline__ float g_log(float x) { return logf(x); }
__device__ __forceinline__ float g_exp(float x) { return expf(x); }
__device__ __forceinline__ float g_log1p(float x) { return log1pf(x); }
__device__ __forceinline__ double g_log1p(double x) { return log1p(x); }
__device__ __forceinline__ float g_cos(float x) { return cosf(x); }
__device__ __forceinline__ double g_cos(double x) { return cos(x); }
__device__ __forceinline__ float g_abs(float x) { return fabsf(x); }
__device__ __forceinline__ double g_abs(double x) { return fabs(x); }
template <typename T> __device__ __forceinline__ T g_fma(T a, T b, T c) { return fma(a, b, c); }
template <typename T> __device__ __forceinline__ T g_min(T a, T b) { return a < b ? a : b; }
template <typename T> __device__ __forceinline__ T g_max(T a, T b) { return a > b ? a : b; }
// torch.clamp(x, lo, hi) (NaN propagates)
template <typename T> __device__ __forceinline__ T g_clamp(T x, T lo, T hi) {
    return x < lo ? lo : (x > hi ? hi : x);
}

// torch.nn.Softplus (beta 1, threshold 20): x > 20 ? x : log1p(exp(x)) — fp64, evaluated as
// max(x, 0) + log1p(exp(-|x|)) without libm (libm's exp + double-double log1p cost 177 VALU
// ops on gfx950; this form 54).  exp: k = rint(a log2e), r = a - k ln2 (two-part ln2),
// degree-13 Taylor on |r| <= 0.347 (truncation < 2e-16), ldexp.  log1p(u), u in (0, 1]:
// m = 1 + u with its exact rounding error c = u - (m - 1); m' = m or m/2 in [0.707, 1.414];
// log m' = 2 atanh(s), s = (m' - 1) / (m' + 1) (one Newton-refined v_rcp_f64), odd series
// to s^21 (|s| <= 0.172: truncation < 1e-16 relative); + j ln2 + c/m.  A few ulp of
// libm, far inside the fp64 parity tolerance (1e-10 relative on decoder outputs).
// polynomial coefficients in constant memory: uniform scalar loads keep them in SGPRs
// (a 64-bit literal cannot feed a VOP3 v_fma_f64; as literals every Horner step costs a
// v_mov_b64 into the v_fmac accumulator)
__constant__ static const double kSpCoef[23] = {
    1.0 / 6227020800.0, 1.0 / 479001600.0, 1.0 / 39916800.0, 1.0 / 3628800.0,   // exp: 1/13!..
    1.0 / 362880.0, 1.0 / 40320.0, 1.0 / 5040.0, 1.0 / 720.0, 1.0 / 120.0, 1.0 / 24.0,
    1.0 / 6.0, 0.5, 1.0,
    1.0 / 21.0, 1.0 / 19.0, 1.0 / 17.0, 1.0 / 15.0, 1.0 / 13.0, 1.0 / 11.0,      // atanh
    1.0 / 9.0, 1.0 / 7.0, 1.0 / 5.0, 1.0 / 3.0};
__device__ __forceinline__ double exp_nonpos_f64(double a) {          // a <= 0
    a = a > -750.0 ? a : -750.0;                                       // exp(-750) == 0
    const double k = __builtin_rint(a * 1.4426950408889634);
    double r = __builtin_fma(-k, 6.93147180369123816490e-01, a);       // ln2 hi
    r = __builtin_fma(-k, 1.90821492927058770002e-10, r);              // ln2 lo
    double p = kSpCoef[0];
#pragma unroll
    for (int i = 1; i < 13; ++i) p = __builtin_fma(p, r, kSpCoef[i]);
    p = __builtin_fma(p, r, 1.0);
    return __builtin_ldexp(p, (int)k);
}
__device__ __forceinline__ double log1p_unit_f64(double u) {          // u in [0, 1]
    const double m = 1.0 + u;
    const double c = u - (m - 1.0);                                    // exact
    const bool hi = m > 1.4142135623730951;
    const double mp = hi ? 0.5 * m : m;
    const double f = mp - 1.0;                                         // exact (Sterbenz)
    const double d = 2.0 + f;
    double rc = __builtin_amdgcn_rcp(d);
    rc = __builtin_fma(__builtin_fma(-d, rc, 1.0), rc, rc);
    double s = f * rc;
    s = __builtin_fma(__builtin_fma(-s, d, f), rc, s);                 // f / d, ~0.5 ulp
    const double z = s * s;
    double q = kSpCoef[13];
#pragma unroll
    for (int i = 14; i < 23; ++i) q = __builtin_fma(q, z, kSpCoef[i]);
    const double s2 = s + s;
    double l = __builtin_fma(s2 * z, q, s2);                           // log m'
    l = hi ? l + 6.93147180559945309417e-01 : l;
    return __builtin_fma(c, __builtin_amdgcn_rcp(m), l);               // + c / m
}
// branch-free: both sides evaluated, selected at the end
__device__ __forceinline__ double softplus_ref(double x) {
    const double r = log1p_unit_f64(exp_nonpos_f64(-__builtin_fabs(x)));
    const double y = x > 0.0 ? x + r : r;
    return x > 20.0 ? x : y;
}
// fp64 exp / log / tanh for the decoders' fp64 (reference-dtype) paths, same scheme as the
// Softplus above: no libm branches or double-double tails, a few ulp.
__device__ __forceinline__ double exp_poly_f64(double r) {           // e^r, |r| <= 0.347
    double p = kSpCoef[0];
#pragma unroll
    for (int i = 1; i < 13; ++i) p = __builtin_fma(p, r, kSpCoef[i]);
    return __builtin_fma(p, r, 1.0);
}
__device__ __forceinline__ double g_exp(double x) {
    x = __builtin_fmin(__builtin_fmax(x, -750.0), 710.0);
    const double k = __builtin_rint(x * 1.4426950408889634);
    double r = __builtin_fma(-k, 6.93147180369123816490e-01, x);
    r = __builtin_fma(-k, 1.90821492927058770002e-10, r);
    return __builtin_ldexp(exp_poly_f64(r), (int)k);
}
// expm1 without cancellation: 2^k (e^r - 1) + (2^k - 1), e^r - 1 = r P(r) by the Taylor
// series (no leading 1); exact path at k = 0
__device__ __forceinline__ double expm1_f64(double x) {
    x = __builtin_fmin(__builtin_fmax(x, -750.0), 710.0);
    const double k = __builtin_rint(x * 1.4426950408889634);
    double r = __builtin_fma(-k, 6.93147180369123816490e-01, x);
    r = __builtin_fma(-k, 1.90821492927058770002e-10, r);
    double p = kSpCoef[0];
#pragma unroll
    for (int i = 1; i < 13; ++i) p = __builtin_fma(p, r, kSpCoef[i]);
    const double em = r * p;                                           // e^r - 1 = r (1 + r/2 + ...)
    const double tk = __builtin_ldexp(1.0, (int)k);
    return __builtin_fma(tk, em, tk - 1.0);
}
__device__ __forceinline__ double g_log(double x) {                   // x > 0, normal
    int e = __builtin_amdgcn_frexp_exp(x);
    double m = __builtin_amdgcn_frexp_mant(x);                         // [0.5, 1)
    const bool lo = m < 0.7071067811865476;
    m = lo ? m + m : m;
    e = lo ? e - 1 : e;
    const double f = m - 1.0;                                          // exact
    const double d = 2.0 + f;
    double rc = __builtin_amdgcn_rcp(d);
    rc = __builtin_fma(__builtin_fma(-d, rc, 1.0), rc, rc);
    double s = f * rc;
    s = __builtin_fma(__builtin_fma(-s, d, f), rc, s);
    const double z = s * s;
    double q = kSpCoef[13];
#pragma unroll
    for (int i = 14; i < 23; ++i) q = __builtin_fma(q, z, kSpCoef[i]);
    const double s2 = s + s;
    const double l = __builtin_fma(s2 * z, q, s2);
    const double de = (double)e;
    return __builtin_fma(de, 6.93147180369123816490e-01, __builtin_fma(de, 1.90821492927058770002e-10, l));
}
// tanh(x) = -expm1(-2|x|) / (2 + expm1(-2|x|)), sign restored
__device__ __forceinline__ double g_tanh(double x) {
    const double em = expm1_f64(-2.0 * __builtin_fabs(x));
    const double d = 2.0 + em;                                         // (1, 2]
    double rc = __builtin_amdgcn_rcp(d);
    rc = __builtin_fma(__builtin_fma(-d, rc, 1.0), rc, rc);
    double t = -em * rc;
    t = __builtin_fma(__builtin_fma(t, d, em), -rc, t);                // -em / d, ~0.5 ulp
    return __builtin_copysign(t, x);
}
template <typename T> __device__ __forceinline__ T sigmoid_ref(T x) {
    return T(1) / (T(1) + g_exp(-x));
}

// (-1)^k for an integer-valued k; equals torch.cos(pi * k) exactly for |k| < ~1e3
// (cos of k*pi rounded rounds to +-1 in both precisions), falling back to cos otherwise.
template <typename T> __device__ __forceinline__ T cos_pi(T k) {
    T r = rint(k);
    if (r == k && g_abs(k) < T(1024)) {
        int ki = (int)r;
        return (ki & 1) ? T(-1) : T(1);
    }
    return g_cos(T(M_PI) * k);
}

// ---------------------------------------------------------------------------------------
// all-reduce sum over aligned groups of G lanes (G a power of two <= 64, wave-uniform).
// Every lane of a group ends with the identical value (each step adds two operands in
// both orders, and fp addition is commutative).  DPP for the in-row steps.
// ---------------------------------------------------------------------------------------
template <int CTRL> __device__ __forceinline__ float dpp_mov(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float group_sum(float v, int G) {
    if (G > 1) v += dpp_mov<0xB1>(v);    // quad_perm [1,0,3,2]  (lane ^ 1)
    if (G > 2) v += dpp_mov<0x4E>(v);    // quad_perm [2,3,0,1]  (lane ^ 2)
    if (G > 4) v += dpp_mov<0x141>(v);   // row_half_mirror      (other quad of the 8)
    if (G > 8) v += dpp_mov<0x140>(v);   // row_mirror           (other 8 of the 16)
    if (G > 16) v += __shfl_xor(v, 16);
    if (G > 32) v += __shfl_xor(v, 32);
    return v;
}
// compile-time group size: the butterfly is straight-line code (no uniform branches
// splitting the caller's basic block, so independent work items interleave)
template <int G> __device__ __forceinline__ float group_sum_c(float v) {
    if constexpr (G > 1) v += dpp_mov<0xB1>(v);
    if constexpr (G > 2) v += dpp_mov<0x4E>(v);
    if constexpr (G > 4) v += dpp_mov<0x141>(v);
    if constexpr (G > 8) v += dpp_mov<0x140>(v);
    if constexpr (G > 16) v += __shfl_xor(v, 16);
    if constexpr (G > 32) v += __shfl_xor(v, 32);
    return v;
}
// fp64: the same butterfly, each step moving the two 32-bit halves with DPP
template <int CTRL> __device__ __forceinline__ double dpp_mov(double v) {
    const int2 h = __builtin_bit_cast(int2, v);
    const int2 r = {__builtin_amdgcn_update_dpp(0, h.x, CTRL, 0xf, 0xf, false),
                    __builtin_amdgcn_update_dpp(0, h.y, CTRL, 0xf, 0xf, false)};
    return __builtin_bit_cast(double, r);
}
template <int G> __device__ __forceinline__ double group_sum_c(double v) {
    if constexpr (G > 1) v += dpp_mov<0xB1>(v);
    if constexpr (G > 2) v += dpp_mov<0x4E>(v);
    if constexpr (G > 4) v += dpp_mov<0x141>(v);
    if constexpr (G > 8) v += dpp_mov<0x140>(v);
    if constexpr (G > 16) v += __shfl_xor(v, 16);
    if constexpr (G > 32) v += __shfl_xor(v, 32);
    return v;
}
__device__ __forceinline__ double group_sum(double v, int G) {
    for (int o = 1; o < G; o <<= 1) v += __shfl_xor(v, o);
    return v;
}

// tanh(a/2) on the native base-2 exp and reciprocal (fp32 GNN path):
// tanh(a/2) = sign(a) (1 - e) / (1 + e), e = exp(-|a|) in (0, 1].  Absolute error ~1e-7
// (1 - e is exact for e >= 1/2), i.e. at the rounding level of the reference's sums.
__device__ __forceinline__ float tanh_half_fast(float a) {
    float e = __builtin_amdgcn_exp2f(fabsf(a) * -1.4426950408889634f);
    float t = (1.0f - e) * __builtin_amdgcn_rcpf(1.0f + e);
    return copysignf(t, a);
}
__device__ __forceinline__ double tanh_half_fast(double a) { return g_tanh(a / 2.0); }
// tanh(a/2) from the base-2 scaled argument a2 = a * log2(e):  1 - 2 / (1 + 2^a2).
// Saturates to +-1 (2^a2 -> inf or 0), never NaN; absolute error ~1.5e-7 near 0, i.e.
// below the rounding of the 24-term check sums it feeds.  4 VALU ops, 2 transcendental.
__device__ __forceinline__ float tanh_half_base2(float a2) {
    const float r = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(a2));
    return __builtin_fmaf(-2.0f, r, 1.0f);
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
