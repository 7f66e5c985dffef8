// gnnd_common.h — shared device/host helpers for libgnnd (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>
#include "../../include/gnnd.h"

#ifndef GNND_BLOCK
#define GNND_BLOCK 256            // threads per decode workgroup (tuning variants: -DGNND_BLOCK=128)
#endif

// Planner A/B switches (GNND_NO_RESIDENT, GNND_LDS_TARGET, ...) are read from the environment
// only in tuning builds (tools/build_variant*.sh pass -DGNND_TUNING): the release library's
// kernel choice, and so its output bits, never depend on the caller's environment
// (tests/test_abi.py::test_release_library_reads_no_tuning_env checks the built .so).
#ifdef GNND_TUNING
#include <stdlib.h>
#define gnnd_tune_env(name) getenv(name)
#else
#define gnnd_tune_env(name) ((const char*)nullptr)
#endif

// ---------------------------------------------------------------------------------------
// debug build (make debug -> gnndecode/libgnnd_debug.so, -DGNND_DEBUG): the kernels check
// the table-derived indices they otherwise trust (LDS positions, variable ids, slots) and
// record a violation as a bit in a per-translation-unit device word (a vector atomic, no
// trap), clamping the index so the launch still completes; gnnd_debug_flags() collects and
// clears the words.  Release builds compile the checks away.
// ---------------------------------------------------------------------------------------
enum GnndDebugBit {
    GNND_DBG_LDS_POS = 0,      // message position outside the codeword's LDS run
    GNND_DBG_VAR = 1,          // variable id >= V
    GNND_DBG_SLOT = 2,         // slot / edge index out of range
    GNND_DBG_NODE = 3,         // node index outside the aggregation side
    GNND_DBG_GRID = 4,         // grid / tile bookkeeping (codeword index, p-grid index)
};
#ifdef GNND_DEBUG
static __device__ unsigned int g_gnnd_debug_word;
__device__ __forceinline__ int gnnd_dcheck_idx(int i, int n, int bit) {
    if (i < 0 || i >= n) {
        atomicOr(&g_gnnd_debug_word, 1u << bit);
        return i < 0 ? 0 : n - 1;
    }
    return i;
}
#define GNND_DIDX(i, n, bit) gnnd_dcheck_idx((i), (n), (bit))
#define GNND_DCHECK(cond, bit) \
    do { if (!(cond)) atomicOr(&g_gnnd_debug_word, 1u << (bit)); } while (0)
// per-TU host getter: returns and clears this translation unit's debug word
#define GNND_DEBUG_TU(name)                                                            \
    extern "C" unsigned gnnd_debug_take_##name(void) {                                \
        unsigned v = 0;                                                                \
        (void)hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_gnnd_debug_word), sizeof(v));       \
        const unsigned z = 0;                                                          \
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_gnnd_debug_word), &z, sizeof(z));         \
        return v;                                                                      \
    }
#else
#define GNND_DIDX(i, n, bit) (i)
#define GNND_DCHECK(cond, bit) do { } while (0)
#define GNND_DEBUG_TU(name) \
    extern "C" unsigned gnnd_debug_take_##name(void) { return 0; }
#endif

// ---------------------------------------------------------------------------------------
// phase timing (timing experiments only, -DGNND_PHASE_PROF): one wave of workgroup 0 (every wave
// with -DGNND_PPROF_ALLWAVES=1) sums the shader-clock cycles (s_memtime) spent between
// consecutive marks and prints the per-phase totals at the end of the launch.  Release builds
// compile the marks away.
// ---------------------------------------------------------------------------------------
struct PhaseProf {
#ifdef GNND_PHASE_PROF
    static constexpr int kN = 20;
    uint64_t acc[kN];
    uint64_t last;
    bool on;
    __device__ void start(bool enable) {
        on = enable;
        for (int i = 0; i < kN; ++i) acc[i] = 0;
        last = __builtin_amdgcn_s_memtime();
    }
    __device__ __forceinline__ void mark(int i) {
        if (on) {
            const uint64_t t = __builtin_amdgcn_s_memtime();
            acc[i] += t - last;
            last = t;
        }
    }
    __device__ void report(const char* tag, int n, int iters) {
        if (on && (threadIdx.x & 63) == 0)
            printf("PHASE %s w%d iters %d | %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu\n",
                   tag, (int)(threadIdx.x >> 6), iters, (unsigned long long)acc[0], (unsigned long long)acc[1],
                   (unsigned long long)acc[2], (unsigned long long)acc[3], (unsigned long long)acc[4],
                   (unsigned long long)acc[5], (unsigned long long)acc[6], (unsigned long long)acc[7],
                   (unsigned long long)acc[8], (unsigned long long)acc[9], (unsigned long long)acc[10],
                   (unsigned long long)acc[11], (unsigned long long)acc[12], (unsigned long long)acc[13],
                   (unsigned long long)acc[14], (unsigned long long)acc[15], (unsigned long long)acc[16],
                   (unsigned long long)acc[17], (unsigned long long)acc[18], (unsigned long long)acc[19]);
        (void)n;
    }
#endif
};
#ifndef GNND_PPROF_ALLWAVES
#define GNND_PPROF_ALLWAVES 0      // 1: every wave of workgroup 0 reports (the reverse pass)
#endif
#ifdef GNND_PHASE_PROF
#define GNND_PPROF(pf) PhaseProf pf
#define GNND_PSTART(pf, on) pf.start(on)
#define GNND_PMARK(pf, i) pf.mark(i)
#define GNND_PREPORT(pf, tag, n, iters) pf.report(tag, n, iters)
#define GNND_PARG(pf, i) , &pf, i
#else
#define GNND_PPROF(pf) do { } while (0)
#define GNND_PSTART(pf, on) do { } while (0)
#define GNND_PMARK(pf, i) do { } while (0)
#define GNND_PREPORT(pf, tag, n, iters) do { } while (0)
#define GNND_PARG(pf, i)
#endif

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
    // T layout of the fp32 resident kernel (x-augmented layouts, gnnd_graph::rlayx): T_v of
    // codeword b sits at LDS row b * ts + tpos(v), tpos in the high half of vlay[i].y (its low
    // half is the first message position) and in the low half of slot_ve (instead of v);
    // placed for bank-conflict-free-er gathers (gnnd_graph.hip place_t_rows).  Identity
    // elsewhere: ts = V, tpos(v) = v.
    int ts;
    // where this graph's rows sit in the caller's batch layout.  A whole graph: identity
    // (xs = N, xv0 = 0, xc0 = V, os = V, o0 = 0, es = E, e0 = 0).  A COMPONENT of a split
    // graph (gnnd_graph::comp) addresses its slice of the parent codeword's rows: variable v
    // of codeword b is x row b*xs + xv0 + v and out row b*os + o0 + v, check c is x row
    // b*xs + xc0 + c, edge e is per-edge row b*es + e0 + e (training tape, m^T).
    int xs, xv0, xc0, os, o0, es, e0;
};
#define GNND_SLOT_PAD 0x80000000u   // padding slot: variable 0, flag bit 31

struct gnnd_graph {
    GraphView view;           // slot plan of the streaming kernel (ties -> smaller R)
    GraphView rview;          // slot plan of the register-resident kernel (ties -> larger R)
    GraphView pview;          // ties -> R = 2: paired-edge fp32 V24 streaming at small batch
    GraphView rlay[7];        // rview with the padded message layout for vgroup 2^i (i = 0:
                              // identity); rlay[i].vlay == nullptr if it does not fit 16 bits
    GraphView rlayx[7];       // the same layouts with one extra position per variable after
                              // its padded messages, holding x_v (written once per decode,
                              // never by the check step): the uniform variable sum then
                              // yields T_v = S_v + x_v directly (T-layout resident models)
    void* dev;                // single device allocation holding every table
    size_t table_bytes;       // bytes of the four CSR/CSC tables (staged to LDS)
    // Disconnected Tanner graphs (the toric code's X and Z halves): ncomp >= 2 equal-shaped
    // components, each a contiguous variable range, check range and edge range, with the
    // same slot plans.  comp[k] is component k as a graph of its own (local ids, addressing
    // fields pointing into the parent rows); dcomp is a device array [3][ncomp] of the
    // components' view / rview / pview, so ONE launch can run every component of every
    // codeword as independent workgroups (no exchange: the components share no edge).
    int ncomp;                // 1: not split
    gnnd_graph* comp[8];
    GraphView* dcomp;
    int nosplit;              // gnnd_graph_set_split(g, 0): decode / train the graph whole
    int min_dc;               // smallest check degree (the fp32 BP ratio-form check step needs 2)
};
constexpr int kMaxComp = 8;

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
// ---------------------------------------------------------------------------------------
// table-driven fp64 Softplus (the fp64 decoder_v2_4 MLPs' inner loop): ~35 VALU ops
// against the 65 of softplus_ref.  Tables (tools/gen_fp64_tables.py, 60-digit decimal,
// correctly rounded) are staged into LDS by the kernel (kFp64TabDoubles doubles: exp part,
// then log part) and indexed per lane.
//   e^y, y <= 0:  y = (k/256) ln2 + r, |r| <= ln2/512;  e^y = 2^(k>>8) T[k & 255] e^r with
//                 e^r by its degree-4 Taylor polynomial (truncation < 4e-17 relative).
//   log1p(u), u in [0, 1]:  m = 1 + u with rounding error c (exact), j = rint(256 (m - 1)),
//                 r_j = RN(1 / (1 + j/256)), t = m r_j - 1 + c r_j (|t| <= 2^-8, two fmas),
//                 log1p(u) = -ln r_j + log1p(t), log1p(t) by its degree-7 series.
// ---------------------------------------------------------------------------------------
__constant__ static const double kExpTab[256] = {
    0x1.0000000000000p+0, 0x1.00b1afa5abcbfp+0, 0x1.0163da9fb3335p+0, 0x1.02168143b0281p+0,
    0x1.02c9a3e778061p+0, 0x1.037d42e11bbccp+0, 0x1.04315e86e7f85p+0, 0x1.04e5f72f654b1p+0,
    0x1.059b0d3158574p+0, 0x1.0650a0e3c1f89p+0, 0x1.0706b29ddf6dep+0, 0x1.07bd42b72a836p+0,
    0x1.0874518759bc8p+0, 0x1.092bdf66607e0p+0, 0x1.09e3ecac6f383p+0, 0x1.0a9c79b1f3919p+0,
    0x1.0b5586cf9890fp+0, 0x1.0c0f145e46c85p+0, 0x1.0cc922b7247f7p+0, 0x1.0d83b23395decp+0,
    0x1.0e3ec32d3d1a2p+0, 0x1.0efa55fdfa9c5p+0, 0x1.0fb66affed31bp+0, 0x1.1073028d7233ep+0,
    0x1.11301d0125b51p+0, 0x1.11edbab5e2ab6p+0, 0x1.12abdc06c31ccp+0, 0x1.136a814f204abp+0,
    0x1.1429aaea92de0p+0, 0x1.14e95934f312ep+0, 0x1.15a98c8a58e51p+0, 0x1.166a45471c3c2p+0,
    0x1.172b83c7d517bp+0, 0x1.17ed48695bbc0p+0, 0x1.18af9388c8deap+0, 0x1.1972658375d2fp+0,
    0x1.1a35beb6fcb75p+0, 0x1.1af99f8138a1cp+0, 0x1.1bbe084045cd4p+0, 0x1.1c82f95281c6bp+0,
    0x1.1d4873168b9aap+0, 0x1.1e0e75eb44027p+0, 0x1.1ed5022fcd91dp+0, 0x1.1f9c18438ce4dp+0,
    0x1.2063b88628cd6p+0, 0x1.212be3578a819p+0, 0x1.21f49917ddc96p+0, 0x1.22bdda27912d1p+0,
    0x1.2387a6e756238p+0, 0x1.2451ffb82140ap+0, 0x1.251ce4fb2a63fp+0, 0x1.25e85711ece75p+0,
    0x1.26b4565e27cddp+0, 0x1.2780e341ddf29p+0, 0x1.284dfe1f56381p+0, 0x1.291ba7591bb70p+0,
    0x1.29e9df51fdee1p+0, 0x1.2ab8a66d10f13p+0, 0x1.2b87fd0dad990p+0, 0x1.2c57e39771b2fp+0,
    0x1.2d285a6e4030bp+0, 0x1.2df961f641589p+0, 0x1.2ecafa93e2f56p+0, 0x1.2f9d24abd886bp+0,
    0x1.306fe0a31b715p+0, 0x1.31432edeeb2fdp+0, 0x1.32170fc4cd831p+0, 0x1.32eb83ba8ea32p+0,
    0x1.33c08b26416ffp+0, 0x1.3496266e3fa2dp+0, 0x1.356c55f929ff1p+0, 0x1.36431a2de883bp+0,
    0x1.371a7373aa9cbp+0, 0x1.37f26231e754ap+0, 0x1.38cae6d05d866p+0, 0x1.39a401b7140efp+0,
    0x1.3a7db34e59ff7p+0, 0x1.3b57fbfec6cf4p+0, 0x1.3c32dc313a8e5p+0, 0x1.3d0e544ede173p+0,
    0x1.3dea64c123422p+0, 0x1.3ec70df1c5175p+0, 0x1.3fa4504ac801cp+0, 0x1.40822c367a024p+0,
    0x1.4160a21f72e2ap+0, 0x1.423fb2709468ap+0, 0x1.431f5d950a897p+0, 0x1.43ffa3f84b9d4p+0,
    0x1.44e086061892dp+0, 0x1.45c2042a7d232p+0, 0x1.46a41ed1d0057p+0, 0x1.4786d668b3237p+0,
    0x1.486a2b5c13cd0p+0, 0x1.494e1e192aed2p+0, 0x1.4a32af0d7d3dep+0, 0x1.4b17dea6db7d7p+0,
    0x1.4bfdad5362a27p+0, 0x1.4ce41b817c114p+0, 0x1.4dcb299fddd0dp+0, 0x1.4eb2d81d8abffp+0,
    0x1.4f9b2769d2ca7p+0, 0x1.508417f4531eep+0, 0x1.516daa2cf6642p+0, 0x1.5257de83f4eefp+0,
    0x1.5342b569d4f82p+0, 0x1.542e2f4f6ad27p+0, 0x1.551a4ca5d920fp+0, 0x1.56070dde910d2p+0,
    0x1.56f4736b527dap+0, 0x1.57e27dbe2c4cfp+0, 0x1.58d12d497c7fdp+0, 0x1.59c0827ff07ccp+0,
    0x1.5ab07dd485429p+0, 0x1.5ba11fba87a03p+0, 0x1.5c9268a5946b7p+0, 0x1.5d84590998b93p+0,
    0x1.5e76f15ad2148p+0, 0x1.5f6a320dceb71p+0, 0x1.605e1b976dc09p+0, 0x1.6152ae6cdf6f4p+0,
    0x1.6247eb03a5585p+0, 0x1.633dd1d1929fdp+0, 0x1.6434634ccc320p+0, 0x1.652b9febc8fb7p+0,
    0x1.6623882552225p+0, 0x1.671c1c70833f6p+0, 0x1.68155d44ca973p+0, 0x1.690f4b19e9538p+0,
    0x1.6a09e667f3bcdp+0, 0x1.6b052fa75173ep+0, 0x1.6c012750bdabfp+0, 0x1.6cfdcddd47645p+0,
    0x1.6dfb23c651a2fp+0, 0x1.6ef9298593ae5p+0, 0x1.6ff7df9519484p+0, 0x1.70f7466f42e87p+0,
    0x1.71f75e8ec5f74p+0, 0x1.72f8286ead08ap+0, 0x1.73f9a48a58174p+0, 0x1.74fbd35d7cbfdp+0,
    0x1.75feb564267c9p+0, 0x1.77024b1ab6e09p+0, 0x1.780694fde5d3fp+0, 0x1.790b938ac1cf6p+0,
    0x1.7a11473eb0187p+0, 0x1.7b17b0976cfdbp+0, 0x1.7c1ed0130c132p+0, 0x1.7d26a62ff86f0p+0,
    0x1.7e2f336cf4e62p+0, 0x1.7f3878491c491p+0, 0x1.80427543e1a12p+0, 0x1.814d2add106d9p+0,
    0x1.82589994cce13p+0, 0x1.8364c1eb941f7p+0, 0x1.8471a4623c7adp+0, 0x1.857f4179f5b21p+0,
    0x1.868d99b4492edp+0, 0x1.879cad931a436p+0, 0x1.88ac7d98a6699p+0, 0x1.89bd0a478580fp+0,
    0x1.8ace5422aa0dbp+0, 0x1.8be05bad61778p+0, 0x1.8cf3216b5448cp+0, 0x1.8e06a5e0866d9p+0,
    0x1.8f1ae99157736p+0, 0x1.902fed0282c8ap+0, 0x1.9145b0b91ffc6p+0, 0x1.925c353aa2fe2p+0,
    0x1.93737b0cdc5e5p+0, 0x1.948b82b5f98e5p+0, 0x1.95a44cbc8520fp+0, 0x1.96bdd9a7670b3p+0,
    0x1.97d829fde4e50p+0, 0x1.98f33e47a22a2p+0, 0x1.9a0f170ca07bap+0, 0x1.9b2bb4d53fe0dp+0,
    0x1.9c49182a3f090p+0, 0x1.9d674194bb8d5p+0, 0x1.9e86319e32323p+0, 0x1.9fa5e8d07f29ep+0,
    0x1.a0c667b5de565p+0, 0x1.a1e7aed8eb8bbp+0, 0x1.a309bec4a2d33p+0, 0x1.a42c980460ad8p+0,
    0x1.a5503b23e255dp+0, 0x1.a674a8af46052p+0, 0x1.a799e1330b358p+0, 0x1.a8bfe53c12e59p+0,
    0x1.a9e6b5579fdbfp+0, 0x1.ab0e521356ebap+0, 0x1.ac36bbfd3f37ap+0, 0x1.ad5ff3a3c2774p+0,
    0x1.ae89f995ad3adp+0, 0x1.afb4ce622f2ffp+0, 0x1.b0e07298db666p+0, 0x1.b20ce6c9a8952p+0,
    0x1.b33a2b84f15fbp+0, 0x1.b468415b749b1p+0, 0x1.b59728de5593ap+0, 0x1.b6c6e29f1c52ap+0,
    0x1.b7f76f2fb5e47p+0, 0x1.b928cf22749e4p+0, 0x1.ba5b030a1064ap+0, 0x1.bb8e0b79a6f1fp+0,
    0x1.bcc1e904bc1d2p+0, 0x1.bdf69c3f3a207p+0, 0x1.bf2c25bd71e09p+0, 0x1.c06286141b33dp+0,
    0x1.c199bdd85529cp+0, 0x1.c2d1cd9fa652cp+0, 0x1.c40ab5fffd07ap+0, 0x1.c544778fafb22p+0,
    0x1.c67f12e57d14bp+0, 0x1.c7ba88988c933p+0, 0x1.c8f6d9406e7b5p+0, 0x1.ca3405751c4dbp+0,
    0x1.cb720dcef9069p+0, 0x1.ccb0f2e6d1675p+0, 0x1.cdf0b555dc3fap+0, 0x1.cf3155b5bab74p+0,
    0x1.d072d4a07897cp+0, 0x1.d1b532b08c968p+0, 0x1.d2f87080d89f2p+0, 0x1.d43c8eacaa1d6p+0,
    0x1.d5818dcfba487p+0, 0x1.d6c76e862e6d3p+0, 0x1.d80e316c98398p+0, 0x1.d955d71ff6075p+0,
    0x1.da9e603db3285p+0, 0x1.dbe7cd63a8315p+0, 0x1.dd321f301b460p+0, 0x1.de7d5641c0658p+0,
    0x1.dfc97337b9b5fp+0, 0x1.e11676b197d17p+0, 0x1.e264614f5a129p+0, 0x1.e3b333b16ee12p+0,
    0x1.e502ee78b3ff6p+0, 0x1.e653924676d76p+0, 0x1.e7a51fbc74c83p+0, 0x1.e8f7977cdb740p+0,
    0x1.ea4afa2a490dap+0, 0x1.eb9f4867cca6ep+0, 0x1.ecf482d8e67f1p+0, 0x1.ee4aaa2188510p+0,
    0x1.efa1bee615a27p+0, 0x1.f0f9c1cb6412ap+0, 0x1.f252b376bba97p+0, 0x1.f3ac948dd7274p+0,
    0x1.f50765b6e4540p+0, 0x1.f6632798844f8p+0, 0x1.f7bfdad9cbe14p+0, 0x1.f91d802243c89p+0,
    0x1.fa7c1819e90d8p+0, 0x1.fbdba3692d514p+0, 0x1.fd3c22b8f71f1p+0, 0x1.fe9d96b2a23d9p+0,
};
__constant__ static const double kLogTab[514] = {
    0x1.0000000000000p+0, 0x0.0p+0, 0x1.fe01fe01fe020p-1, 0x1.ff00aa2b10ba0p-9,
    0x1.fc07f01fc07f0p-1, 0x1.fe02a6b106799p-8, 0x1.fa11caa01fa12p-1, 0x1.7dc475f810a69p-7,
    0x1.f81f81f81f820p-1, 0x1.fc0a8b0fc03c4p-7, 0x1.f6310aca0dbb5p-1, 0x1.3cea44346a584p-6,
    0x1.f44659e4a4271p-1, 0x1.7b91b07d5b126p-6, 0x1.f25f644230ab5p-1, 0x1.b9fc027af919ap-6,
    0x1.f07c1f07c1f08p-1, 0x1.f829b0e7832f8p-6, 0x1.ee9c7f8458e02p-1, 0x1.1b0d98923d97fp-5,
    0x1.ecc07b301ecc0p-1, 0x1.39e87b9febd68p-5, 0x1.eae807aba01ebp-1, 0x1.58a5bafc8e4d3p-5,
    0x1.e9131abf0b767p-1, 0x1.77458f632dcffp-5, 0x1.e741aa59750e4p-1, 0x1.95c830ec8e3f2p-5,
    0x1.e573ac901e574p-1, 0x1.b42dd711971b9p-5, 0x1.e3a9179dc1a73p-1, 0x1.d276b8adb0b56p-5,
    0x1.e1e1e1e1e1e1ep-1, 0x1.f0a30c01162a8p-5, 0x1.e01e01e01e01ep-1, 0x1.075983598e471p-4,
    0x1.de5d6e3f8868ap-1, 0x1.16536eea37ae3p-4, 0x1.dca01dca01dcap-1, 0x1.253f62f0a1417p-4,
    0x1.dae6076b981dbp-1, 0x1.341d7961bd1d0p-4, 0x1.d92f2231e7f8ap-1, 0x1.42edcbea646eep-4,
    0x1.d77b654b82c34p-1, 0x1.51b073f06183cp-4, 0x1.d5cac807572b2p-1, 0x1.60658a93750c4p-4,
    0x1.d41d41d41d41dp-1, 0x1.6f0d28ae56b4ep-4, 0x1.d272ca3fc5b1ap-1, 0x1.7da766d7b12d0p-4,
    0x1.d0cb58f6ec074p-1, 0x1.8c345d6319b23p-4, 0x1.cf26e5c44bfc6p-1, 0x1.9ab42462033aep-4,
    0x1.cd85689039b0bp-1, 0x1.a926d3a4ad562p-4, 0x1.cbe6d9601cbe7p-1, 0x1.b78c82bb0eda0p-4,
    0x1.ca4b3055ee191p-1, 0x1.c5e548f5bc743p-4, 0x1.c8b265afb8a42p-1, 0x1.d4313d66cb35dp-4,
    0x1.c71c71c71c71cp-1, 0x1.e27076e2af2eap-4, 0x1.c5894d10d4986p-1, 0x1.f0a30c01162a4p-4,
    0x1.c3f8f01c3f8f0p-1, 0x1.fec9131dbeabcp-4, 0x1.c26b5392ea01cp-1, 0x1.0671512ca596fp-3,
    0x1.c0e070381c0e0p-1, 0x1.0d77e7cd08e5bp-3, 0x1.bf583ee868d8bp-1, 0x1.14785846742acp-3,
    0x1.bdd2b899406f7p-1, 0x1.1b72ad52f67a2p-3, 0x1.bc4fd65883e7bp-1, 0x1.2266f190a5acdp-3,
    0x1.bacf914c1bad0p-1, 0x1.29552f81ff521p-3, 0x1.b951e2b18ff23p-1, 0x1.303d718e47fd5p-3,
    0x1.b7d6c3dda338bp-1, 0x1.371fc201e8f75p-3, 0x1.b65e2e3beee05p-1, 0x1.3dfc2b0ecc62ap-3,
    0x1.b4e81b4e81b4fp-1, 0x1.44d2b6ccb7d1cp-3, 0x1.b37484ad806cep-1, 0x1.4ba36f39a55e5p-3,
    0x1.b2036406c80d9p-1, 0x1.526e5e3a1b438p-3, 0x1.b094b31d922a4p-1, 0x1.59338d9982085p-3,
    0x1.af286bca1af28p-1, 0x1.5ff3070a793d6p-3, 0x1.adbe87f94905ep-1, 0x1.66acd4272ad51p-3,
    0x1.ac5701ac5701bp-1, 0x1.6d60fe719d21bp-3, 0x1.aaf1d2f87ebfdp-1, 0x1.740f8f54037a3p-3,
    0x1.a98ef606a63bep-1, 0x1.7ab890210d907p-3, 0x1.a82e65130e159p-1, 0x1.815c0a14357e9p-3,
    0x1.a6d01a6d01a6dp-1, 0x1.87fa06520c911p-3, 0x1.a574107688a4ap-1, 0x1.8e928de886d41p-3,
    0x1.a41a41a41a41ap-1, 0x1.9525a9cf456b6p-3, 0x1.a2c2a87c51ca0p-1, 0x1.9bb362e7dfb85p-3,
    0x1.a16d3f97a4b02p-1, 0x1.a23bc1fe2b561p-3, 0x1.a01a01a01a01ap-1, 0x1.a8becfc882f19p-3,
    0x1.9ec8e951033d9p-1, 0x1.af3c94e80bff3p-3, 0x1.9d79f176b682dp-1, 0x1.b5b519e8fb5a6p-3,
    0x1.9c2d14ee4a102p-1, 0x1.bc286742d8cd4p-3, 0x1.9ae24ea5510dap-1, 0x1.c2968558c18c2p-3,
    0x1.999999999999ap-1, 0x1.c8ff7c79a9a20p-3, 0x1.9852f0d8ec0ffp-1, 0x1.cf6354e09c5ddp-3,
    0x1.970e4f80cb872p-1, 0x1.d5c216b4fbb94p-3, 0x1.95cbb0be377aep-1, 0x1.dc1bca0abec7bp-3,
    0x1.948b0fcd6e9e0p-1, 0x1.e27076e2af2e8p-3, 0x1.934c67f9b2ce6p-1, 0x1.e8c0252aa5a60p-3,
    0x1.920fb49d0e229p-1, 0x1.ef0adcbdc5935p-3, 0x1.90d4f120190d5p-1, 0x1.f550a564b7b37p-3,
    0x1.8f9c18f9c18fap-1, 0x1.fb9186d5e3e29p-3, 0x1.8e6527af1373fp-1, 0x1.00e6c45ad501dp-2,
    0x1.8d3018d3018d3p-1, 0x1.0402594b4d041p-2, 0x1.8bfce8062ff3ap-1, 0x1.071b85fcd590dp-2,
    0x1.8acb90f6bf3aap-1, 0x1.0a324e27390e2p-2, 0x1.899c0f601899cp-1, 0x1.0d46b579ab74bp-2,
    0x1.886e5f0abb04ap-1, 0x1.1058bf9ae4ad4p-2, 0x1.87427bcc092b9p-1, 0x1.136870293a8b0p-2,
    0x1.8618618618618p-1, 0x1.1675cababa60fp-2, 0x1.84f00c2780614p-1, 0x1.1980d2dd4236fp-2,
    0x1.83c977ab2beddp-1, 0x1.1c898c16999fbp-2, 0x1.82a4a0182a4a0p-1, 0x1.1f8ff9e48a2f3p-2,
    0x1.8181818181818p-1, 0x1.22941fbcf7966p-2, 0x1.8060180601806p-1, 0x1.2596010df763ap-2,
    0x1.7f405fd017f40p-1, 0x1.2895a13de86a4p-2, 0x1.7e225515a4f1dp-1, 0x1.2b9303ab89d25p-2,
    0x1.7d05f417d05f4p-1, 0x1.2e8e2bae11d31p-2, 0x1.7beb3922e017cp-1, 0x1.31871c9544185p-2,
    0x1.7ad2208e0ecc3p-1, 0x1.347dd9a987d56p-2, 0x1.79baa6bb6398bp-1, 0x1.3772662bfd85cp-2,
    0x1.78a4c8178a4c8p-1, 0x1.3a64c556945eap-2, 0x1.77908119ac60dp-1, 0x1.3d54fa5c1f710p-2,
    0x1.767dce434a9b1p-1, 0x1.404308686a7e4p-2, 0x1.756cac201756dp-1, 0x1.432ef2a04e813p-2,
    0x1.745d1745d1746p-1, 0x1.4618bc21c5ec2p-2, 0x1.734f0c541fe8dp-1, 0x1.49006804009d0p-2,
    0x1.724287f46debcp-1, 0x1.4be5f957778a1p-2, 0x1.713786d9c7c09p-1, 0x1.4ec9732600269p-2,
    0x1.702e05c0b8170p-1, 0x1.51aad872df82ep-2, 0x1.6f26016f26017p-1, 0x1.548a2c3add263p-2,
    0x1.6e1f76b4337c7p-1, 0x1.5767717455a6cp-2, 0x1.6d1a62681c861p-1, 0x1.5a42ab0f4cfe2p-2,
    0x1.6c16c16c16c17p-1, 0x1.5d1bdbf5809cap-2, 0x1.6b1490aa31a3dp-1, 0x1.5ff3070a793d4p-2,
    0x1.6a13cd1537290p-1, 0x1.62c82f2b9c796p-2, 0x1.691473a88d0c0p-1, 0x1.659b57303e1f2p-2,
    0x1.6816816816817p-1, 0x1.686c81e9b14adp-2, 0x1.6719f3601671ap-1, 0x1.6b3bb2235943dp-2,
    0x1.661ec6a5122f9p-1, 0x1.6e08eaa2ba1e4p-2, 0x1.6524f853b4aa3p-1, 0x1.70d42e2789236p-2,
    0x1.642c8590b2164p-1, 0x1.739d7f6bbd007p-2, 0x1.63356b88ac0dep-1, 0x1.7664e1239dbcfp-2,
    0x1.623fa77016240p-1, 0x1.792a55fdd47a1p-2, 0x1.614b36831ae94p-1, 0x1.7bede0a37afbfp-2,
    0x1.6058160581606p-1, 0x1.7eaf83b82afc2p-2, 0x1.5f66434292dfcp-1, 0x1.816f41da0d495p-2,
    0x1.5e75bb8d015e7p-1, 0x1.842d1da1e8b18p-2, 0x1.5d867c3ece2a5p-1, 0x1.86e919a330ba1p-2,
    0x1.5c9882b931057p-1, 0x1.89a3386c1425bp-2, 0x1.5babcc647fa91p-1, 0x1.8c5b7c858b48bp-2,
    0x1.5ac056b015ac0p-1, 0x1.8f11e873662c8p-2, 0x1.59d61f123ccaap-1, 0x1.91c67eb45a83ep-2,
    0x1.58ed2308158edp-1, 0x1.947941c2116fbp-2, 0x1.5805601580560p-1, 0x1.972a341135159p-2,
    0x1.571ed3c506b3ap-1, 0x1.99d958117e08ap-2, 0x1.56397ba7c52e2p-1, 0x1.9c86b02dc0862p-2,
    0x1.5555555555555p-1, 0x1.9f323ecbf984dp-2, 0x1.54725e6bb82fep-1, 0x1.a1dc064d5b995p-2,
    0x1.5390948f40febp-1, 0x1.a484090e5bb09p-2, 0x1.52aff56a8054bp-1, 0x1.a72a4966bd9e9p-2,
    0x1.51d07eae2f815p-1, 0x1.a9cec9a9a084ap-2, 0x1.50f22e111c4c5p-1, 0x1.ac718c258b0e5p-2,
    0x1.5015015015015p-1, 0x1.af1293247786bp-2, 0x1.4f38f62dd4c9bp-1, 0x1.b1b1e0ebdfc5ap-2,
    0x1.4e5e0a72f0539p-1, 0x1.b44f77bcc8f64p-2, 0x1.4d843bedc2c4cp-1, 0x1.b6eb59d3cf35cp-2,
    0x1.4cab88725af6ep-1, 0x1.b9858969310fdp-2, 0x1.4bd3edda68fe1p-1, 0x1.bc1e08b0dad0ap-2,
    0x1.4afd6a052bf5bp-1, 0x1.beb4d9da71b7ap-2, 0x1.4a27fad76014ap-1, 0x1.c149ff115f027p-2,
    0x1.49539e3b2d067p-1, 0x1.c3dd7a7cdad4dp-2, 0x1.4880522014880p-1, 0x1.c66f4e3ff6ff9p-2,
    0x1.47ae147ae147bp-1, 0x1.c8ff7c79a9a21p-2, 0x1.46dce34596066p-1, 0x1.cb8e0744d7acap-2,
    0x1.460cbc7f5cf9ap-1, 0x1.ce1af0b85f3ecp-2, 0x1.453d9e2c776cap-1, 0x1.d0a63ae721e64p-2,
    0x1.446f86562d9fbp-1, 0x1.d32fe7e00ebd5p-2, 0x1.43a2730abee4dp-1, 0x1.d5b7f9ae2c684p-2,
    0x1.42d6625d51f87p-1, 0x1.d83e7258a2f3ep-2, 0x1.420b5265e5951p-1, 0x1.dac353e2c5955p-2,
    0x1.4141414141414p-1, 0x1.dd46a04c1c4a1p-2, 0x1.40782d10e6566p-1, 0x1.dfc859906d5b5p-2,
    0x1.3fb013fb013fbp-1, 0x1.e24881a7c6c26p-2, 0x1.3ee8f42a5af07p-1, 0x1.e4c71a8687704p-2,
    0x1.3e22cbce4a902p-1, 0x1.e744261d68789p-2, 0x1.3d5d991aa75c6p-1, 0x1.e9bfa659861f5p-2,
    0x1.3c995a47babe7p-1, 0x1.ec399d2468cc1p-2, 0x1.3bd60d9232955p-1, 0x1.eeb20c640ddf3p-2,
    0x1.3b13b13b13b14p-1, 0x1.f128f5faf06ecp-2, 0x1.3a524387ac822p-1, 0x1.f39e5bc811e5dp-2,
    0x1.3991c2c187f63p-1, 0x1.f6123fa7028adp-2, 0x1.38d22d366088ep-1, 0x1.f884a36fe9ec1p-2,
    0x1.3813813813814p-1, 0x1.faf588f78f31dp-2, 0x1.3755bd1c945eep-1, 0x1.fd64f20f61571p-2,
    0x1.3698df3de0748p-1, 0x1.ffd2e0857f497p-2, 0x1.35dce5f9f2af8p-1, 0x1.011fab125ff8ap-1,
    0x1.3521cfb2b78c1p-1, 0x1.02552a5a5d0ffp-1, 0x1.34679ace01346p-1, 0x1.0389eefce633cp-1,
    0x1.33ae45b57bcb2p-1, 0x1.04bdf9da926d2p-1, 0x1.32f5ced6a1dfap-1, 0x1.05f14bd26459cp-1,
    0x1.323e34a2b10bfp-1, 0x1.0723e5c1cdf41p-1, 0x1.3187758e9ebb6p-1, 0x1.0855c884b450ep-1,
    0x1.30d190130d190p-1, 0x1.0986f4f573521p-1, 0x1.301c82ac40260p-1, 0x1.0ab76bece14d2p-1,
    0x1.2f684bda12f68p-1, 0x1.0be72e4252a83p-1, 0x1.2eb4ea1fed14bp-1, 0x1.0d163ccb9d6b8p-1,
    0x1.2e025c04b8097p-1, 0x1.0e44985d1cc8cp-1, 0x1.2d50a012d50a0p-1, 0x1.0f7241c9b497dp-1,
    0x1.2c9fb4d812ca0p-1, 0x1.109f39e2d4c96p-1, 0x1.2bef98e5a3711p-1, 0x1.11cb81787ccf8p-1,
    0x1.2b404ad012b40p-1, 0x1.12f719593efbdp-1, 0x1.2a91c92f3c105p-1, 0x1.1422025243d45p-1,
    0x1.29e4129e4129ep-1, 0x1.154c3d2f4d5eap-1, 0x1.293725bb804a5p-1, 0x1.1675cababa60ep-1,
    0x1.288b01288b013p-1, 0x1.179eabbd899a0p-1, 0x1.27dfa38a1ce4dp-1, 0x1.18c6e0ff5cf07p-1,
    0x1.27350b8812735p-1, 0x1.19ee6b467c96fp-1, 0x1.268b37cd60127p-1, 0x1.1b154b57da29ep-1,
    0x1.25e22708092f1p-1, 0x1.1c3b81f713c25p-1, 0x1.2539d7e9177b2p-1, 0x1.1d610fe677003p-1,
    0x1.2492492492492p-1, 0x1.1e85f5e7040d1p-1, 0x1.23eb79717605bp-1, 0x1.1faa34b87094cp-1,
    0x1.23456789abcdfp-1, 0x1.20cdcd192ab6ep-1, 0x1.22a0122a0122ap-1, 0x1.21f0bfc65beecp-1,
    0x1.21fb78121fb78p-1, 0x1.23130d7bebf43p-1, 0x1.21579804855e6p-1, 0x1.2434b6f483934p-1,
    0x1.20b470c67c0d9p-1, 0x1.2555bce98f7cap-1, 0x1.2012012012012p-1, 0x1.26762013430e0p-1,
    0x1.1f7047dc11f70p-1, 0x1.2795e1289b11bp-1, 0x1.1ecf43c7fb84cp-1, 0x1.28b500df60783p-1,
    0x1.1e2ef3b3fb874p-1, 0x1.29d37fec2b08bp-1, 0x1.1d8f5672e4abdp-1, 0x1.2af15f02640acp-1,
    0x1.1cf06ada2811dp-1, 0x1.2c0e9ed448e8cp-1, 0x1.1c522fc1ce059p-1, 0x1.2d2b4012edc9dp-1,
    0x1.1bb4a4046ed29p-1, 0x1.2e47436e40268p-1, 0x1.1b17c67f2bae3p-1, 0x1.2f62a99509546p-1,
    0x1.1a7b9611a7b96p-1, 0x1.307d7334f10bep-1, 0x1.19e0119e0119ep-1, 0x1.3197a0fa7fe6ap-1,
    0x1.19453808ca29cp-1, 0x1.32b1339121d71p-1, 0x1.18ab083902bdbp-1, 0x1.33ca2ba328994p-1,
    0x1.1811811811812p-1, 0x1.34e289d9ce1d2p-1, 0x1.1778a191bd684p-1, 0x1.35fa4edd36ea0p-1,
    0x1.16e0689427379p-1, 0x1.37117b54747b6p-1, 0x1.1648d50fc3201p-1, 0x1.38280fe58797fp-1,
    0x1.15b1e5f75270dp-1, 0x1.393e0d3562a1ap-1, 0x1.151b9a3fdd5c9p-1, 0x1.3a5373e7ebdf9p-1,
    0x1.1485f0e0acd3bp-1, 0x1.3b68449fffc23p-1, 0x1.13f0e8d344724p-1, 0x1.3c7c7fff73206p-1,
    0x1.135c81135c811p-1, 0x1.3d9026a7156fbp-1, 0x1.12c8b89edc0acp-1, 0x1.3ea33936b2f5bp-1,
    0x1.12358e75d3033p-1, 0x1.3fb5b84d16f43p-1, 0x1.11a3019a74826p-1, 0x1.40c7a4880dceap-1,
    0x1.1111111111111p-1, 0x1.41d8fe84672afp-1, 0x1.107fbbe011080p-1, 0x1.42e9c6ddf80bfp-1,
    0x1.0fef010fef011p-1, 0x1.43f9fe2f9ce67p-1, 0x1.0f5edfab325a2p-1, 0x1.4509a5133bb0ap-1,
    0x1.0ecf56be69c90p-1, 0x1.4618bc21c5ec2p-1, 0x1.0e40655826011p-1, 0x1.472743f33aaadp-1,
    0x1.0db20a88f4696p-1, 0x1.48353d1ea88dfp-1, 0x1.0d24456359e3ap-1, 0x1.4942a83a2fc07p-1,
    0x1.0c9714fbcda3bp-1, 0x1.4a4f85db03ebbp-1, 0x1.0c0a7868b4171p-1, 0x1.4b5bd6956e273p-1,
    0x1.0b7e6ec259dc8p-1, 0x1.4c679afccee39p-1, 0x1.0af2f722eecb5p-1, 0x1.4d72d3a39fd01p-1,
    0x1.0a6810a6810a7p-1, 0x1.4e7d811b75bb0p-1, 0x1.09ddba6af8360p-1, 0x1.4f87a3f5026e9p-1,
    0x1.0953f39010954p-1, 0x1.50913cc01686bp-1, 0x1.08cabb37565e2p-1, 0x1.519a4c0ba3446p-1,
    0x1.0842108421084p-1, 0x1.52a2d265bc5abp-1, 0x1.07b9f29b8eae2p-1, 0x1.53aad05b99b7cp-1,
    0x1.073260a47f7c6p-1, 0x1.54b2467999498p-1, 0x1.06ab59c7912fbp-1, 0x1.55b9354b40bcep-1,
    0x1.0624dd2f1a9fcp-1, 0x1.56bf9d5b3f399p-1, 0x1.059eea0727586p-1, 0x1.57c57f336f191p-1,
    0x1.05197f7d73404p-1, 0x1.58cadb5cd7989p-1, 0x1.04949cc1664c5p-1, 0x1.59cfb25fae87fp-1,
    0x1.0410410410410p-1, 0x1.5ad404c359f2dp-1, 0x1.038c6b78247fcp-1, 0x1.5bd7d30e71c73p-1,
    0x1.03091b51f5e1ap-1, 0x1.5cdb1dc6c1765p-1, 0x1.02864fc7729e9p-1, 0x1.5ddde57149923p-1,
    0x1.0204081020408p-1, 0x1.5ee02a9241676p-1, 0x1.0182436517a37p-1, 0x1.5fe1edad18919p-1,
    0x1.0101010101010p-1, 0x1.60e32f44788d9p-1, 0x1.0080402010080p-1, 0x1.61e3efda46467p-1,
    0x1.0000000000000p-1, 0x1.62e42fefa39efp-1,
};
// Softplus table (tools/gen_fp64_tables.py): {ln(1 + e^-a_j), 1 / (1 + e^a_j)} at a_j = j / 64,
// j = 0..2048, then a zero entry (softplus_sp, the fp64 reverse pass's sp_and_grad_n)
__constant__ static const double kSpTab[4100] = {
    0x1.62e42fefa39efp-1, 0x1.0000000000000p-1, 0x1.5ee82fecf8f72p-1, 0x1.fc0005554cccep-2,
    0x1.5af42fc4f9aa5p-1, 0x1.f8002aa999a08p-2, 0x1.57082f17abb83p-1, 0x1.f4008ff7e6dc6p-2,
    0x1.53242d452673bp-1, 0x1.f001553336a71p-2, 0x1.4f48296da67c2p-1, 0x1.ec029a429075bp-2,
    0x1.4b742271a9acep-1, 0x1.e8047efd07c30p-2, 0x1.47a816f212fadp-1, 0x1.e4072325c7010p-2,
    0x1.43e4055056374p-1, 0x1.e00aa6681fcf3p-2, 0x1.4027ebaeabac4p-1, 0x1.dc0f2853a17f9p-2,
    0x1.3c73c7f04b84dp-1, 0x1.d814c85836ef0p-2, 0x1.38c797b9b0f0bp-1, 0x1.d41ba5c24cb36p-2,
    0x1.35235870e4f37p-1, 0x1.d023dfb7009eep-2, 0x1.3187073dd0c9dp-1, 0x1.cc2d95305b924p-2,
    0x1.2df2a10a97d08p-1, 0x1.c838e4f996948p-2, 0x1.2a662283f8d49p-1, 0x1.c445edab6c1fbp-2,
    0x1.26e18819b6b47p-1, 0x1.c054cda8768f9p-2, 0x1.2364cdff08364p-1, 0x1.bc65a3199c96ep-2,
    0x1.1feff02b0ef62p-1, 0x1.b8788bea8c9a4p-2, 0x1.1c82ea59554e7p-1, 0x1.b48da5c647ca7p-2,
    0x1.191db80a53199p-1, 0x1.b0a50e13bdcf7p-2, 0x1.15c05483f92a8p-1, 0x1.acbee1f279ce4p-2,
    0x1.126abad2435a6p-1, 0x1.a8db3e37618e4p-2, 0x1.0f1ce5c7d103cp-1, 0x1.a4fa3f6987782p-2,
    0x1.0bd6cffe83c7ap-1, 0x1.a11c01bf10222p-2, 0x1.089873d82472ap-1, 0x1.9d40a11a2c151p-2,
    0x1.0561cb7f0dd9cp-1, 0x1.99683906266bep-2, 0x1.0232d0e6dd851p-1, 0x1.9592e4b488e87p-2,
    0x1.fe16fb9a53f7ep-2, 0x1.91c0befa560dbp-2, 0x1.f7d797747d0d4p-2, 0x1.8df1e24d59c7bp-2,
    0x1.f1a76803b86f6p-2, 0x1.8a2668c1911f6p-2, 0x1.eb865f88001cdp-2, 0x1.865e6c06a970cp-2,
    0x1.e5746fdb5c064p-2, 0x1.829a0565978dfp-2, 0x1.df718a738199ep-2, 0x1.7ed94dbe4732ap-2,
    0x1.d97da0637c5fbp-2, 0x1.7b1c5d856320ep-2, 0x1.d398a25d5f43cp-2, 0x1.77634cc23635ep-2,
    0x1.cdc280b3fe295p-2, 0x1.73ae330ca5bddp-2, 0x1.c7fb2b5caf625p-2, 0x1.6ffd278b45420p-2,
    0x1.c24291f114a3dp-2, 0x1.6c5040f18404ep-2, 0x1.bc98a3b0eb113p-2, 0x1.68a7957df4552p-2,
    0x1.b6fd4f83e1f61p-2, 0x1.65033af8acd79p-2, 0x1.b17083fb77c6dp-2, 0x1.616346b1c3df2p-2,
    0x1.abf22f54dcffep-2, 0x1.5dc7cd7fe4dfcp-2, 0x1.a6823f7adc7aap-2, 0x1.5a30e3bf0001cp-2,
    0x1.a120a207c8d00p-2, 0x1.569e9d4f13cfcp-2, 0x1.9bcd44476e5ffp-2, 0x1.53110d9310f36p-2,
    0x1.9688133909968p-2, 0x1.4f88476fd7eabp-2, 0x1.9150fb914105bp-2, 0x1.4c045d4b50976p-2,
    0x1.8c27e9bc22ee1p-2, 0x1.4885610b9b828p-2, 0x1.870cc9df25cf0p-2, 0x1.450b64165ca64p-2,
    0x1.81ff87db2b992p-2, 0x1.419677501f875p-2, 0x1.7d000f4e871e0p-2, 0x1.3e26ab1bd460dp-2,
    0x1.780e4b970359dp-2, 0x1.3abc0f5a661e4p-2, 0x1.732a27d3ec337p-2, 0x1.3756b36a68d72p-2,
    0x1.6e538ee81852cp-2, 0x1.33f6a627e07adp-2, 0x1.698a6b7bf3abcp-2, 0x1.309bf5ec1f531p-2,
    0x1.64cea7ff8a616p-2, 0x1.2d46b08dbbfe4p-2, 0x1.60202eac93a15p-2, 0x1.29f6e3609e7d9p-2,
    0x1.5b7ee9887c1ecp-2, 0x1.26ac9b3623eb1p-2, 0x1.56eac2666fd14p-2, 0x1.2367e45d5869ap-2,
    0x1.5263a2e962a0bp-2, 0x1.2028caa346d91p-2, 0x1.4de9748617a71p-2, 0x1.1cef59535dd5cp-2,
    0x1.497c208526b4bp-2, 0x1.19bb9b37e985dp-2, 0x1.451b9004ffc50p-2, 0x1.168d9a9aa1b29p-2,
    0x1.40c7abfbec124p-2, 0x1.136561454ba86p-2, 0x1.3c805d3a0c7bep-2, 0x1.1042f8826f54bp-2,
    0x1.38458c6b54f25p-2, 0x1.0d26691e1f159p-2, 0x1.34172219849f5p-2, 0x1.0a0fbb66d1acep-2,
    0x1.2ff506ae1a836p-2, 0x1.06fef72e4dc51p-2, 0x1.2bdf227446422p-2, 0x1.03f423caa6741p-2,
    0x1.27d55d9ad4dccp-2, 0x1.00ef481748277p-2, 0x1.23d7a0361917fp-2, 0x1.fbe0d4ec2ac4cp-3,
    0x1.1fe5d241cf50ap-2, 0x1.f5ef21a125693p-3, 0x1.1bffdba2fc839p-2, 0x1.f009813242a2cp-3,
    0x1.1825a429c84e0p-2, 0x1.ea2ffd988f57ep-3, 0x1.1457139351b0fp-2, 0x1.e4629fe40efc7p-3,
    0x1.1094118b7e62ap-2, 0x1.dea1703e813dfp-3, 0x1.0cdc85aec47c0p-2, 0x1.d8ec75ee4017ep-3,
    0x1.0930578bee529p-2, 0x1.d343b75935199p-3, 0x1.058f6ea5d8518p-2, 0x1.cda73a07e4a8ep-3,
    0x1.01f9b27528a73p-2, 0x1.c81702a88e0d5p-3, 0x1.fcde14d4013e9p-3, 0x1.c29315125f120p-3,
    0x1.f5debbdb4f04bp-3, 0x1.bd1b7448ba0cfp-3, 0x1.eef528c85db0fp-3, 0x1.b7b0227e8d1ffp-3,
    0x1.e8212a5c1fd99p-3, 0x1.b2512119b9872p-3, 0x1.e1628f5384e72p-3, 0x1.acfe70b689cebp-3,
    0x1.dab9266a986bbp-3, 0x1.a7b8112b35cb7p-3, 0x1.d424be5f93503p-3, 0x1.a27e018b73371p-3,
    0x1.cda525f5dea88p-3, 0x1.9d50402c11d4ap-3, 0x1.c73a2bf908019p-3, 0x1.982ecaa6a205cp-3,
    0x1.c0e39f3fa7016p-3, 0x1.93199ddd24bfep-3, 0x1.baa14eae34378p-3, 0x1.8e10b5fdc3d2cp-3,
    0x1.b4730939d0fc1p-3, 0x1.89140e86917a5p-3, 0x1.ae589deb0044cp-3, 0x1.8423a2494e38dp-3,
    0x1.a851dbe05056dp-3, 0x1.7f3f6b6f33fcep-3, 0x1.a25e9250f543cp-3, 0x1.7a67637cc59d8p-3,
    0x1.9c7e908f5420fp-3, 0x1.759b8355a1bb0p-3, 0x1.96b1a60b7eee5p-3, 0x1.70dbc340581b1p-3,
    0x1.90f7a255a1246p-3, 0x1.6c281aea409c0p-3, 0x1.8b5055205ce49p-3, 0x1.6780816b52e19p-3,
    0x1.85bb8e4318cadp-3, 0x1.62e4ed49fde48p-3, 0x1.80391dbc3e62ap-3, 0x1.5e55547efe94dp-3,
    0x1.7ac8d3b369447p-3, 0x1.59d1ac7934c4fp-3, 0x1.756a807b86e48p-3, 0x1.5559ea21759b3p-3,
    0x1.701df494e71dep-3, 0x1.50ee01de5accfp-3, 0x1.6ae300af3d87fp-3, 0x1.4c8de7980def4p-3,
    0x1.65b975ab93a81p-3, 0x1.48398ebc0f2d8p-3, 0x1.60a1249e2c126p-3, 0x1.43f0ea40f6bf3p-3,
    0x1.5b99ded056905p-3, 0x1.3fb3ecaa307bcp-3, 0x1.56a375c23565ep-3, 0x1.3b82880bb0f25p-3,
    0x1.51bdbb2c73cffp-3, 0x1.375cae0da3729p-3, 0x1.4ce88101edd9fp-3, 0x1.33424ff01079ap-3,
    0x1.4823997149a9fp-3, 0x1.2f335e8e7bfd6p-3, 0x1.436ed6e682642p-3, 0x1.2b2fca637b16fp-3,
    0x1.3eca0c0c64ca4p-3, 0x1.2737838c40937p-3, 0x1.3a350bcdfdbb6p-3, 0x1.234a79cc1ff85p-3,
    0x1.35afa957fabbap-3, 0x1.1f689c90068fdp-3, 0x1.3139b819fcac4p-3, 0x1.1b91daf1ea17dp-3,
    0x1.2cd30bc7dcde3p-3, 0x1.17c623bc2cb27p-3, 0x1.287b785ae4ab1p-3, 0x1.1405656cf5c08p-3,
    0x1.2432d212f7c19p-3, 0x1.104f8e397f508p-3, 0x1.1ff8ed77b1533p-3, 0x1.0ca48c1157d5dp-3,
    0x1.1bcd9f5974536p-3, 0x1.09044ca197df0p-3, 0x1.17b0bcd26ef80p-3, 0x1.056ebd580b890p-3,
    0x1.13a21b4791acep-3, 0x1.01e3cb664f724p-3, 0x1.0fa1906979ad6p-3, 0x1.fcc6c789c1ebfp-4,
    0x1.0baef2354f760p-3, 0x1.f5dae66c42f9dp-4, 0x1.07ca16f59943cp-3, 0x1.ef03cc92996bap-4,
    0x1.03f2d54301d49p-3, 0x1.e84152bac31afp-4, 0x1.00290405139e9p-3, 0x1.e1935147fb83cp-4,
    0x1.f8d8f4e5d1686p-4, 0x1.daf9a04857e3cp-4, 0x1.f17a20279f16dp-4, 0x1.d474177a481b8p-4,
    0x1.ea35397fc9bc9p-4, 0x1.ce028e51fc259p-4, 0x1.e309f14145b86p-4, 0x1.c7a4dbfeadff4p-4,
    0x1.dbf7f862cbc61p-4, 0x1.c15ad76fcfe50p-4, 0x1.d4ff007fcdef3p-4, 0x1.bb24575a1ecfap-4,
    0x1.ce1ebbd958699p-4, 0x1.b501323c9923ap-4, 0x1.c756dd56ded28p-4, 0x1.aef13e65598dap-4,
    0x1.c0a71886f6366p-4, 0x1.a8f451f6560c5p-4, 0x1.ba0f219ffc538p-4, 0x1.a30a42ea032fap-4,
    0x1.b38ead80ac87bp-4, 0x1.9d32e717db9b7p-4, 0x1.ad2571b0a2d71p-4, 0x1.976e1438cbe0fp-4,
    0x1.a6d32460cd7a9p-4, 0x1.91bb9feb82ca2p-4, 0x1.a0977c6bcd643p-4, 0x1.8c1b5fb8a6354p-4,
    0x1.9a72315646266p-4, 0x1.868d2916eca5bp-4, 0x1.9462fb4f1dabfp-4, 0x1.8110d16f1bb44p-4,
    0x1.8e69932fac2b3p-4, 0x1.7ba62e1feb8cfp-4, 0x1.8885b27bdcc1dp-4, 0x1.764d1481cfad3p-4,
    0x1.82b713623f222p-4, 0x1.710559eaa51aap-4, 0x1.7cfd70bc0abc4p-4, 0x1.6bced3b1464cap-4,
    0x1.7758860d13cc6p-4, 0x1.66a957310508ep-4, 0x1.71c80f83b2b46p-4, 0x1.6194b9cd0a749p-4,
    0x1.6c4bc9f89e092p-4, 0x1.5c90d0f39da16p-4, 0x1.66e372eeb7b7bp-4, 0x1.579d722150debp-4,
    0x1.618ec892cda74p-4, 0x1.52ba72e4161b3p-4, 0x1.5c4d89bb4e3b1p-4, 0x1.4de7a8de3aa5fp-4,
    0x1.571f75e7f115ep-4, 0x1.4924e9c94aa01p-4, 0x1.52044d4154801p-4, 0x1.44720b78dc725p-4,
    0x1.4cfbd0988fcecp-4, 0x1.3fcee3dd449d2p-4, 0x1.4805c166bb2adp-4, 0x1.3b3b490632395p-4,
    0x1.4321e1cc6d13fp-4, 0x1.36b7112534847p-4, 0x1.3e4ff4912dfa9p-4, 0x1.3242129029d2dp-4,
    0x1.398fbd22e24adp-4, 0x1.2ddc23c398437p-4, 0x1.34e0ff952b406p-4, 0x1.29851b64f0945p-4,
    0x1.304380a0beda5p-4, 0x1.253cd044bb756p-4, 0x1.2bb705a2b7440p-4, 0x1.21031960b1b94p-4,
    0x1.273b549bda06bp-4, 0x1.1cd7cde5bfc5ap-4, 0x1.22d0342fd7566p-4, 0x1.18bac531f4a33p-4,
    0x1.1e756ba481cabp-4, 0x1.14abd6d65d0fap-4, 0x1.1a2ac2e0fed28p-4, 0x1.10aada98caf38p-4,
    0x1.15f0026cf0307p-4, 0x1.0cb7a875899e7p-4, 0x1.11c4f36f96cc8p-4, 0x1.08d218a0ff2ccp-4,
    0x1.0da95faeef248p-4, 0x1.04fa03893b786p-4, 0x1.099d118ec7a5bp-4, 0x1.012f41d774f8dp-4,
    0x1.059fd40fd1361p-4, 0x1.fae358e2e7e6fp-5, 0x1.01b172ceaa336p-4, 0x1.f38238f5d8c04p-5,
    0x1.fba37405c85acp-5, 0x1.ec3ad6ad8dc42p-5, 0x1.f400ecfc09386p-5, 0x1.e50ce550b271ep-5,
    0x1.ec7aeb5501accp-5, 0x1.ddf818a91d125p-5, 0x1.e5110b156b0a2p-5, 0x1.d6fc2505ffbb4p-5,
    0x1.ddc2e96fb3aa0p-5, 0x1.d018bf3dfa83ap-5, 0x1.d69024c1dd431p-5, 0x1.c94d9cb10fa85p-5,
    0x1.cf785c9353a93p-5, 0x1.c29a734a7a5dap-5, 0x1.c87b3192bc6bcp-5, 0x1.bbfef98269099p-5,
    0x1.c1984593bfc32p-5, 0x1.b57ae65f9ba04p-5, 0x1.bacf3b8ccb3acp-5, 0x1.af0df178e6da8p-5,
    0x1.b41fb794ce842p-5, 0x1.a8b7d2f69cfbep-5, 0x1.ad895ee0f2da0p-5, 0x1.a2784393dcdd5p-5,
    0x1.a70bd7c24d59dp-5, 0x1.9c4efc9fc7ec7p-5, 0x1.a0a6c9a38cb60p-5, 0x1.963bb7fe9fd0ap-5,
    0x1.9a59dd06a2a18p-5, 0x1.903e302acc623p-5, 0x1.9424bb8269517p-5, 0x1.8a562035ca9edp-5,
    0x1.8e070fc045701p-5, 0x1.848343c905445p-5, 0x1.88008579c4d8bp-5, 0x1.7ec5572697b74p-5,
    0x1.8210c9763a72ap-5, 0x1.791c1729fbd98p-5, 0x1.7c378988577ddp-5, 0x1.73874148a3719p-5,
    0x1.7674748bc2a11p-5, 0x1.6e0693927dc1ep-5, 0x1.70c73a62ad09dp-5, 0x1.6899ccb269eb4p-5,
    0x1.6b2f8bf365e63p-5, 0x1.6340abee96b4ep-5, 0x1.65ad1b25ec85bp-5, 0x1.5dfaf128d04f4p-5,
    0x1.603f9ae18164ap-5, 0x1.58c85cdebca7bp-5, 0x1.5ae6bf0a36692p-5, 0x1.53a8b02a06dc9p-5,
    0x1.55a23c7e7e925p-5, 0x1.4e9bacc07a61cp-5, 0x1.5071c914bd5b8p-5, 0x1.49a114f40e610p-5,
    0x1.4b551b98d60fep-5, 0x1.44b8abb2e1df4p-5, 0x1.464bebc9bb4b5p-5, 0x1.3fe23487292e7p-5,
    0x1.4155f256fee1fp-5, 0x1.3b1d73970d2e6p-5, 0x1.3c72e8de6266bp-5, 0x1.366a2da47cdf7p-5,
    0x1.37a289e968854p-5, 0x1.31c8280cf1c3dp-5, 0x1.32e490eae764ep-5, 0x1.2d3728c9278d2p-5,
    0x1.2e38ba3c9c447p-5, 0x1.28b6f66cc78d9p-5, 0x1.299ec31cc0811p-5, 0x1.244758260864fp-5,
    0x1.251669aba0344p-5, 0x1.1fe815bd425bcp-5, 0x1.209f6ce93296dp-5, 0x1.1b98f79478df1p-5,
    0x1.1c398cb2b452fp-5, 0x1.1759c6a6d98aep-5, 0x1.17e489c043eddp-5, 0x1.132a4c88312eep-5,
    0x1.13a025a280713p-5, 0x1.0f0a536457387p-5, 0x1.0f6c22c02a796p-5, 0x1.0af9a5fe8fe6ap-5,
    0x1.0b484453c7cc4p-5, 0x1.06f80fb0e5af4p-5, 0x1.07344e69499bep-5, 0x1.03055c6b7a348p-5,
    0x1.033005dbb5952p-5, 0x1.fe42b1679e58ap-6, 0x1.fe7660a5a3b5bp-6, 0x1.f697a3480f2c8p-6,
    0x1.f6ab2881a8146p-6, 0x1.ef0929d44333bp-6, 0x1.eefdf1c026cc3p-6, 0x1.e796e18e52cdbp-6,
    0x1.e76e4c617c898p-6, 0x1.e040681ccad94p-6, 0x1.dffbc9ed25b0ep-6, 0x1.d9055c48f879ep-6,
    0x1.d8a5fd6d36db3p-6, 0x1.d1e55dfd28d63p-6, 0x1.d16c7b69dc68cp-6, 0x1.cae00e42dd6e9p-6,
    0x1.ca4ed9e4e159cp-6, 0x1.c3f50f40f5a58p-6, 0x1.c34cb0553d946p-6, 0x1.bd240439ce0f9p-6,
    0x1.bc6597a2abc1fp-6, 0x1.b66c9189561d6p-6, 0x1.b5992a2146e72p-6, 0x1.afce5ca31cab7p-6,
    0x1.aee7038d2fdb9p-6, 0x1.a9490c1054030p-6, 0x1.a84ec1063ac1dp-6, 0x1.a2dc476dcdcfdp-6,
    0x1.a1d0010ba49e5p-6, 0x1.9c87b769ef8cfp-6, 0x1.9b6a6377d12b3p-6, 0x1.964b05c29fe5bp-6,
    0x1.951d897c1103ep-6, 0x1.9025dd432d853p-6, 0x1.8ee9159c70419p-6, 0x1.8a17e9c22fc90p-6,
    0x1.88ccabab8da0bp-6, 0x1.8420d81f61cafp-6, 0x1.82c7f0c67a44ap-6, 0x1.7e405641782fbp-6,
    0x1.7cda8b50a22e0p-6, 0x1.78761313f225ap-6, 0x1.770422efbd75fp-6, 0x1.72c1be84e5fc0p-6,
    0x1.71446087ca5f3p-6, 0x1.6d230982c9b6bp-6, 0x1.6b9aee37104c4p-6, 0x1.6799a5fa37ffdp-6,
    0x1.660777522ba84p-6, 0x1.622546d3b1d50p-6, 0x1.6089a86022cf6p-6, 0x1.5cc59ff15d4b5p-6,
    0x1.5b212f1684015p-6, 0x1.577a662cc1c17p-6, 0x1.55cdba558c675p-6, 0x1.52434f5481d51p-6,
    0x1.508efa245836cp-6, 0x1.4d20122a136cep-6, 0x1.4b649fad1bf67p-6, 0x1.4810665f7626ap-6,
    0x1.464e5d3966ed6p-6, 0x1.43140494e874bp-6, 0x1.414be62e6ebeap-6, 0x1.3e2aa6569bb5dp-6,
    0x1.3c5cef0964372p-6, 0x1.3954061a678bcp-6, 0x1.37812d5bd14e8p-6, 0x1.348fdf3d7cb75p-6,
    0x1.32b857c8005d7p-6, 0x1.2fddee0217b95p-6, 0x1.2e0225fd6c896p-6, 0x1.2b3def8d33791p-6,
    0x1.295e50b53b654p-6, 0x1.26afa1e43c2c3p-6, 0x1.24cc91aebfc59p-6, 0x1.2232c3eac2badp-6,
    0x1.204ca3ac05c5fp-6, 0x1.1dc7156030d7cp-6, 0x1.1bde426e67fc0p-6, 0x1.196c56dd7e027p-6,
    0x1.17812ab32dd48p-6, 0x1.152249d2e5a71p-6, 0x1.13351a3033151p-6, 0x1.10e8b0859e8dcp-6,
    0x1.0ef9cf90987dcp-6, 0x1.0cbf4e0d93c85p-6, 0x1.0acf0a717d82ep-6, 0x1.08a5e6531f4ccp-6,
    0x1.06b48b5ec3195p-6, 0x1.049c3e0cc6678p-6, 0x1.02aa13cfd78d3p-6, 0x1.00a21abcf82f4p-6,
    0x1.fd5ecc4916b3fp-7, 0x1.f96e855f9c447p-7, 0x1.f5888b43ddf7ap-7, 0x1.f1b6f9f19e265p-7,
    0x1.edd0ecde7360ep-7, 0x1.ea1d22e169144p-7, 0x1.e6377b25723a5p-7, 0x1.e2a091666577bp-7,
    0x1.debbc1dd939f9p-7, 0x1.db40d83986716p-7, 0x1.d75d4e7db11e5p-7, 0x1.d3fd8b90e4e51p-7,
    0x1.d01bb028d8df0p-7, 0x1.ccd6411b606f9p-7, 0x1.c8f677a8733e5p-7, 0x1.c5ca8ffc467efp-7,
    0x1.c1ed376679bccp-7, 0x1.beda10c6ffc37p-7, 0x1.baff8367bf2c1p-7, 0x1.b8045d7ac42c2p-7,
    0x1.b42cf14648ff1p-7, 0x1.b149117e559fap-7, 0x1.ad75182bb9a0dp-7, 0x1.aaa7c99bc19e3p-7,
    0x1.a6d790cbcbb72p-7, 0x1.a42023fc29f8fp-7, 0x1.a053f55ede33fp-7, 0x1.9db1c02394c71p-7,
    0x1.99e9e19c9117ep-7, 0x1.975c3eecc3be2p-7, 0x1.9398f2b672c8bp-7, 0x1.911f428513132p-7,
    0x1.8d60c752bddcbp-7, 0x1.8afa6e686004ap-7, 0x1.8740ff87273c9p-7, 0x1.84ed675cf72e2p-7,
    0x1.81393cd3bc7c1p-7, 0x1.7ef7d36f8ac27p-7, 0x1.7b49221dd24a1p-7, 0x1.791959ef30c76p-7,
    0x1.757053ab02d6fp-7, 0x1.7351a369696e0p-7, 0x1.6fae771c3c120p-7, 0x1.6da059a62d9cdp-7,
    0x1.6a033368dd9b7p-7, 0x1.680527a405c3bp-7, 0x1.646e30d9e64aap-7, 0x1.627fb994290bep-7,
    0x1.5eef190531271p-7, 0x1.5d0fbcd6a4f76p-7, 0x1.598596c8c1b15p-7, 0x1.57b4dff68d7fep-7,
    0x1.543156461f5abp-7, 0x1.526ed2a635c41p-7, 0x1.4ef204ddc0092p-7, 0x1.4d3d45bb71517p-7,
    0x1.49c7512a81846p-7, 0x1.481feb2bde157p-7, 0x1.44b0eafd31aa0p-7, 0x1.4316760937025p-7,
    0x1.3fae83582545bp-7, 0x1.3e209a7daf6ebp-7, 0x1.3abfcc6add6a1p-7, 0x1.393e0dc857397p-7,
    0x1.35e4798dbb280p-7, 0x1.346e863987b82p-7, 0x1.311c3f3dc17fep-7, 0x1.2fb1bb2f59743p-7,
    0x1.2c66d318656abp-7, 0x1.2b07651222bd4p-7, 0x1.27c3ebd76bd73p-7, 0x1.266f3d50ff112p-7,
    0x1.2333414cd5776p-7, 0x1.21e8fe5e5f5dfp-7, 0x1.1eb48c5ed83bep-7, 0x1.1d7463aca31d4p-7,
    0x1.1a478703e6584p-7, 0x1.191129aaba495p-7, 0x1.15ebec3ec2aecp-7, 0x1.14bf0dc0d02b6p-7,
    0x1.11a1781aa27eap-7, 0x1.107dce4cff00ap-7, 0x1.0d67e7a75c323p-7, 0x1.0c4d2aa00c72dp-7,
    0x1.093ef8f5a329ap-7, 0x1.082ce2fa2ee21p-7, 0x1.05266b13505edp-7, 0x1.041cb887db79ap-7,
    0x1.011dfe07b7bf9p-7, 0x1.001c6d5e9d0bfp-7, 0x1.fa4ae5a014347p-8, 0x1.f85788f3e75dep-8,
    0x1.f27916b786f6ep-8, 0x1.f09503707a24ap-8, 0x1.eac615124bb06p-8, 0x1.e8f0d3af4b10ep-8,
    0x1.e33168437fc5ap-8, 0x1.e16a84e64372ep-8, 0x1.dbba99adffcfep-8, 0x1.da01a3fee1f0dp-8,
    0x1.d461347da5219p-8, 0x1.d2b5bf9050623p-8, 0x1.cd24c5a09ad13p-8, 0x1.cb8667d98ac89p-8,
    0x1.c604dbc0ca066p-8, 0x1.c4732ebb97518p-8, 0x1.bf01073d5d450p-8, 0x1.bd7ba7b3cf4bcp-8,
    0x1.b818da245a728p-8, 0x1.b69f67d638f8ep-8, 0x1.b14be82c53529p-8, 0x1.afde05c7f2247p-8,
    0x1.aa99c6ae2c37ep-8, 0x1.a93719b9ab674p-8, 0x1.a4020c9ef8a6ep-8, 0x1.a2aa3d6233fedp-8,
    0x1.9d845289eda7ep-8, 0x1.9c370bf9161dfp-8, 0x1.9720328a69879p-8, 0x1.95dd2231439c5p-8,
    0x1.90d5484610c3ap-8, 0x1.8f9c1e33d2e96p-8, 0x1.8aa330e6ffe3ap-8, 0x1.89739f9acc270p-8,
    0x1.84898b1611fd6p-8, 0x1.8363476c064e7p-8, 0x1.7e87f6f53ba49p-8, 0x1.7d6ab81414437p-8,
    0x1.789e1619fa06cp-8, 0x1.7789956141b68p-8, 0x1.72cb8b87d5f40p-8, 0x1.71bf847e9fb98p-8,
    0x1.6d0ffbaafa965p-8, 0x1.6c0c2bef20e69p-8, 0x1.676b0c52df998p-8, 0x1.666f3388c4fb4p-8,
    0x1.61dc64ad0685ep-8, 0x1.60e8446fd3c76p-8, 0x1.5c63ad3fcb107p-8, 0x1.5b77091227510p-8,
    0x1.57008fe54624fp-8, 0x1.561b2d22850c0p-8, 0x1.51b2b7c6436cbp-8, 0x1.50d45d9406051p-8,
    0x1.4c79d1554916fp-8, 0x1.4ba248958de01p-8, 0x1.47558a49b1a84p-8, 0x1.46849d8d5087cp-8,
    0x1.4245919ad795bp-8, 0x1.417b0d14666ddp-8, 0x1.3d49977b52720p-8, 0x1.3c8548f26f39dp-8,
    0x1.38614d5445738p-8, 0x1.37a3041942c55p-8, 0x1.338c65c0bf1a1p-8, 0x1.32d3f2a0b0437p-8,
    0x1.2eca948929bb8p-8, 0x1.2e17c9c24b717p-8, 0x1.2a1b8e9eccc04p-8, 0x1.296e3fd547aecp-8,
    0x1.257f0a175e576p-8, 0x1.24d70c4a60d99p-8, 0x1.20f4be28a56c4p-8, 0x1.2051e7a7d1ce9p-8,
    0x1.1c7c63242ba73p-8, 0x1.1bde8b8558689p-8, 0x1.1815b272ff42ep-8, 0x1.177cb28846de4p-8,
    0x1.13c0669184825p-8, 0x1.132c185fa25b4p-8, 0x1.0f7c3b0b56920p-8, 0x1.0eec79c04eb27p-8,
    0x1.0b48ec7737a01p-8, 0x1.0abd946147067p-8, 0x1.072638730ff8bp-8, 0x1.069f26f7e346bp-8,
    0x1.0313dd9ffbf25p-8, 0x1.0290f1342a5e3p-8, 0x1.fe23373cd0f11p-9, 0x1.fd25677a61e39p-9,
    0x1.f63e66147c069p-9, 0x1.f548605b09166p-9, 0x1.ee78caee338fcp-9, 0x1.ed8a521f461f9p-9,
    0x1.e6d1ead929e9bp-9, 0x1.e5eac3b4fcbf9p-9, 0x1.df494cc5338cbp-9, 0x1.de693ddc17f89p-9,
    0x1.d7de797b8c899p-9, 0x1.d7054b1fc1257p-9, 0x1.d090fb97b8fa5p-9, 0x1.cfbe77cfae95fp-9,
    0x1.c9605f80800abp-9, 0x1.c89451f9896efp-9, 0x1.c24c3361013a7p-9, 0x1.c18669626a8a4p-9,
    0x1.bb540721e37efp-9, 0x1.ba944f806e13dp-9, 0x1.b4776c629de93p-9, 0x1.b3bd97745da1dp-9,
    0x1.adb5f672d976cp-9, 0x1.ad01d6037085cp-9, 0x1.a70f3a4bebb5ap-9, 0x1.a660a19122142p-9,
    0x1.a082ce8a69e37p-9, 0x1.9fd992191da22p-9, 0x1.9a104b67d4319p-9, 0x1.996c41293ff7cp-9,
    0x1.93b74ab458d93p-9, 0x1.931849dbadf5dp-9, 0x1.8d7767d0aeaa8p-9, 0x1.8cdd48d1002fbp-9,
    0x1.87503fa806c46p-9, 0x1.86badc2a83389p-9, 0x1.814170aa15217p-9, 0x1.80b0a3848c65bp-9,
    0x1.7b4a9ac52fa9cp-9, 0x1.7abe3ff0e2c55p-9, 0x1.756b5f6083790p-9, 0x1.74e353f13c0cep-9,
    0x1.6fa361566008dp-9, 0x1.6f1f8371cd3fap-9, 0x1.69f244ee97f1cp-9, 0x1.697273c3eed05p-9,
    0x1.6457afd8f6f57p-9, 0x1.63dbcb98d400bp-9, 0x1.5ed34927cd048p-9, 0x1.5e5b32fc55421p-9,
    0x1.5964b94a8df62p-9, 0x1.58f0534fcd5a6p-9, 0x1.540baa0885a55p-9, 0x1.539ad74509130p-9,
    0x1.4ec7c67ba02acp-9, 0x1.4e5a6ad949345p-9, 0x1.4998bb0b45eb4p-9, 0x1.492ebb505694ep-9,
    0x1.447e35674b30ep-9, 0x1.4417772fa800fp-9, 0x1.3f77e482f30aap-9, 0x1.3f144e3999c0dp-9,
    0x1.3a8578900529dp-9, 0x1.3a24f168b684dp-9, 0x1.35a6a2f9f67a5p-9, 0x1.354912eb117dfp-9,
    0x1.30db166124300p-9, 0x1.3080661db16b1p-9, 0x1.2c22869621066p-9, 0x1.2bca9f880c629p-9,
    0x1.277ca89514702p-9, 0x1.272774d794221p-9, 0x1.22e932812b749p-9, 0x1.22969cdb52ac6p-9,
    0x1.1e67dba01afadp-9, 0x1.1e17cf7f97005p-9, 0x1.19f85c55b3417p-9, 0x1.19aac5c9b1b26p-9,
    0x1.159a6e1f84450p-9, 0x1.154f39d3c1347p-9, 0x1.114dcb9092d66p-9, 0x1.1104e6c88d964p-9,
    0x1.0d12304d1e22ep-9, 0x1.0ccb88df738b6p-9, 0x1.08e759067572ep-9, 0x1.08a2dd585e829p-9,
    0x1.04cd0376dde1cp-9, 0x1.048aa277d19bbp-9, 0x1.00c2ee5d87d49p-9, 0x1.00829782ff499p-9,
    0x1.f991b2f527eb2p-10, 0x1.f914f977dedbfp-10, 0x1.f1bd0b164ef4dp-10, 0x1.f14426bb677cap-10,
    0x1.ea07688b1ef8ap-10, 0x1.e9923b31547fap-10, 0x1.e27050aae655ap-10, 0x1.e1febd1d9b55fp-10,
    0x1.daf74ab029428p-10, 0x1.da8934a0270d8p-10, 0x1.d39bdfb14051ap-10, 0x1.d3312badaf96ap-10,
    0x1.cc5d9a9913621p-10, 0x1.cbf62e08abbcep-10, 0x1.c53c081ff094cp-10, 0x1.c4d7c93a5d757p-10,
    0x1.be36b6c47edb7p-10, 0x1.bdd58c8bf8274p-10, 0x1.b74d36c4cbbbep-10, 0x1.b6ef08ffe093dp-10,
    0x1.b07f1a1773e03p-10, 0x1.b023d14b06053p-10, 0x1.a9cbf464e6110p-10, 0x1.a97379ce546a3p-10,
    0x1.a3335b00c0357p-10, 0x1.a2dd98903f08bp-10, 0x1.9cb4e4e345f7ep-10, 0x1.9c61c536636f3p-10,
    0x1.96502aa2f0af4p-10, 0x1.95ff98ff44513p-10, 0x1.9004c66e182d0p-10, 0x1.8fb6aebc1bf8dp-10,
    0x1.89d25404b4136p-10, 0x1.8986a2cac5fa9p-10, 0x1.83b870b235568p-10, 0x1.836f130fbfd97p-10,
    0x1.7db6bb47778d7p-10, 0x1.7d6f9ef040487p-10, 0x1.77ccd414c9b9ep-10, 0x1.7787e74c64ba6p-10,
    0x1.71fa5ce40e2d5p-10, 0x1.71b78e7974ef7p-10, 0x1.6c3ef8f2f1346p-10, 0x1.6bfe383c3c328p-10,
    0x1.669a4ced3632bp-10, 0x1.665b89c377f82p-10, 0x1.610bfee71ad9ap-10, 0x1.60cf29a25b929p-10,
    0x1.5b93b657d026fp-10, 0x1.5b58bfcb28afcp-10, 0x1.56311c1408d80p-10, 0x1.55f7f589dc54ep-10,
    0x1.50e3da489d00ap-10, 0x1.50ac757ef00fdp-10, 0x1.4bab9c754275ap-10, 0x1.4b75eb9a2f135p-10,
    0x1.46880f6759bafp-10, 0x1.465405159ef72p-10, 0x1.4178e134cf287p-10, 0x1.414670707bd4cp-10,
    0x1.3c7dc1370ff7cp-10, 0x1.3c4cdd6a477a5p-10, 0x1.3796600612ef9p-10, 0x1.3766fcfdeb6e3p-10,
    0x1.32c26f737461cp-10, 0x1.3294815ced7f2p-10, 0x1.2e01a285a532cp-10, 0x1.2dd51deab69cep-10,
    0x1.2953ad732ca15p-10, 0x1.29288737ebb72p-10, 0x1.24b8459dfc86cp-10, 0x1.248e72fdd8605p-10,
    0x1.202f218ed7ca4p-10, 0x1.20069819eaf3ap-10, 0x1.1bb7f8f0cac08p-10, 0x1.1b90ae8941fdcp-10,
    0x1.1752848cb533bp-10, 0x1.172c6f644aa91p-10, 0x1.12fe7e44e5d04p-10, 0x1.12d994da6fef3p-10,
    0x1.0ebba110c6b3ap-10, 0x1.0e97da2dda510p-10, 0x1.0a89a8f89adb7p-10, 0x1.0a66fbaf3fda1p-10,
    0x1.066853114c34cp-10, 0x1.0646b6b9c4311p-10, 0x1.02575d784a0adp-10, 0x1.0236c9aee87c4p-10,
    0x1.fcad0e9eef2eep-11, 0x1.fc6de7e515baep-11, 0x1.f4cb217254ecbp-11, 0x1.f48debcdea99fp-11,
    0x1.ed0875a8717dbp-11, 0x1.eccd21d1f7352p-11, 0x1.e5648f702d0f6p-11, 0x1.e52b0e9850b60p-11,
    0x1.dddef4e20532bp-11, 0x1.dda738adf1189p-11, 0x1.d6772df8842a0p-11, 0x1.d641287e4b718p-11,
    0x1.cf2cc488d5ac9p-11, 0x1.cef8684bfcc70p-11, 0x1.c7ff443b78adep-11, 0x1.c7cc84299911dp-11,
    0x1.c0ee3a850db9cp-11, 0x1.c0bd09f293fcbp-11, 0x1.b9f9369f41764p-11, 0x1.b9c9894444fb6p-11,
    0x1.b31fc981d2df6p-11, 0x1.b2f193770652ep-11, 0x1.ac6185dbb4d1ap-11, 0x1.ac34bb976ead6p-11,
    0x1.a5be000c4a797p-11, 0x1.a592965fa4d74p-11, 0x1.9f34ce1cbe402p-11, 0x1.9f0aba30cd425p-11,
    0x1.98c587b972d01p-11, 0x1.989cbf0c90ef5p-11, 0x1.926fc62b8dca9p-11, 0x1.92483e8ebd5d9p-11,
    0x1.8c3324529bcd4p-11, 0x1.8c0cd3e6fd232p-11, 0x1.860f3e9e4d639p-11, 0x1.85ea1bd2a8d00p-11,
    0x1.8003b3084c857p-11, 0x1.7fdfb496afc1fp-11, 0x1.7a10210e2a42ep-11, 0x1.79ed3df9988d7p-11,
    0x1.743429ab643fap-11, 0x1.7412593d98a3dp-11, 0x1.6e6f6f5381a20p-11, 0x1.6e4ea91ac2de1p-11,
    0x1.68c195ec471aep-11, 0x1.68a1d1b94c95ep-11, 0x1.632a42c801ac2p-11, 0x1.630b78abe8f86p-11,
    0x1.5da91c9fe7d60p-11, 0x1.5d8b44ea3a3d4p-11, 0x1.583dcb8e90d50p-11, 0x1.5820decb58700p-11,
    0x1.52e7f90a81991p-11, 0x1.52cbf0006d79bp-11, 0x1.4da74fe0cf234p-11, 0x1.4d8c238f6619ep-11,
    0x1.487b7c2fd5f63p-11, 0x1.486125cdb77fcp-11, 0x1.43642b620646cp-11, 0x1.434aa45b39354p-11,
    0x1.3e610c28c49e1p-11, 0x1.3e484e1d130e2p-11, 0x1.3971ce775e9afp-11, 0x1.3959d338becfcp-11,
    0x1.3496237e1386bp-11, 0x1.347ee50f1d458p-11, 0x1.2fcdbda5306eep-11, 0x1.2fb736379e793p-11,
    0x1.2b1850883f787p-11, 0x1.2b027a7b7cc47p-11, 0x1.267590f14a214p-11, 0x1.266066d10a75ap-11,
    0x1.21e534d42e269p-11, 0x1.21d0b15711bf3p-11, 0x1.1d66f34a04c75p-11, 0x1.1d53115046ac9p-11,
    0x1.18fa848c9c1b7p-11, 0x1.18e73f1ecad83p-11, 0x1.149fa1f20238ep-11, 0x1.148cf43fc29d7p-11,
    0x1.105605e821e16p-11, 0x1.1043eb46fb851p-11, 0x1.0c1d6bf07074dp-11, 0x1.0c0bdfdaa3a86p-11,
    0x1.07f5909bace3fp-11, 0x1.07e48eaf11cc4p-11, 0x1.03de3185af625p-11, 0x1.03cdb5829df22p-11,
    0x1.ffae1aa2932a2p-12, 0x1.ff8e263314416p-12, 0x1.f7bfc7486dfcfp-12, 0x1.f7a0ce73f64b7p-12,
    0x1.eff0ea463ace5p-12, 0x1.efd2e55002287p-12, 0x1.e84106db3a0c8p-12, 0x1.e823ee435e82dp-12,
    0x1.e0afa234e0555p-12, 0x1.e0936eb6870c9p-12, 0x1.d93c436734533p-12, 0x1.d920edf6b9136p-12,
    0x1.d1e673654aac1p-12, 0x1.d1cbf52e7db48p-12, 0x1.caadbcf9df8cep-12, 0x1.ca940f5e513c8p-12,
    0x1.c391acc00d5e5p-12, 0x1.c378c9556743ap-12, 0x1.bc91d11c20301p-12, 0x1.bc79b1aa8b173p-12,
    0x1.b5adba34856a9p-12, 0x1.b59658b51c03ep-12, 0x1.aee4f9ead758cp-12, 0x1.aece508625146p-12,
    0x1.a83723d5041c8p-12, 0x1.a8212ce18fdb0p-12, 0x1.a1a3cd368fa21p-12, 0x1.a18e833771ddep-12,
    0x1.9b2a8cf9f02a5p-12, 0x1.9b15ea9d743e9p-12, 0x1.94cafbaa05013p-12, 0x1.94b6fbc855380p-12,
    0x1.8e84b36ba6fc4p-12, 0x1.8e715105830e4p-12, 0x1.88574ff7525adp-12, 0x1.88448634d00f2p-12,
    0x1.82426e92e9a46p-12, 0x1.823038c23f409p-12, 0x1.7c45ae0b91240p-12, 0x1.7c34079fe95f7p-12,
    0x1.7660aeafa29f6p-12, 0x1.764f933ff9cebp-12, 0x1.70931248b8eb2p-12, 0x1.70827d8ec31bbp-12,
    0x1.6adc7c15d2fe3p-12, 0x1.6acc69eceabb4p-12, 0x1.653c90c58e28bp-12, 0x1.652cfd29aba5ep-12,
    0x1.5fb2f67077130p-12, 0x1.5fa3dd7d2f7a6p-12, 0x1.5a3f5493712bbp-12, 0x1.5a30b282fdcf8p-12,
    0x1.54e1540a342cfp-12, 0x1.54d32534815e6p-12, 0x1.4f989f09df616p-12, 0x1.4f8adfe3a2b12p-12,
    0x1.4a64e11ba2544p-12, 0x1.4a578e357801ep-12, 0x1.4545c7177a980p-12, 0x1.4538dd1d09f83p-12,
    0x1.403aff1f0650fp-12, 0x1.402e7ad62cf30p-12, 0x1.3b4438986b31ep-12, 0x1.3b3816e06e909p-12,
    0x1.36612429519aep-12, 0x1.365561fa17242p-12, 0x1.319173b1f38aap-12, 0x1.31860e1b3ecd1p-12,
    0x1.2cd4da483f14fp-12, 0x1.2cc9ce70f5e22p-12, 0x1.282b0c330c114p-12, 0x1.2820575880666p-12,
    0x1.2393bee564b5bp-12, 0x1.23895e5aa43d2p-12, 0x1.1f0ea8f9e0d44p-12, 0x1.1f049a2709d3bp-12,
    0x1.1a9b822e13714p-12, 0x1.1a91c28faefa3p-12, 0x1.163a035e0a69dp-12, 0x1.163090846ba2ep-12,
    0x1.11e9e67fdfe4dp-12, 0x1.11e0be0e88435p-12, 0x1.0daae69f5d46cp-12, 0x1.0da2064c6592cp-12,
    0x1.097cbfd9af64fp-12, 0x1.0974256d3560ep-12, 0x1.055f2f592bb32p-12, 0x1.0556d8acc4438p-12,
    0x1.0151f3512629ap-12, 0x1.0149de4f53d8cp-12, 0x1.faa995f3af424p-13, 0x1.fa99eb3b0ab9ap-13,
    0x1.f2ceed18a8c8cp-13, 0x1.f2bfbdc0a8a96p-13, 0x1.eb136e7d256ecp-13, 0x1.eb04b6ba421a9p-13,
    0x1.e3769e7f0229fp-13, 0x1.e3685aa39565bp-13, 0x1.dbf8036657cbap-13, 0x1.dbea2fe1b1850p-13,
    0x1.d497255de4e59p-13, 0x1.d489bebb67354p-13, 0x1.cd538e6b95af2p-13, 0x1.cd469151d7dcap-13,
    0x1.c62cca6929741p-13, 0x1.c620339921c52p-13, 0x1.bf2266fcf517dp-13, 0x1.bf1633512935cp-13,
    0x1.b833f392c23c9p-13, 0x1.b8281ffe7dfafp-13, 0x1.b1610154ca9acp-13, 0x1.b1558ae35cee9p-13,
    0x1.aaa92324cf1c1p-13, 0x1.aa9e06f8cd118p-13, 0x1.a40bed954a4b4p-13, 0x1.a40128e7d7cbap-13,
    0x1.9d88f6e2bdad9p-13, 0x1.9d7e8702dbe72p-13, 0x1.971fd6ed199b1p-13, 0x1.9715b93efadefp-13,
    0x1.90d027313f2dfp-13, 0x1.90c6592da0190p-13, 0x1.8a9982c29be21p-13, 0x1.8a9001f621a6ap-13,
    0x1.847b8644de7ecp-13, 0x1.8472504f7a276p-13, 0x1.7e75cfe5c4e74p-13, 0x1.7e6ce27a1b6b8p-13,
    0x1.7887ff5702705p-13, 0x1.787f5839d974fp-13, 0x1.72b1b5c83e593p-13, 0x1.72a952cfed77bp-13,
    0x1.6cf295e12a097p-13, 0x1.6cea74f5107afp-13, 0x1.674a43bbaeb58p-13, 0x1.674262d3ad3e8p-13,
    0x1.61b864de320dep-13, 0x1.61b0c20229096p-13, 0x1.5c3ca035f19dbp-13, 0x1.5c35397d43077p-13,
    0x1.56d69e11747f3p-13, 0x1.56cf71a289ddap-13, 0x1.5186081b130e7p-13, 0x1.517f142ae71d1p-13,
    0x1.4c4a895394428p-13, 0x1.4c43cc2540409p-13, 0x1.4723ce0ce058ap-13, 0x1.471d45f12cde1p-13,
    0x1.421183e4c87c7p-13, 0x1.420b2f39c1ba5p-13, 0x1.3d1359bfe31adp-13, 0x1.3d0d36f0706bdp-13,
    0x1.3828ffc47c8d7p-13, 0x1.38230d47fb3c9p-13, 0x1.335227559bcf3p-13, 0x1.334c63af7cfb2p-13,
    0x1.2e8e830e1ae96p-13, 0x1.2e88eccd846cap-13, 0x1.29ddc6bbd2ccfp-13, 0x1.29d85c7b43121p-13,
    0x1.253fa75ada4a2p-13, 0x1.253a67bfcef61p-13, 0x1.20b3db10d7db7p-13, 0x1.20aec4cb77370p-13,
    0x1.1c3a192865f98p-13, 0x1.1c352af32b043p-13, 0x1.17d21a0c89ae8p-13, 0x1.17cd52abf2c68p-13,
    0x1.137b97443b210p-13, 0x1.1376f5867b2b7p-13, 0x1.0f364b6dffcf8p-13, 0x1.0f31ce2ab1cd4p-13,
    0x1.0b01f23b96369p-13, 0x1.0afd98537332dp-13, 0x1.06de486db29c3p-13, 0x1.06da10ca49e25p-13,
    0x1.02cb0bcfccbe5p-13, 0x1.02c6f5633e446p-13, 0x1.fd8ff667fc3e2p-14, 0x1.fd8809f16e29fp-14,
    0x1.f5a9acdde1603p-14, 0x1.f5a1feced441bp-14, 0x1.ede2bca7bb330p-14, 0x1.eddb4b14ba1fdp-14,
    0x1.e63aa96137bdbp-14, 0x1.e633726debf8cp-14, 0x1.deb0f8937d43cp-14, 0x1.dea9fa7237331p-14,
    0x1.d74531ad858d1p-14, 0x1.d73e6a9ec9581p-14, 0x1.cff6ddfc9774dp-14, 0x1.cff04c4ead2f4p-14,
    0x1.c8c588a4de48cp-14, 0x1.c8bf2ab3658e5p-14, 0x1.c1b0be9a1e82bp-14, 0x1.c1aa92cda567cp-14,
    0x1.bab80e988767bp-14, 0x1.bab2136624a57p-14, 0x1.b3db091da11b3p-14, 0x1.b3d53d06915d7p-14,
    0x1.ad19406156b57p-14, 0x1.ad13a1f29cf15p-14, 0x1.a672484f1bee0p-14, 0x1.a66cd62124aa3p-14,
    0x1.9fe5b67f2deddp-14, 0x1.9fe06f357564cp-14, 0x1.9973222feedd4p-14, 0x1.996e0478a9e26p-14,
    0x1.931a243f5bc3cp-14, 0x1.93152ed323578p-14, 0x1.8cda57249c522p-14, 0x1.8cd588c61bcdcp-14,
    0x1.86b356e9ac2fdp-14, 0x1.86aeae6551f62p-14, 0x1.80a4c1251d66ep-14, 0x1.80a03d50ce051p-14,
    0x1.7aae34f3f38b1p-14, 0x1.7aa9d4aebf372p-14, 0x1.74cf52f3973a2p-14, 0x1.74cb1525719bap-14,
    0x1.6f07bd3be1952p-14, 0x1.6f03a0d55bc6cp-14, 0x1.695717593f538p-14, 0x1.69531b53440bcp-14,
    0x1.63bd0646eb132p-14, 0x1.63b929a27ce33p-14, 0x1.5e3930693e88cp-14, 0x1.5e35722f38210p-14,
    0x1.58cb3d881a36cp-14, 0x1.58c79cc8f0a11p-14, 0x1.5372d6c963508p-14, 0x1.536f529cea117p-14,
    0x1.4e2fa6ab97739p-14, 0x1.4e2c3e30c6824p-14, 0x1.4901590075dedp-14, 0x1.48fe0b5d31664p-14,
    0x1.43e79ae7bdd40p-14, 0x1.43e467489faf4p-14, 0x1.3ee21aca01ceap-14, 0x1.3edf006224b20p-14,
    0x1.39f088538f3eap-14, 0x1.39ed865c5b812p-14, 0x1.3512946f6a74fp-14, 0x1.350faa28646d0p-14,
    0x1.3047f1425e728p-14, 0x1.30451df0f6598p-14, 0x1.2b905226204a9p-14, 0x1.2b8d9515839b4p-14,
    0x1.26eb6ba485cb6p-14, 0x1.26e8c425720f5p-14, 0x1.2258f372cf1fep-14, 0x1.225660db66210p-14,
    0x1.1dd8a06d0320ap-14, 0x1.1dd62218a073dp-14, 0x1.196a2a915e090p-14, 0x1.1967bfe06de68p-14,
    0x1.150d4afbd247ap-14, 0x1.150af353a9a85p-14, 0x1.10c1bbe19b23ep-14, 0x1.10bf76ac5117dp-14,
    0x1.0c87388ce0efbp-14, 0x1.0c8505392925bp-14, 0x1.085d7d586e81fp-14, 0x1.085b5b5974f60p-14,
    0x1.044447ab77b40p-14, 0x1.04423678bd7bap-14, 0x1.003b55f5709f7p-14, 0x1.0039550aa9cb5p-14,
    0x1.f884cf53eab28p-15, 0x1.f880ed0dcfc72p-15, 0x1.f0b27a7983d34p-15, 0x1.f0aeb6ca4b51ap-15,
    0x1.e8ff303b747fbp-15, 0x1.e8fb8a3233ab3p-15, 0x1.e16a756a03c5ap-15, 0x1.e166ec1d393fbp-15,
    0x1.d9f3d0be463fep-15, 0x1.d9f0634b9fa9dp-15, 0x1.d29acad28af68p-15, 0x1.d297785eac5eap-15,
    0x1.cb5eee1ae647bp-15, 0x1.cb5bb5d133548p-15, 0x1.c43fc6ddda639p-15, 0x1.c43ca7f0412e2p-15,
    0x1.bd3ce32d1ce46p-15, 0x1.bd39dcd3e2757p-15, 0x1.b655d2de7910ap-15, 0x1.b652e4580773bp-15,
    0x1.af8a2784ce55bp-15, 0x1.af8750158434cp-15, 0x1.a8d974692a8a0p-15, 0x1.a8d6b35b2c46ap-15,
    0x1.a2434e83ff8a5p-15, 0x1.a240a32709c83p-15, 0x1.9bc74c7673c45p-15, 0x1.9bc4b61faf596p-15,
    0x1.95650683cd446p-15, 0x1.9562848da4846p-15, 0x1.8f1c168af6ddep-15, 0x1.8f19a854ec361p-15,
    0x1.88ec18001f05cp-15, 0x1.88e9bceea4de6p-15, 0x1.82d4a7e66ff9fp-15, 0x1.82d25f62c1d3dp-15,
    0x1.7cd564c9e0d19p-15, 0x1.7cd32e41dd960p-15, 0x1.76edeeb91f130p-15, 0x1.76ebc99f248c4p-15,
    0x1.711de73f906e5p-15, 0x1.711bd30a57dffp-15, 0x1.6b64f15f6c3d1p-15, 0x1.6b62ed89e812ep-15,
    0x1.65c2b18bec68bp-15, 0x1.65c0bd9526f43p-15, 0x1.6036cda3955b0p-15, 0x1.6034e90e90969p-15,
    0x1.5ac0ecea949d4p-15, 0x1.5abf173e2aed5p-15, 0x1.5560b80535cc7p-15, 0x1.555ef0cbfbb68p-15,
    0x1.5015d8f26d897p-15, 0x1.50141fba945a1p-15, 0x1.4adffb067a0ebp-15, 0x1.4ade4f61b3660p-15,
    0x1.45becae59914dp-15, 0x1.45bd2c68fb53cp-15, 0x1.40b1f67ed2b2dp-15, 0x1.40b064c2be40dp-15,
    0x1.3bb92d06d8e55p-15, 0x1.3bb7a7a6de492p-15, 0x1.36d41ef2fb6c3p-15, 0x1.36d2a58dc2303p-15,
    0x1.32027df42fad1p-15, 0x1.3201102b5e09cp-15, 0x1.2d43fcf22c4c1p-15, 0x1.2d429a6a4f91bp-15,
    0x1.28985006982c0p-15, 0x1.2896f8670de67p-15, 0x1.23ff2c784c898p-15, 0x1.23fddf6b2c57ep-15,
    0x1.1f7848b6a9e58p-15, 0x1.1f7705e8b0004p-15, 0x1.1b035c54ff73ap-15, 0x1.1b02237577dc1p-15,
    0x1.16a0200604c48p-15, 0x1.169ef0c6b717ep-15, 0x1.124e4d9765622p-15, 0x1.124d27ac814bbp-15,
    0x1.0e0d9fed5e187p-15, 0x1.0e0c830d685ddp-15, 0x1.09ddd2fe6ba33p-15, 0x1.09dcbee22bc5ap-15,
    0x1.05bea3cf0a7cdp-15, 0x1.05bd983178eb2p-15, 0x1.01afd06d87897p-15, 0x1.01aecd0bbc5e9p-15,
    0x1.fb622fdbc2b94p-16, 0x1.fb60390e074b0p-16, 0x1.f38474cb73ac6p-16, 0x1.f3828d75deb7ap-16,
    0x1.ebc5f1d0afae2p-16, 0x1.ebc419796ad03p-16, 0x1.e4262b05719a8p-16, 0x1.e424613666069p-16,
    0x1.dca4a66f63b0dp-16, 0x1.dca2eab61caa5p-16, 0x1.d540ebf84092ap-16, 0x1.d53f3de5ced08p-16,
    0x1.cdfa8566527e8p-16, 0x1.cdf8e48f306f6p-16, 0x1.c6d0fe55104e6p-16, 0x1.c6cf6a5107378p-16,
    0x1.bfc3e42dd7c48p-16, 0x1.bfc25c97e5b40p-16, 0x1.b8d2c620c4b13p-16, 0x1.b8d14a97033dfp-16,
    0x1.b1fd351da480cp-16, 0x1.b1fbc5413050ap-16, 0x1.ab42c3cd05bf6p-16, 0x1.ab415f41e6cecp-16,
    0x1.a4a3068963251p-16, 0x1.a4a1acf675c8dp-16, 0x1.9e1d935869bc7p-16, 0x1.9e1c446748591p-16,
    0x1.97b201e459b7fp-16, 0x1.97b0bd4147285p-16, 0x1.915feb75818d3p-16, 0x1.915eb0cf54335p-16,
    0x1.8b26eaebd2ec9p-16, 0x1.8b25b9f3e0672p-16, 0x1.85069cb891303p-16, 0x1.850575229ab02p-16,
    0x1.7efe9ed818dbap-16, 0x1.7efd805a38146p-16, 0x1.790e90cbbfca6p-16, 0x1.790d7b1e54786p-16,
    0x1.73361393cdaa2p-16, 0x1.733506716baabp-16, 0x1.6d74c9a98c613p-16, 0x1.6d73c4ceea57cp-16,
    0x1.67ca56f970021p-16, 0x1.67c95a2556856p-16, 0x1.623660dd55ee0p-16, 0x1.62356bd08f3abp-16,
    0x1.5cb88e16dacbcp-16, 0x1.5cb7a09422f6cp-16, 0x1.575086c9c6f78p-16, 0x1.574fa095bc9cfp-16,
    0x1.51fdf47691123p-16, 0x1.51fd1557a67d4p-16, 0x1.4cc081f4f659ap-16, 0x1.4cbfa9b36320fp-16,
    0x1.4797db6ea8725p-16, 0x1.479709d45b85ep-16, 0x1.4283ae5a104dap-16, 0x1.4282e332a2727p-16,
    0x1.3d83a97525d9ap-16, 0x1.3d82e48dcc901p-16, 0x1.38977cc05c270p-16, 0x1.3896bde7dcf80p-16,
    0x1.33bed979a1b4dp-16, 0x1.33be208045e33p-16, 0x1.2ef9721774914p-16, 0x1.2ef8becefd2c2p-16,
    0x1.2a46fa440a01dp-16, 0x1.2a464c7fa454bp-16, 0x1.25a726d889647p-16, 0x1.25a67e6cc3c28p-16,
    0x1.2119add859fdcp-16, 0x1.21190a9b18e5ap-16, 0x1.1c9e466c8369cp-16, 0x1.1c9da834f6fe6p-16,
    0x1.1834a8df20647p-16, 0x1.18340f85ba390p-16, 0x1.13dc8e96e3a18p-16, 0x1.13dbf9f54cd5fp-16,
    0x1.0f95b212ae6c3p-16, 0x1.0f952203be176p-16, 0x1.0b5fcee538c84p-16, 0x1.0b5f4344eaadcp-16,
    0x1.073aa1b0cacebp-16, 0x1.073a1a5c365d8p-16, 0x1.0325e82307019p-16, 0x1.032564f8569a3p-16,
    0x1.fe42c1e18aa8dp-17, 0x1.fe41c39e5ba66p-17, 0x1.f65997a3fd4c8p-17, 0x1.f658a1336e613p-17,
    0x1.ee8fd2fb90d85p-17, 0x1.ee8ee42004fc9p-17, 0x1.e6e4f74cc0987p-17, 0x1.e6e40fca800b0p-17,
    0x1.df5889ea8ed3cp-17, 0x1.df57a987b82b8p-17, 0x1.d7ea120eda499p-17, 0x1.d7e9389353fd3p-17,
    0x1.d09918d2d21b3p-17, 0x1.d09846083c7abp-17, 0x1.c965292787a7bp-17, 0x1.c9645cd92f445p-17,
    0x1.c24dcfce9de3cp-17, 0x1.c24d09c96e630p-17, 0x1.bb529b5315b7bp-17, 0x1.bb51db658d0e5p-17,
    0x1.b4731c0236f1fp-17, 0x1.b47261fc59032p-17, 0x1.adaee3e4955b2p-17, 0x1.adae2f97dff97p-17,
    0x1.a70586b7317cfp-17, 0x1.a704d7f690c9ap-17, 0x1.a07699e4b4ae0p-17, 0x1.a075f08477d42p-17,
    0x1.9a01b47ec7f61p-17, 0x1.9a011054963dfp-17, 0x1.93a66f3785605p-17, 0x1.93a5d01a53996p-17,
    0x1.8d64645b0352fp-17, 0x1.8d63ca230990fp-17, 0x1.873b2fc8f984ep-17, 0x1.873a9a4fa92dap-17,
    0x1.812a6eee7f2b6p-17, 0x1.8129de0e79531p-17, 0x1.7b31c0bfe1fc7p-17, 0x1.7b313454ee0dep-17,
    0x1.7550c5b295a2ap-17, 0x1.75503d999850ep-17, 0x1.6f871fb73b41dp-17, 0x1.6f869bce2dc18p-17,
    0x1.69d47233c0ad9p-17, 0x1.69d3f259a832dp-17, 0x1.643861fd96f20p-17, 0x1.6437e6127c720p-17,
    0x1.5eb29553ffd49p-17, 0x1.5eb21d38e8075p-17, 0x1.5942b3da71ef7p-17, 0x1.59423f7155911p-17,
    0x1.53e86693130f7p-17, 0x1.53e7f5bed75e7p-17, 0x1.4ea357d9487bap-17, 0x1.4ea2ea7db7f1dp-17,
    0x1.4973335c5ccf5p-17, 0x1.4972c95e2014ap-17, 0x1.4457a61a3b119p-17, 0x1.44573f5ed225dp-17,
    0x1.3f505e5a3eb52p-17, 0x1.3f4ffac7fa504p-17, 0x1.3a5d0ba8182e9p-17, 0x1.3a5cab2613548p-17,
    0x1.357d5ecec5ce7p-17, 0x1.357d0144df962p-17, 0x1.30b109d3a08fbp-17, 0x1.30b0af2a761a5p-17,
    0x1.2bf7bff17c89dp-17, 0x1.2bf76812632a7p-17, 0x1.27513593dcbadp-17, 0x1.2750e068dc4b5p-17,
    0x1.22bd205239da0p-17, 0x1.22bccdc6073d4p-17, 0x1.1e3b36eb5bea6p-17, 0x1.1e3ae6e953b92p-17,
    0x1.19cb3140c6400p-17, 0x1.19cae3b4e7a02p-17, 0x1.156cc85235b0dp-17, 0x1.156c7d291d552p-17,
    0x1.111fb63930a83p-17, 0x1.111f6d6013f76p-17, 0x1.0ce3b624a8d61p-17, 0x1.0ce36f8951380p-17,
    0x1.08b88454ae341p-17, 0x1.08b83fe574842p-17, 0x1.049dde16331bap-17, 0x1.049d9bc1fb3efp-17,
    0x1.009381bee129fp-17, 0x1.0093417515c81p-17, 0x1.f9325d51fd5c1p-18, 0x1.f931e0b31a17dp-18,
    0x1.f15d4a5ec8c11p-18, 0x1.f15cd19570b6fp-18, 0x1.e9a74d5306470p-18, 0x1.e9a6d84106986p-18,
    0x1.e20feacef3169p-18, 0x1.e20f795706becp-18, 0x1.da96a95c71e35p-18, 0x1.da963b623a662p-18,
    0x1.d33b116773aabp-18, 0x1.d33aa6cf71fcfp-18, 0x1.cbfcad367e936p-18, 0x1.cbfc45e60c3adp-18,
    0x1.c4db08e352742p-18, 0x1.c4daa4c09addbp-18, 0x1.bdd5b253aa8dbp-18, 0x1.bdd55145a4986p-18,
    0x1.b6ec39321c02fp-18, 0x1.b6ebdb2083bd9p-18, 0x1.b01e2ee7109e3p-18, 0x1.b01dd3ba61360p-18,
    0x1.a96b2691dd71ep-18, 0x1.a96ace334b518p-18, 0x1.a2d2b501f4e81p-18, 0x1.a2d25f5b68047p-18,
    0x1.9c5470b033d21p-18, 0x1.9c541dac42246p-18, 0x1.95eff1b8490e0p-18, 0x1.95efa14231391p-18,
    0x1.8fa4d1d237590p-18, 0x1.8fa483d5db78dp-18, 0x1.8972ac4bf0e53p-18, 0x1.897260b5d1879p-18,
    0x1.83591e030c4e5p-18, 0x1.8358d4c04392bp-18, 0x1.7d57c55e9287bp-18, 0x1.7d577e5ccf65cp-18,
    0x1.776e4248e5608p-18, 0x1.776dfd766713dp-18, 0x1.719c3629be3cep-18, 0x1.719bf3754fd4ap-18,
    0x1.6be143e044a41p-18, 0x1.6be1033938b5bp-18, 0x1.663d0fbd3c443p-18, 0x1.663cd11368c02p-18,
    0x1.60af3f7d4a0fdp-18, 0x1.60af02c10436dp-18, 0x1.5b377a4350187p-18, 0x1.5b373f656890bp-18,
    0x1.55d56892dfcc5p-18, 0x1.55d52f849ed5dp-18, 0x1.5088b44ac23eep-18, 0x1.50887cfde4054p-18,
    0x1.4b51089f9623ap-18, 0x1.4b50d306472d2p-18, 0x1.462e121683263p-18, 0x1.462dde235cdecp-18,
    0x1.411f7e80024a3p-18, 0x1.411f4c2607aa0p-18, 0x1.3c24fcf2baffep-18, 0x1.3c24cc25554bap-18,
    0x1.373e3dc6749aep-18, 0x1.373e0e79703e7p-18, 0x1.326af28f1bdacp-18, 0x1.326ac4b6a55bep-18,
    0x1.2daace17dc352p-18, 0x1.2daaa1a87d3eep-18, 0x1.28fd845e4c939p-18, 0x1.28fd594ce9186p-18,
    0x1.2462ca8daf37ap-18, 0x1.2462a0cf82aa5p-18, 0x1.1fda56fa4478fp-18, 0x1.1fda2e84df1bcp-18,
    0x1.1b63e11cb0135p-18, 0x1.1b63b9e5f45bbp-18, 0x1.16ff218d70ba0p-18, 0x1.16fefb8b90c95p-18,
    0x1.12abd20069a90p-18, 0x1.12abad29e4d8dp-18, 0x1.0e69ad407deb8p-18, 0x1.0e69898c1e6dbp-18,
    0x1.0a386f2b3d12ap-18, 0x1.0a384c9015a38p-18, 0x1.0617d4aca1161p-18, 0x1.0617b3220ac18p-18,
    0x1.02079bbadd1b8p-18, 0x1.02077b387512cp-18, 0x1.fc0f06a479c25p-19, 0x1.fc0ec79fc4c47p-19,
    0x1.f42e96e229123p-19, 0x1.f42e59cdcdad4p-19, 0x1.ec6d6a27810b3p-19, 0x1.ec6d2ef439dd2p-19,
    0x1.e4cb04616aca3p-19, 0x1.e4cacb006ab83p-19, 0x1.dd46eb693e7f2p-19, 0x1.dd46b3cc2d026p-19,
    0x1.d5e0a6fd210e8p-19, 0x1.d5e07116169dcp-19, 0x1.ce97c0b87ffe6p-19, 0x1.ce978c7a02947p-19,
    0x1.c76bc40cab385p-19, 0x1.c76b9169aaf51p-19, 0x1.c05c3e398c289p-19, 0x1.c05c0d25600d0p-19,
    0x1.b968be4679c5ep-19, 0x1.b9688eb4dc8a2p-19, 0x1.b290d4fb2910ep-19, 0x1.b290a6e036127p-19,
    0x1.abd414d8b997dp-19, 0x1.abd3e828e9e09p-19, 0x1.a5321212dd911p-19, 0x1.a531e6c304f56p-19,
    0x1.9eaa62891d1e6p-19, 0x1.9eaa388e67720p-19, 0x1.983c9dc0344cfp-19, 0x1.983c751022ae2p-19,
    0x1.91e85cdb8b68ap-19, 0x1.91e8356bf1a00p-19, 0x1.8bad3a96c9392p-19, 0x1.8bad145dcb2efp-19,
    0x1.858ad33f7ec33p-19, 0x1.858aae338e081p-19, 0x1.7f80c4aeec27fp-19, 0x1.7f80a0c6c5913p-19,
    0x1.798eae43de3eap-19, 0x1.798e8b7687958p-19, 0x1.73b430dca4875p-19, 0x1.73b40f216a4a7p-19,
    0x1.6df0eed11f14fp-19, 0x1.6df0ce1f924b6p-19, 0x1.68448bece4109p-19, 0x1.68446c3cd82dfp-19,
    0x1.62aead697c777p-19, 0x1.62ae8eb30550dp-19, 0x1.5d2ef9e8b7b80p-19, 0x1.5d2edc242788ep-19,
    0x1.57c5196f15d33p-19, 0x1.57c4fc94fb520p-19, 0x1.5270b55e47a89p-19, 0x1.527099676c2a3p-19,
    0x1.4d31786fc514dp-19, 0x1.4d315d552abf0p-19, 0x1.48070eaf788d2p-19, 0x1.4806f46a58970p-19,
    0x1.42f125767fe10p-19, 0x1.42f10c0048e14p-19, 0x1.3def6b6601cf2p-19, 0x1.3def52b85617dp-19,
    0x1.39019062181b2p-19, 0x1.39017876cc21fp-19, 0x1.3427458ccdd16p-19, 0x1.34272e5de6a4fp-19,
    0x1.2f603d41316a9p-19, 0x1.2f6026c8e333cp-19, 0x1.2aac2b0e7a7f0p-19, 0x1.2aac1547270d9p-19,
    0x1.260ac3b342bc0p-19, 0x1.260aae97781f7p-19, 0x1.217bbd18d1cfdp-19, 0x1.217ba8a348fa8p-19,
    0x1.1cfece4e7bffap-19, 0x1.1cfeba7a17755p-19, 0x1.1893af85131f0p-19, 0x1.18939c4cddad5p-19,
    0x1.143a1a0a699e3p-19, 0x1.143a0769951f3p-19, 0x1.0ff1c844e768dp-19, 0x1.0ff1b636cb8fap-19,
    0x1.0bba75af304ddp-19, 0x1.0bba642f497c5p-19, 0x1.0793ded3dbaa8p-19, 0x1.0793cdddc9d0bp-19,
    0x1.037dc1493d158p-19, 0x1.037db0d8c2994p-19, 0x1.feefb75a7b895p-20, 0x1.feef977c7ce47p-20,
    0x1.f703db428cd8cp-20, 0x1.f703bc5f8cdf0p-20, 0x1.ef376f8c72ae0p-20, 0x1.ef37519cb877cp-20,
    0x1.e789f770f8e6fp-20, 0x1.e789da6d085f6p-20, 0x1.dffaf8182638cp-20, 0x1.dffadbf8be3e5p-20,
    0x1.d889f8918eb08p-20, 0x1.d889dd4fa7453p-20, 0x1.d13681ccc4adbp-20, 0x1.d13667618d34ap-20,
    0x1.ca001e91e7db8p-20, 0x1.ca0004f6c564dp-20, 0x1.c2e65b7a51b33p-20, 0x1.c2e642a8dd554p-20,
    0x1.bbe8c6e95f11ap-20, 0x1.bbe8aedb644f7p-20, 0x1.b506f105566d8p-20, 0x1.b506d9b4d1a96p-20,
    0x1.ae406bb06a3b1p-20, 0x1.ae4055178735dp-20, 0x1.a794ca81d70f7p-20, 0x1.a794b49aef732p-20,
    0x1.a103a2bf1d13bp-20, 0x1.a1038d84b70a2p-20, 0x1.9a8c8b55545c6p-20, 0x1.9a8c76c22130bp-20,
    0x1.942f1cd29bba6p-20, 0x1.942f08e176852p-20, 0x1.8deaf15fa19c1p-20, 0x1.8deade0b8dfa4p-20,
    0x1.87bfa4b946974p-20, 0x1.87bf91fd6f6b0p-20, 0x1.81acd42a59367p-20, 0x1.81acc2020f71ap-20,
    0x1.7bb21e856aa44p-20, 0x1.7bb20cec241d1p-20, 0x1.75cf241ebbd3cp-20, 0x1.75cf13101221bp-20,
    0x1.700386c642c2fp-20, 0x1.7003763df2258p-20, 0x1.6a4ee9c1c778fp-20, 0x1.6a4ed9bbadc68p-20,
    0x1.64b0f1c71860ep-20, 0x1.64b0e23f33fe5p-20, 0x1.5f2944f655a59p-20, 0x1.5f2935e8c4859p-20,
    0x1.59b78ad45331bp-20, 0x1.59b77c3d51dc8p-20, 0x1.545b6c4510fb9p-20, 0x1.545b5e20f99dep-20,
    0x1.4f14938649436p-20, 0x1.4f1485d192c50p-20, 0x1.49e2ac2a146d0p-20, 0x1.49e29ee1518e8p-20,
    0x1.44c56311a21fep-20, 0x1.44c55631809f4p-20, 0x1.3fbc66680757fp-20, 0x1.3fbc59ed4f1c2p-20,
    0x1.3ac7659d21152p-20, 0x1.3ac75984b35fdp-20, 0x1.35e611608b574p-20, 0x1.35e605a761fd4p-20,
    0x1.31181b9cac15ap-20, 0x1.3118103fd8bd6p-20, 0x1.2c5d3771d1e39p-20, 0x1.2c5d2c6e7d495p-20,
    0x1.27b5193165f30p-20, 0x1.27b50e84cf336p-20, 0x1.231f765931293p-20, 0x1.231f6c00ad108p-20,
    0x1.1e9c058eb3f8ep-20, 0x1.1e9bfb87ac58cp-20, 0x1.1a2a7e9a90b88p-20, 0x1.1a2a74e283c1dp-20,
    0x1.15ca9a640829cp-20, 0x1.15ca90f887ccap-20, 0x1.117c12ec87eb9p-20, 0x1.117c09cb393bap-20,
    0x1.0d3ea34b4a8edp-20, 0x1.0d3e9a71e52c8p-20, 0x1.091207a90907ap-20, 0x1.0911ff15568e0p-20,
    0x1.04f5fd3bbd36ap-20, 0x1.04f5f4eb98addp-20, 0x1.00ea424275465p-20, 0x1.00ea3a33ca9a6p-20,
    0x1.f9dd2c026f331p-21, 0x1.f9dd1c64062a8p-21, 0x1.f2057179ee137p-21, 0x1.f205625689ab9p-21,
    0x1.ea4cd76f2e675p-21, 0x1.ea4cc8c305b33p-21, 0x1.e2b2e2580126ap-21, 0x1.e2b2d41f6908dp-21,
    0x1.db37189488601p-21, 0x1.db370acbf2a00p-21, 0x1.d3d902679d36ap-21, 0x1.d3d8f50b979cdp-21,
    0x1.cc9829ef540a6p-21, 0x1.cc981cfc8783ep-21, 0x1.c5741b1d9e54dp-21, 0x1.c5740e90ce1d9p-21,
    0x1.be6c63b109c39p-21, 0x1.be6c578712971p-21, 0x1.b780932d9c1c4p-21, 0x1.b7808763736cdp-21,
    0x1.b0b03ad5cb782p-21, 0x1.b0b02f687eac2p-21, 0x1.a9faeda39266fp-21, 0x1.a9fae290461c2p-21,
    0x1.a36040419f899p-21, 0x1.a36035858ede5p-21, 0x1.9cdfc904a0384p-21, 0x1.9cdfbe9d1c1a7p-21,
    0x1.96791fe4a5c91p-21, 0x1.967915cf1449ep-21, 0x1.902bde76a50bcp-21, 0x1.902bd4b080b9ap-21,
    0x1.89f79fe60f94cp-21, 0x1.89f7966ce6d9cp-21, 0x1.83dc00ee866f7p-21, 0x1.83dbf7bffaf50p-21,
    0x1.7dd89fd5a5d39p-21, 0x1.7dd896ef6beacp-21, 0x1.77ed1c64e97a7p-21, 0x1.77ed13c4c7890p-21,
    0x1.721917e3a931ep-21, 0x1.72190f8777240p-21, 0x1.6c5c35112d4d2p-21, 0x1.6c5c2cf6d40b7p-21,
    0x1.66b6181eda951p-21, 0x1.66b61044537e7p-21, 0x1.612666aa75597p-21, 0x1.61265f0dc9c1ep-21,
    0x1.5bacc7b87b492p-21, 0x1.5bacc057c3fbap-21, 0x1.5648e3ae93b50p-21, 0x1.5648dc87f87a2p-21,
    0x1.50fa644e15e65p-21, 0x1.50fa5d5fcd0ddp-21, 0x1.4bc0f4aea52f5p-21, 0x1.4bc0edf6f31dep-21,
    0x1.469c4138e2616p-21, 0x1.469c3ab619219p-21, 0x1.418bf7a132526p-21, 0x1.418bf151b1296p-21,
    0x1.3c8fc6e2991ebp-21, 0x1.3c8fc0c4cc23dp-21, 0x1.37a75f39a9d52p-21, 0x1.37a7594c098d3p-21,
    0x1.32d2721f8a3bep-21, 0x1.32d26c609b36fp-21, 0x1.2e10b2450a5e6p-21, 0x1.2e10acb35cd92p-21,
    0x1.2961d38dcf966p-21, 0x1.2961ce27ff1e1p-21, 0x1.24c58b0b92c1bp-21, 0x1.24c585d045db2p-21,
    0x1.203b8ef97159ep-21, 0x1.203b89e7592afp-21, 0x1.1bc396b75121ap-21, 0x1.1bc391cd291d9p-21,
    0x1.175d5ac5561f6p-21, 0x1.175d5601e3b5ap-21, 0x1.130894bf6a9b1p-21, 0x1.130890217ce8dp-21,
    0x1.0ec4ff58d8d91p-21, 0x1.0ec4fadf485cdp-21, 0x1.0a925657f64a9p-21, 0x1.0a925201a49a4p-21,
    0x1.06705691dfef2p-21, 0x1.0670525db770ap-21, 0x1.025ebde647a26p-21, 0x1.025eb9d33b460p-21,
    0x1.fcba9676a426ap-22, 0x1.fcba8e90ba214p-22, 0x1.f4d77cf30a45ap-22, 0x1.f4d7754b556eap-22,
    0x1.ed13b10f8ccfcp-22, 0x1.ed13a9a4232fdp-22, 0x1.e56eb68ed334fp-22, 0x1.e56eaf5dd9e7fp-22,
    0x1.dde813209d49dp-22, 0x1.dde80c284807dp-22, 0x1.d67f4e5a1e3bfp-22, 0x1.d67f4798aee68p-22,
    0x1.cf33f1ae75de2p-22, 0x1.cf33eb223c106p-22, 0x1.c805886747d2bp-22, 0x1.c805820ea075ap-22,
    0x1.c0f39f9d701ecp-22, 0x1.c0f39976c5002p-22, 0x1.b9fdc631d4b0bp-22, 0x1.b9fdc03b9c1d9p-22,
    0x1.b3238cc653675p-22, 0x1.b32386ff0fc9cp-22, 0x1.ac6485b6cc291p-22, 0x1.ac64801d0ba86p-22,
    0x1.a5c04512469aap-22, 0x1.a5c03fa4a2bf6p-22, 0x1.9f3660943308fp-22, 0x1.9f365b5150630p-22,
    0x1.98c66f9dc6194p-22, 0x1.98c66a8453e8fp-22, 0x1.92700b2f6ed5ap-22, 0x1.9270063e26b7ap-22,
    0x1.8c32cde266ad6p-22, 0x1.8c32c9180c493p-22, 0x1.860e53e25b021p-22, 0x1.860e4f3dbbbabp-22,
    0x1.80023ae72fdbcp-22, 0x1.8002366722835p-22, 0x1.7a0e222edb60fp-22, 0x1.7a0e1dd23fee1p-22,
    0x1.7431aa7759afap-22, 0x1.7431a63d18f5bp-22, 0x1.6e6c75f8b8b68p-22, 0x1.6e6c71dfc41fdp-22,
    0x1.68be285f3bb02p-22, 0x1.68be24668cfa0p-22, 0x1.632666c595e08p-22, 0x1.632662ec2eda1p-22,
    0x1.5da4d7af3c3a7p-22, 0x1.5da4d3f42684dp-22, 0x1.58392302cd90fp-22, 0x1.58391f651a61cp-22,
    0x1.52e2f20490fb1p-22, 0x1.52e2ee8358e0cp-22, 0x1.4da1ef510a129p-22, 0x1.4da1ebeb6cba7p-22,
    0x1.4875c6d7a2b67p-22, 0x1.4875c38cc6b4ap-22, 0x1.435e25d569fb9p-22, 0x1.435e22a47c94cp-22,
    0x1.3e5abacfe7f86p-22, 0x1.3e5ab7b81ced0p-22, 0x1.396b359006178p-22, 0x1.396b32909770ap-22,
    0x1.348f471d0ba0ep-22, 0x1.348f4435397efp-22, 0x1.2fc6a1b7ae28ep-22, 0x1.2fc69ee6be938p-22,
    0x1.2b10f8d535966p-22, 0x1.2b10f61a744dep-22, 0x1.266e011ab3719p-22, 0x1.266dfe7571c20p-22,
    0x1.21dd70584d303p-22, 0x1.21dd6dc7e1c5bp-22, 0x1.1d5efd8499329p-22, 0x1.1d5efb085feedp-22,
    0x1.18f260b80e27dp-22, 0x1.18f25e4f67f94p-22, 0x1.1497532884905p-22, 0x1.149750d2d74a3p-22,
    0x1.104d8f24ca164p-22, 0x1.104d8ce1804a2p-22, 0x1.0c14d01046759p-22, 0x1.0c14cddecf4dfp-22,
    0x1.07ecd25eb1ad6p-22, 0x1.07ecd03e80c9bp-22, 0x1.03d5538fdb372p-22, 0x1.03d5518068884p-22,
    0x1.ff9c245703fcbp-23, 0x1.ff9c20589349bp-23, 0x1.f7ad9b7a79b05p-23, 0x1.f7ad979b7e06bp-23,
    0x1.efde8da0e6703p-23, 0x1.efde89e0680bep-23, 0x1.e82e7dd8cbc3fp-23, 0x1.e82e7a35da806p-23,
    0x1.e09cf1208eb2ep-23, 0x1.e09ced9a41cedp-23, 0x1.d9296e5ec7a15p-23, 0x1.d9296af43d84fp-23,
    0x1.d1d37e5ab0b1ap-23, 0x1.d1d37b0b0eb5ep-23, 0x1.ca9aabb4b22f1p-23, 0x1.ca9aa87f24671p-23,
    0x1.c37e82df0c8bcp-23, 0x1.c37e7fc2c58fcp-23, 0x1.bc7e92169f7c5p-23, 0x1.bc7e8f12d8367p-23,
    0x1.b59a695bcdbdap-23, 0x1.b59a666fc5382p-23, 0x1.aed19a6b7d12dp-23, 0x1.aed197967847ap-23,
    0x1.a823b8b8320b6p-23, 0x1.a823b5f97bb58p-23, 0x1.a19059634723bp-23, 0x1.a19056ba2f920p-23,
    0x1.9b1713363ed2cp-23, 0x1.9b1710a21bbbbp-23, 0x1.94b77e9c301a7p-23, 0x1.94b77c1c5c71fp-23,
    0x1.8e71359b4d318p-23, 0x1.8e71332f28ff5p-23, 0x1.8843d3ce83df2p-23, 0x1.8843d1757416fp-23,
    0x1.822ef65f37223p-23, 0x1.822ef418a57cfp-23, 0x1.7c323bff11c04p-23, 0x1.7c3239ca6c968p-23,
    0x1.764d44e1f158fp-23, 0x1.764d42beab7e7p-23, 0x1.707fb2b7e99cap-23, 0x1.707fb0a57a3d1p-23,
    0x1.6ac928a75f46bp-23, 0x1.6ac926a541c39p-23, 0x1.65294b473a7cep-23, 0x1.65294954ee4c1p-23,
    0x1.5f9fc0993036dp-23, 0x1.5f9fbeb638c2cp-23, 0x1.5a2c30042252bp-23, 0x1.5a2c2e3006dafp-23,
    0x1.54ce424e95fcbp-23, 0x1.54ce4088e177fp-23, 0x1.4f85a1994010ap-23, 0x1.4f859fe1810f7p-23,
    0x1.4a51f959a71f0p-23, 0x1.4a51f7af6faf5p-23, 0x1.4532f654dabedp-23, 0x1.4532f4b7c050ap-23,
    0x1.4028469a3fd85p-23, 0x1.40284509db22cp-23, 0x1.3b31997e71951p-23, 0x1.3b3197fa5e7d0p-23,
    0x1.364e9f9636a39p-23, 0x1.364e9e1e14222p-23, 0x1.317f0ab18a7dap-23, 0x1.317f0944fa884p-23,
    0x1.2cc28dd6ba621p-23, 0x1.2cc28c7561d2dp-23, 0x1.2818dd3d95b3ap-23, 0x1.2818dbe71c32ap-23,
    0x1.2381ae4ab1706p-23, 0x1.2381acfec15d7p-23, 0x1.1efcb78abe751p-23, 0x1.1efcb64904d27p-23,
    0x1.1a89b0adf242ap-23, 0x1.1a89af761ea04p-23, 0x1.1628528381fc2p-23, 0x1.1628515546636p-23,
    0x1.11d856f52f545p-23, 0x1.11d855d04034dp-23, 0x1.0d997902e724ap-23, 0x1.0d9977e6fb411p-23,
    0x1.096b74be71667p-23, 0x1.096b73ab41c26p-23, 0x1.054e0747324abp-23, 0x1.054e063c7a18cp-23,
    0x1.0140eec5fc2a6p-23, 0x1.0140edc378bb3p-23, 0x1.fa87d4d1e41eap-24, 0x1.fa87d2dcc5813p-24,
    0x1.f2ad74bef5217p-24, 0x1.f2ad72d9417acp-24, 0x1.eaf23fac858a1p-24, 0x1.eaf23dd5c36acp-24,
    0x1.e355b9e6a20f7p-24, 0x1.e355b81e5bc48p-24, 0x1.dbd769a44ea9ep-24, 0x1.dbd767ea121f5p-24,
    0x1.d476d6ffe9f9bp-24, 0x1.d476d553489e1p-24, 0x1.cd338befaee3ep-24, 0x1.cd338a503d8cap-24,
    0x1.c60d143e53ec8p-24, 0x1.c60d12abaabb3p-24, 0x1.bf02fd83c7d93p-24, 0x1.bf02fbfd82216p-24,
    0x1.b814d71e0b271p-24, 0x1.b814d5a3c7555p-24, 0x1.b142322a25e1fp-24, 0x1.b14230bb85635p-24,
    0x1.aa8aa17d396c0p-24, 0x1.aa8aa019e0968p-24, 0x1.a3edb99dadc7cp-24, 0x1.a3edb84543c34p-24,
    0x1.9d6b10bc79f58p-24, 0x1.9d6b0f6ea8a5ep-24, 0x1.97023eae86fb3p-24, 0x1.97023d6afaea3p-24,
    0x1.90b2dce62d2a1p-24, 0x1.90b2dbac95731p-24, 0x1.8a7c866ccb3ccp-24, 0x1.8a7c853cd9783p-24,
    0x1.845ed7dc76e4ap-24, 0x1.845ed6b5df148p-24, 0x1.7e596f59c6640p-24, 0x1.7e596e3c3ee0cp-24,
    0x1.786bec8db2cf4p-24, 0x1.786beb78f4359p-24, 0x1.7295f09f92950p-24, 0x1.7295ef9357b3dp-24,
    0x1.6cd71e2f2bec2p-24, 0x1.6cd71d2b31b34p-24, 0x1.672f194edec88p-24, 0x1.672f1852e4382p-24,
    0x1.619d877de5fa0p-24, 0x1.619d8689ac122p-24, 0x1.5c220fa2af18dp-24, 0x1.5c220eb5f8c9cp-24,
    0x1.56bc5a0548e56p-24, 0x1.56bc591fdb004p-24, 0x1.516c1049e7c23p-24, 0x1.516c0f6b88ea5p-24,
    0x1.4c30dd6b7ff04p-24, 0x1.4c30dc93f88cdp-24, 0x1.470a6db67537cp-24, 0x1.470a6ce58f65cp-24,
    0x1.41f86ec35fa79p-24, 0x1.41f86df8e72c7p-24, 0x1.3cfa8f71e517ep-24, 0x1.3cfa8eada7548p-24,
    0x1.38107fe3a71ecp-24, 0x1.38107f257302ap-24, 0x1.3339f17745233p-24, 0x1.3339f0beeb206p-24,
    0x1.2e7696c372415p-24, 0x1.2e769610c4404p-24, 0x1.29c623921eaf1p-24, 0x1.29c622e4f0036p-24,
    0x1.25284cdbb4556p-24, 0x1.25284c33d9b27p-24, 0x1.209cc8c266508p-24, 0x1.209cc81fb5beep-24,
    0x1.1c234e8d930dcp-24, 0x1.1c234defe3e06p-24, 0x1.17bb96a538bb1p-24, 0x1.17bb960c63856p-24,
    0x1.13655a8d7bc18p-24, 0x1.136559f95a4d6p-24, 0x1.0f2054e23f01dp-24, 0x1.0f205452ac462p-24,
    0x1.0aec4152cd8cfp-24, 0x1.0aec40c7a5a44p-24, 0x1.06c8dc9d95937p-24, 0x1.06c8dc16b5b31p-24,
    0x1.02b5e48bf446bp-24, 0x1.02b5e4093ab5fp-24, 0x1.fd662fdc24d35p-25, 0x1.fd662edebcf2ep-25,
    0x1.f5806d2da29c3p-25, 0x1.f5806c3806a19p-25, 0x1.edba02af8ffacp-25, 0x1.edba01c1827dbp-25,
    0x1.e61273faa09a3p-25, 0x1.e6127313e6160p-25, 0x1.de894695473ecp-25, 0x1.de8945b5a603cp-25,
    0x1.d71e01ec0e23bp-25, 0x1.d71e01134e484p-25, 0x1.cfd02f4a0db98p-25, 0x1.cfd02e77f90cbp-25,
    0x1.c89f59d1814e8p-25, 0x1.c89f5905e34a0p-25, 0x1.c18b0e747928dp-25, 0x1.c18b0daf1ee3fp-25,
    0x1.ba92dbeda99dfp-25, 0x1.ba92db2e61c13p-25, 0x1.b3b652b956b54p-25, 0x1.b3b651fff16dbp-25,
    0x1.acf5050e5be30p-25, 0x1.acf5045aaad65p-25, 0x1.a64e86d74f6d4p-25, 0x1.a64e862925ae4p-25,
    0x1.9fc26dabc10c7p-25, 0x1.9fc26d02f30fdp-25, 0x1.995050c9935bfp-25, 0x1.99505025f6ed4p-25,
    0x1.92f7c90e6faf6p-25, 0x1.92f7c86fdbe6bp-25, 0x1.8cb870f153e55p-25, 0x1.8cb87057a11cep-25,
    0x1.8691e47c39ceap-25, 0x1.8691e3e74198fp-25, 0x1.8083c145d7c60p-25, 0x1.8083c0b574e44p-25,
    0x1.7a8da66b7a137p-25, 0x1.7a8da5df886c2p-25, 0x1.74af348af4b94p-25, 0x1.74af3403514f4p-25,
    0x1.6ee80dbcad496p-25, 0x1.6ee80d3936331p-25, 0x1.6937d58dbc641p-25, 0x1.6937d50e50c31p-25,
    0x1.639e30fa26825p-25, 0x1.639e307ea67b0p-25, 0x1.5e1ac6672bae3p-25, 0x1.5e1ac5ef785ffp-25,
    0x1.58ad3d9dadd01p-25, 0x1.58ad3d29a94d7p-25, 0x1.53553fc4ad352p-25, 0x1.53553f543a7c6p-25,
    0x1.4e12775bdaf8bp-25, 0x1.4e1276eeddecap-25, 0x1.48e4903640f82p-25, 0x1.48e48fcc9e58dp-25,
    0x1.43cb3774fefc9p-25, 0x1.43cb370e9c60dp-25, 0x1.3ec61b821cc65p-25, 0x1.3ec61b1ee094fp-25,
    0x1.39d4ec0b70a68p-25, 0x1.39d4ebab42100p-25, 0x1.34f759fd9a563p-25, 0x1.34f759a0614e6p-25,
    0x1.302d177f11b9ap-25, 0x1.302d1724b6f1cp-25, 0x1.2b75d7eb49417p-25, 0x1.2b75d793b6226p-25,
    0x1.26d14fcde39bep-25, 0x1.26d14f7902405p-25, 0x1.223f34ddfc684p-25, 0x1.223f348bb7977p-25,
    0x1.1dbf3df983a31p-25, 0x1.1dbf3da9c6cb6p-25, 0x1.19512320ab7edp-25, 0x1.195122d362b0bp-25,
    0x1.14f49d7168616p-25, 0x1.14f49d26804a2p-25, 0x1.10a9672302bd5p-25, 0x1.10a966da68a29p-25,
    0x1.0c6f3b81ba80fp-25, 0x1.0c6f3b3b5c3bcp-25, 0x1.0845d6ea7bd46p-25, 0x1.0845d6a647ccep-25,
    0x1.042cf6c6a4e33p-25, 0x1.042cf6848a0bfp-25, 0x1.00245987dc6c6p-25, 0x1.00245947ca3e5p-25,
    0x1.f8577d47f1af8p-26, 0x1.f8577ccbbe9c3p-26, 0x1.f085cd21ef1c2p-26, 0x1.f085cca98e442p-26,
    0x1.e8d3258208a6cp-26, 0x1.e8d3250d5bf13p-26, 0x1.e13f0b3d20c9dp-26, 0x1.e13f0acc0b0afp-26,
    0x1.d9c90510f2360p-26, 0x1.d9c904a35727cp-26, 0x1.d2709b9c7ba3dp-26, 0x1.d2709b323fdeep-26,
    0x1.cb35595889ba0p-26, 0x1.cb3558f192aeep-26, 0x1.c416ca905e908p-26, 0x1.c416ca2c9280ep-26,
    0x1.bd147d5a765b2p-26, 0x1.bd147cf9bc538p-26, 0x1.b62e019168c80p-26, 0x1.b62e0133a8996p-26,
    0x1.af62e8cce69ffp-26, 0x1.af62e87208d9bp-26, 0x1.a8b2c65ad3382p-26, 0x1.a8b2c602c1227p-26,
    0x1.a21d2f387947cp-26, 0x1.a21d2ee31cddap-26, 0x1.9ba1ba0bdab3cp-26, 0x1.9ba1b9b91e9dap-26,
    0x1.953fff1d1ae64p-26, 0x1.953ffeccea74ap-26, 0x1.8ef7985003483p-26, 0x1.8ef798024a6e9p-26,
    0x1.88c8211da175bp-26, 0x1.88c820d24cc58p-26, 0x1.82b1368dfec6ap-26, 0x1.82b13644fb6a4p-26,
    0x1.7cb27731f0c6ep-26, 0x1.7cb276eb2c7d2p-26, 0x1.76cb831d023bep-26, 0x1.76cb82d86b535p-26,
    0x1.70fbfbdf74555p-26, 0x1.70fbfb9cf9a7ep-26, 0x1.6b43848057a97p-26, 0x1.6b43843fe8980p-26,
    0x1.65a1c177bc9e7p-26, 0x1.65a1c139490cfp-26, 0x1.601658a8fae3ep-26, 0x1.6016586c73353p-26,
    0x1.5aa0f15d0fa10p-26, 0x1.5aa0f12264b2dp-26, 0x1.5541343d11fcfp-26, 0x1.5541340435244p-26,
    0x1.4ff6cb4cbda92p-26, 0x1.4ff6cb15a0ae7p-26, 0x1.4ac161e513161p-26, 0x1.4ac161afa831dp-26,
    0x1.45a0a4af0cfc1p-26, 0x1.45a0a47b46d34p-26, 0x1.4094419e6ae46p-26, 0x1.4094416c3c852p-26,
    0x1.3b9be7ec905e1p-26, 0x1.3b9be7bbed3cap-26, 0x1.36b74813788e0p-26, 0x1.36b747e454815p-26,
    0x1.31e613c8bdc7bp-26, 0x1.31e6139b0d067p-26, 0x1.2d27fdf8b4e06p-26, 0x1.2d27fdcc6bfe3p-26,
    0x1.287cbac19bee6p-26, 0x1.287cba96afd8dp-26, 0x1.23e3ff6edc267p-26, 0x1.23e3ff4542224p-26,
    0x1.1f5d82745e8c1p-26, 0x1.1f5d824c0c328p-26, 0x1.1ae8fb69f32a4p-26, 0x1.1ae8fb42de669p-26,
    0x1.16862306ca8a7p-26, 0x1.168622e0e9973p-26, 0x1.1234b31d01219p-26, 0x1.1234b2f84a865p-26,
    0x1.0df466953c6c2p-26, 0x1.0df46671a6fb0p-26, 0x1.09c4f96a5972dp-26, 0x1.09c4f947dc465p-26,
    0x1.05a628a52c72bp-26, 0x1.05a62883beeb6p-26, 0x1.0197b25851650p-26, 0x1.0197b237eb274p-26,
    0x1.fb32ab381a46dp-27, 0x1.fb32aaf94c2b1p-27, 0x1.f355a5147dcdcp-27, 0x1.f355a4d79e5dep-27,
    0x1.eb97d474c3c10p-27, 0x1.eb97d439c3c4dp-27, 0x1.e3f8bd7b3d57cp-27, 0x1.e3f8bd420e0efp-27,
    0x1.dc77e635d8b92p-27, 0x1.dc77e5fe6bd7ap-27, 0x1.d514d69681d11p-27, 0x1.d514d660c97b5p-27,
    0x1.cdcf186ba1650p-27, 0x1.cdcf1837902cbp-27, 0x1.c6a63758b9f0dp-27, 0x1.c6a6372642d15p-27,
    0x1.bf99c0cf21d52p-27, 0x1.bf99c09e38307p-27, 0x1.b8a94406da638p-27, 0x1.b8a943d771feep-27,
    0x1.b1d451f78354fp-27, 0x1.b1d451c990562p-27, 0x1.ab1a7d516a3aep-27, 0x1.ab1a7d24e124ep-27,
    0x1.a47b5a76b57b0p-27, 0x1.a47b5a4b8b2b4p-27, 0x1.9df67f74aa689p-27, 0x1.9df67f4ad4145p-27,
    0x1.978b83fd0e101p-27, 0x1.978b83d481418p-27, 0x1.913a015fa04afp-27, 0x1.913a013852deap-27,
    0x1.8b019283b0b32p-27, 0x1.8b01925d98d58p-27, 0x1.84e1d3e1cd0f6p-27, 0x1.84e1d3bce13a5p-27,
    0x1.7eda637d88d46p-27, 0x1.7eda6359bfccbp-27, 0x1.78eae0df5d555p-27, 0x1.78eae0bcae28ap-27,
    0x1.7312ed0ea243fp-27, 0x1.7312eced04463p-27, 0x1.6d522a8b9e1ddp-27, 0x1.6d522a6b08e76p-27,
    0x1.67a83d49ae294p-27, 0x1.67a83d2a1994ap-27, 0x1.6214caa985a35p-27, 0x1.6214ca8ae9cb3p-27,
    0x1.5c97797383c3ap-27, 0x1.5c977955d900ep-27, 0x1.572ff1d2203afp-27, 0x1.572ff1b55f22cp-27,
    0x1.51dddd4c6dd36p-27, 0x1.51dddd308f355p-27, 0x1.4ca0e6c0b2da3p-27, 0x1.4ca0e6a5afbe8p-27,
    0x1.4778ba5f16fd9p-27, 0x1.4778ba44e8a34p-27, 0x1.426505a466479p-27, 0x1.4265058b0622fp-27,
    0x1.3d657754e8e4ap-27, 0x1.3d65773c509d9p-27, 0x1.3879bf774f610p-27, 0x1.3879bf5f78d13p-27,
    0x1.33a18f4fb30d2p-27, 0x1.33a18f38983efp-27, 0x1.2edc995aaa38fp-27, 0x1.2edc994445657p-27,
    0x1.2a2a91486ff6ap-27, 0x1.2a2a9132bb848p-27, 0x1.258b2bf81f180p-27, 0x1.258b2be3159a2p-27,
    0x1.20fe1f73001a3p-27, 0x1.20fe1f5e9c4e0p-27, 0x1.1c8322e7e9b3cp-27, 0x1.1c8322d426803p-27,
    0x1.1819eea6b3bc1p-27, 0x1.1819ee938c304p-27, 0x1.13c23c1bbc231p-27, 0x1.13c23c092b751p-27,
    0x1.0f7bc5cb7db14p-27, 0x1.0f7bc5b97f3cbp-27, 0x1.0b46474e38496p-27, 0x1.0b46473cc78eap-27,
    0x1.07217d4baa66fp-27, 0x1.07217d3ac309bp-27, 0x1.030d2576db948p-27, 0x1.030d2566795aep-27,
    0x1.fe11fd13ef2d3p-28, 0x1.fe11fcf42ccfcp-28, 0x1.f629908474122p-28, 0x1.f6299065abd9dp-28,
    0x1.ee6086b7d45b0p-28, 0x1.ee608699fe95ap-28, 0x1.e6b6631ccd54cp-28, 0x1.e6b662ffe28cbp-28,
    0x1.df2aab1081f7dp-28, 0x1.df2aaaf47af23p-28, 0x1.d7bce5d6d0afbp-28, 0x1.d7bce5bba66abp-28,
    0x1.d06c9c92c78f6p-28, 0x1.d06c9c7873403p-28, 0x1.c9395a3f3677fp-28, 0x1.c9395a25b1896p-28,
    0x1.c222aba75ebc0p-28, 0x1.c222ab8ea2cccp-28, 0x1.bb281f5fbfca5p-28, 0x1.bb281f47c6ab4p-28,
    0x1.b44945bf006c1p-28, 0x1.b44945a7c41ecp-28, 0x1.ad85b0d6f4265p-28, 0x1.ad85b0c06edb9p-28,
    0x1.a6dcf46dbc4dep-28, 0x1.a6dcf457e8644p-28, 0x1.a04ea5f704609p-28, 0x1.a04ea5e1dc62fp-28,
    0x1.99da5c8d5936ep-28, 0x1.99da5c78d7db3p-28, 0x1.937fb0eb9aa46p-28, 0x1.937fb0d7baca2p-28,
    0x1.8d3e3d66871ccp-28, 0x1.8d3e3d5343cc0p-28, 0x1.87159de660f7bp-28, 0x1.87159dd3b55f6p-28,
    0x1.81056fe0acec4p-28, 0x1.81056fce94617p-28, 0x1.7b0d525209617p-28, 0x1.7b0d52407f5ddp-28,
    0x1.752ce5b81e2f9p-28, 0x1.752ce5a71e50ap-28, 0x1.6f63cc0ba4734p-28, 0x1.6f63cbfb2a78fp-28,
    0x1.69b1a8ba8610fp-28, 0x1.69b1a8aa8ddcap-28, 0x1.641620a2148bdp-28, 0x1.641620929a1f7p-28,
    0x1.5e90da0956d39p-28, 0x1.5e90d9fa56506p-28, 0x1.59217c9b6dacfp-28, 0x1.59217c8ce352cp-28,
    0x1.53c7b1620e5cep-28, 0x1.53c7b153f6890p-28, 0x1.4e8322c0133c7p-28, 0x1.4e8322b26a68ep-28,
    0x1.49537c6c21df3p-28, 0x1.49537c5ee4a1bp-28, 0x1.44386b6b6676ep-28, 0x1.44386b5e91800p-28,
    0x1.3f319e0c641f0p-28, 0x1.3f319dfff4397p-28, 0x1.3a3ec3e1d9be6p-28, 0x1.3a3ec3d5cbce2p-28,
    0x1.355f8dbdbb2c5p-28, 0x1.355f8db20c2ddp-28, 0x1.3093adac3e494p-28, 0x1.3093ada0eb50cp-28,
    0x1.2bdad6eefbbbep-28, 0x1.2bdad6e401f48p-28, 0x1.2734bdf82303ep-28, 0x1.2734bded7faf2p-28,
    0x1.22a11865c1971p-28, 0x1.22a1185b720c1p-28, 0x1.1e1f9cfd1cbbap-28, 0x1.1e1f9cf31e667p-28,
    0x1.19b003a61dd6cp-28, 0x1.19b0039c6e37bp-28, 0x1.15520566d0e4ep-28, 0x1.1552055d6d901p-28,
    0x1.11055c5ef4d4dp-28, 0x1.11055c55db716p-28, 0x1.0cc9c3c39d7ddp-28, 0x1.0cc9c3bacbc54p-28,
    0x1.089ef7dae6eadp-28, 0x1.089ef7d25aa8cp-28, 0x1.0484b5f7b9b71p-28, 0x1.0484b5ef70c86p-28,
    0x1.007abc75a0369p-28, 0x1.007abc6d9888fp-28, 0x1.f901956958537p-29, 0x1.f9019559c7767p-29,
    0x1.f12d422ad9719p-29, 0x1.f12d421bc32e8p-29, 0x1.e97801e9e8ef5p-29, 0x1.e97801db49809p-29,
    0x1.e1e15951de63ap-29, 0x1.e1e15943b2214p-29, 0x1.da68cef78e7fap-29, 0x1.da68cee9d1de7p-29,
    0x1.d30deb51b4521p-29, 0x1.d30deb4463e2fp-29, 0x1.cbd038b178a90p-29, 0x1.cbd038a49117bp-29,
    0x1.c4af433b171a9p-29, 0x1.c4af432e952d1p-29, 0x1.bdaa98dea03edp-29, 0x1.bdaa98d280d4ap-29,
    0x1.b6c1c950d8a7bp-29, 0x1.b6c1c94518b8fp-29, 0x1.aff466043423ap-29, 0x1.aff465f8d0c04p-29,
    0x1.a9420221ecdbep-29, 0x1.a9420216e32afp-29, 0x1.a2aa328335dedp-29, 0x1.a2aa3278831ddp-29,
    0x1.9c2c8daa88aa5p-29, 0x1.9c2c8da02a2c9p-29, 0x1.95c8abbd0d4acp-29, 0x1.95c8abb300789p-29,
    0x1.8f7e267c1ca49p-29, 0x1.8f7e26725efabp-29, 0x1.894c993edc819p-29, 0x1.894c99356b907p-29,
    0x1.8333a0ebf4fabp-29, 0x1.8333a0e2ce662p-29, 0x1.7d32dbf35eda7p-29, 0x1.7d32dbea8058cp-29,
    0x1.7749ea484a945p-29, 0x1.7749ea3fb1edcp-29, 0x1.71786d5b1f6fbp-29, 0x1.71786d52ca7e2p-29,
    0x1.6bbe08139286ap-29, 0x1.6bbe080b7f34cp-29, 0x1.661a5ecad5393p-29, 0x1.661a5ec301822p-29,
    0x1.608d1745dab93p-29, 0x1.608d173e44a80p-29, 0x1.5b15d8afb451bp-29, 0x1.5b15d8a85a00cp-29,
    0x1.55b44b9404109p-29, 0x1.55b44b8ce3a95p-29, 0x1.506819d98579cp-29, 0x1.506819d29d340p-29,
    0x1.4b30eebcabeb7p-29, 0x1.4b30eeb5fa0d3p-29, 0x1.460e76ca565e8p-29, 0x1.460e76c3d93b2p-29,
    0x1.41005fda982d2p-29, 0x1.41005fd44e256p-29, 0x1.3c06590b968dap-29, 0x1.3c0659057e0efp-29,
    0x1.372012bc7a6dcp-29, 0x1.372012b691f1fp-29, 0x1.324d3e88765e9p-29, 0x1.324d3e82bc6b9p-29,
    0x1.2d8d8f41e0417p-29, 0x1.2d8d8f3c5368bp-29, 0x1.28e0b8ed5e668p-29, 0x1.28e0b8e7fd44cp-29,
    0x1.244670bd27d14p-29, 0x1.244670b7f10e2p-29, 0x1.1fbe6d0c57553p-29, 0x1.1fbe6d0749a31p-29,
    0x1.1b48655a5141ep-29, 0x1.1b4865556b5d5p-29, 0x1.16e412463b52ep-29, 0x1.16e412417c025p-29,
    0x1.12912d8a869c4p-29, 0x1.12912d85ecafep-29, 0x1.0e4f71f88b2bep-29, 0x1.0e4f71f4157d3p-29,
    0x1.0a1e9b743518fp-29, 0x1.0a1e9b6fe28a7p-29, 0x1.05fe66efc2bd4p-29, 0x1.05fe66eb923a5p-29,
    0x1.01ee926793d38p-29, 0x1.01ee926384500p-29, 0x1.fbddb9bc126f8p-30, 0x1.fbddb9b4335f8p-30,
    0x1.f3fe0caeea100p-30, 0x1.f3fe0ca748ff4p-30, 0x1.ec3d9fac35c82p-30, 0x1.ec3d9fa4d0ce5p-30,
    0x1.e49bf6ac80194p-30, 0x1.e49bf6a5555d0p-30, 0x1.dd18979496445p-30, 0x1.dd18978da3fb1p-30,
    0x1.d5b30a2de68d4p-30, 0x1.d5b30a272afa4p-30, 0x1.ce6ad81efcc71p-30, 0x1.ce6ad818763b7p-30,
    0x1.c73f8ce41cb35p-30, 0x1.c73f8cddc98d6p-30, 0x1.c030b5c7f9bc6p-30, 0x1.c030b5c1d8675p-30,
    0x1.b93de1dc8b972p-30, 0x1.b93de1d69a8aap-30, 0x1.b266a1f3ff593p-30, 0x1.b266a1ee3d18fp-30,
    0x1.abaa8899c4924p-30, 0x1.abaa88942fad9p-30, 0x1.a5092a0bb5fa0p-30, 0x1.a5092a064d0bcp-30,
    0x1.9e821c335d450p-30, 0x1.9e821c2e1ef2dp-30, 0x1.9814f69f51b44p-30, 0x1.9814f69a3cae9p-30,
    0x1.91c1527cb0f5fp-30, 0x1.91c15277c3f78p-30, 0x1.8b86ca90b1ef0p-30, 0x1.8b86ca8bebbc8p-30,
    0x1.8564fb325105cp-30, 0x1.8564fb2db06dbp-30, 0x1.7f5b82441589bp-30, 0x1.7f5b823f9963dp-30,
    0x1.7969ff2defd39p-30, 0x1.7969ff299700dp-30, 0x1.739012d72fbc7p-30, 0x1.739012d2f926ap-30,
    0x1.6dcd5fa0930adp-30, 0x1.6dcd5f9c7da45p-30, 0x1.6821895e6b76ap-30, 0x1.6821895a7639fp-30,
    0x1.628c3552dbe69p-30, 0x1.628c354f05d67p-30, 0x1.5d0d0a282c8afp-30, 0x1.5d0d0a2474b1dp-30,
    0x1.57a3afeb357aap-30, 0x1.57a3afe79aea9p-30, 0x1.524fd005df794p-30, 0x1.524fd002614b9p-30,
    0x1.4d111539ba8e9p-30, 0x1.4d11153657e3bp-30, 0x1.47e72b9aaa185p-30, 0x1.47e72b9762178p-30,
    0x1.42d1c089a6015p-30, 0x1.42d1c08677d8ap-30, 0x1.3dd082af90ca7p-30, 0x1.3dd082ac7bae5p-30,
    0x1.38e321f82211ap-30, 0x1.38e321f5253cdp-30, 0x1.34094f8ce546fp-30, 0x1.34094f89fffa2p-30,
    0x1.2f42bdd04c3e9p-30, 0x1.2f42bdcd7dc07p-30, 0x1.2a8f2058d5519p-30, 0x1.2a8f20561cee8p-30,
    0x1.25ee2bec44bf3p-30, 0x1.25ee2be9a1c91p-30, 0x1.215f967af1035p-30, 0x1.215f967862d16p-30,
    0x1.1ce3171b21d54p-30, 0x1.1ce31718a7c3fp-30, 0x1.1878660481865p-30, 0x1.187866021af72p-30,
    0x1.141f3c8ba0768p-30, 0x1.141f3c894ccfcp-30, 0x1.0fd7551d8a57bp-30, 0x1.0fd7551b49047p-30,
    0x1.0ba06b3b6cf87p-30, 0x1.0ba06b393d686p-30, 0x1.077a3b7650513p-30, 0x1.077a3b7431f87p-30,
    0x1.0364836adf8f5p-30, 0x1.03648368d1e64p-30, 0x1.febe037a85b3fp-31, 0x1.febe03768aba5p-31,
    0x1.f6d2ec2a131eep-31, 0x1.f6d2ec26377f0p-31, 0x1.ef07423249713p-31, 0x1.ef07422e8c341p-31,
    0x1.e75a88d7e2e56p-31, 0x1.e75a88d4431bdp-31, 0x1.dfcc454ea6203p-31, 0x1.dfcc454b22e22p-31,
    0x1.d85bfeb1b9629p-31, 0x1.d85bfeae51cf3p-31, 0x1.d1093dfc1431fp-31, 0x1.d1093df8c76f5p-31,
    0x1.c9d38e010efe0p-31, 0x1.c9d38dfddc390p-31, 0x1.c2ba7b65104c5p-31, 0x1.c2ba7b61f6b83p-31,
    0x1.bbbd949656f52p-31, 0x1.bbbd949355cb7p-31, 0x1.b4dc69c5e0fdfp-31, 0x1.b4dc69c2f77e7p-31,
    0x1.ae168ce06e9ffp-31, 0x1.ae168cdd9c103p-31, 0x1.a76b9187a10adp-31, 0x1.a76b9184e4b63p-31,
    0x1.a0db0d0b34762p-31, 0x1.a0db0d088dad7p-31, 0x1.9a6496625513ap-31, 0x1.9a64965fc32d5p-31,
    0x1.9407c6250e79fp-31, 0x1.9407c62290d16p-31, 0x1.8dc43685d51c0p-31, 0x1.8dc436836b11dp-31,
    0x1.8799834b29686p-31, 0x1.87998348d2621p-31, 0x1.818749c95428bp-31, 0x1.818749c70f908p-31,
    0x1.7b8d28dc3bbe0p-31, 0x1.7b8d28da0902cp-31, 0x1.75aac0e151d72p-31, 0x1.75aac0df306c2p-31,
    0x1.6fdfb3b1993fdp-31, 0x1.6fdfb3af889cap-31, 0x1.6a2ba49bc368ep-31, 0x1.6a2ba499c3097p-31,
    0x1.648e385e654bfp-31, 0x1.648e385c74b01p-31, 0x1.5f071522434ccp-31, 0x1.5f07152061f85p-31,
    0x1.5995e274b3be3p-31, 0x1.5995e272e138ep-31, 0x1.543a494217b05p-31, 0x1.543a494053857p-31,
    0x1.4ef3f3d069aefp-31, 0x1.4ef3f3ceb36d8p-31, 0x1.49c28db9e21aap-31, 0x1.49c28db83954fp-31,
    0x1.44a5c3e7b0c48p-31, 0x1.44a5c3e615108p-31, 0x1.3f9d448ccb7b0p-31, 0x1.3f9d448b3c71bp-31,
    0x1.3aa8bf20d1320p-31, 0x1.3aa8bf1f4e6fap-31, 0x1.35c7e45b01762p-31, 0x1.35c7e4598a9a0p-31,
    0x1.30fa662d47da3p-31, 0x1.30fa662bdc869p-31, 0x1.2c3ff7bf5b0f5p-31, 0x1.2c3ff7bdfae96p-31,
    0x1.27984d69ef5a2p-31, 0x1.27984d689a09cp-31, 0x1.23031cb1fc177p-31, 0x1.23031cb0b1476p-31,
    0x1.1e801c441405ep-31, 0x1.1e801c42d3636p-31, 0x1.1a0f03efd0087p-31, 0x1.1a0f03ee99436p-31,
    0x1.15af8ca34c1aap-31, 0x1.15af8ca21ee54p-31, 0x1.11617066b62bdp-31, 0x1.11617065923aep-31,
    0x1.0d246a57ee9c8p-31, 0x1.0d246a56d3a6fp-31, 0x1.08f836a63a169p-31, 0x1.08f836a527d5bp-31,
    0x1.04dc928e047bcp-31, 0x1.04dc928cfaab0p-31, 0x1.00d13c54b4a74p-31, 0x1.00d13c53b3042p-31,
    0x1.f9abe689217c4p-32, 0x1.f9abe6872e107p-32, 0x1.f1d4ef51659d8p-32, 0x1.f1d4ef4f818f4p-32,
    0x1.ea1d15921af9bp-32, 0x1.ea1d159045d01p-32, 0x1.e283ddcd00f74p-32, 0x1.e283ddcb3a3cdp-32,
    0x1.db08ce6df92cdp-32, 0x1.db08ce6c406ffp-32, 0x1.d3ab6fc36e15ap-32, 0x1.d3ab6fc1c2e82p-32,
    0x1.cc6b4bf6d7edfp-32, 0x1.cc6b4bf539e51p-32, 0x1.c547ef055f40fp-32, 0x1.c547ef03cdf52p-32,
    0x1.be40e6b89cb16p-32, 0x1.be40e6b717be5p-32, 0x1.b755c29f7589cp-32, 0x1.b755c29dfc8e2p-32,
    0x1.b086140714a13p-32, 0x1.b0861405a73ecp-32, 0x1.a9d16df3ff24ep-32, 0x1.a9d16df29d006p-32,
    0x1.a337651b44d7ap-32, 0x1.a3376519ed987p-32, 0x1.9cb78fdbcb595p-32, 0x1.9cb78fda7ea9ap-32,
    0x1.96518637b40d0p-32, 0x1.965186367199bp-32, 0x1.9004e1cddc321p-32, 0x1.9004e1cca3aa7p-32,
    0x1.89d13dd376c99p-32, 0x1.89d13dd247df8p-32, 0x1.83b6370dbfe0fp-32, 0x1.83b6370c9a48cp-32,
    0x1.7db36bcbc8dddp-32, 0x1.7db36bcaac4e1p-32, 0x1.77c87be05d667p-32, 0x1.77c87bdf49980p-32,
    0x1.71f5089c0086fp-32, 0x1.71f5089af534cp-32, 0x1.6c38b4c701b12p-32, 0x1.6c38b4c5fe987p-32,
    0x1.6693249ba93a1p-32, 0x1.6693249aae1a2p-32, 0x1.6103fdc07bf6ep-32, 0x1.6103fdbf8890ep-32,
    0x1.5b8ae742959d4p-32, 0x1.5b8ae741a9b45p-32, 0x1.56278990198e2p-32, 0x1.5627898f34e74p-32,
    0x1.50d98e72b9b06p-32, 0x1.50d98e71dc128p-32, 0x1.4ba0a10a5304ep-32, 0x1.4ba0a1097c388p-32,
    0x1.467c6dc79f9d2p-32, 0x1.467c6dc6cf6c9p-32, 0x1.416ca266fd9ffp-32, 0x1.416ca26633d72p-32,
    0x1.3c70edeb4b089p-32, 0x1.3c70edea87751p-32, 0x1.37890098d5cddp-32, 0x1.37890098183ecp-32,
    0x1.32b48bf060201p-32, 0x1.32b48befa8660p-32, 0x1.2df342aa386f3p-32, 0x1.2df342a9865c4p-32,
    0x1.2944d8b164e8cp-32, 0x1.2944d8b0b8506p-32, 0x1.24a9031ee2224p-32, 0x1.24a9031e3ad94p-32,
    0x1.201f7834f4a26p-32, 0x1.201f7834527efp-32, 0x1.1ba7ef5a8cff9p-32, 0x1.1ba7ef59efd93p-32,
    0x1.17422116be48ap-32, 0x1.1742211625f81p-32, 0x1.12edc70c46703p-32, 0x1.12edc70bb2cf5p-32,
    0x1.0eaa9bf52872bp-32, 0x1.0eaa9bf4995c8p-32, 0x1.0a785b9e57f08p-32, 0x1.0a785b9dcd415p-32,
    0x1.0656c2e375f7fp-32, 0x1.0656c2e2ef8d2p-32, 0x1.02458faa9eb98p-32, 0x1.02458faa1c716p-32,
    0x1.fc8901c08fc7fp-33, 0x1.fc8901bf933bfp-33, 0x1.f4a6ace65ecd4p-33, 0x1.f4a6ace56a066p-33,
    0x1.ece3a2a0b4af4p-33, 0x1.ece3a29fc7705p-33, 0x1.e53f66be477e3p-33, 0x1.e53f66bd618bep-33,
    0x1.ddb97efab60f4p-33, 0x1.ddb97ef9d7301p-33, 0x1.d65172f6e3ac7p-33, 0x1.d65172f60ba8ap-33,
    0x1.cf06cc3172187p-33, 0x1.cf06cc30a0ba1p-33, 0x1.c7d915ff596f4p-33, 0x1.c7d915fe8e81fp-33,
    0x1.c0c7dd849d6bcp-33, 0x1.c0c7dd83d8bcbp-33, 0x1.b9d2b1ad1f9e3p-33, 0x1.b9d2b1ac60fc5p-33,
    0x1.b2f923258e216p-33, 0x1.b2f92324d55cfp-33, 0x1.ac3ac4546e5bbp-33, 0x1.ac3ac453bb469p-33,
    0x1.a5972953435ebp-33, 0x1.a597295295cc1p-33, 0x1.9f0de7e7cf764p-33, 0x1.9f0de7e7273abp-33,
    0x1.989e977d707bap-33, 0x1.989e977ccd6d2p-33, 0x1.9248d11e9682fp-33, 0x1.9248d11df878cp-33,
    0x1.8c0c2f6e54795p-33, 0x1.8c0c2f6dbb4bep-33, 0x1.85e84ea20a4ddp-33, 0x1.85e84ea175d6dp-33,
    0x1.7fdccc7b283efp-33, 0x1.7fdccc7a98596p-33, 0x1.79e948410ae9cp-33, 0x1.79e948407f719p-33,
    0x1.740d62baefb74p-33, 0x1.740d62ba68898p-33, 0x1.6e48be2a01488p-33, 0x1.6e48be297e437p-33,
    0x1.689afe437b815p-33, 0x1.689afe42fc844p-33, 0x1.6303c82ae6d4ap-33, 0x1.6303c82a6bbfcp-33,
    0x1.5d82c26c6a751p-33, 0x1.5d82c26bf329ap-33, 0x1.581794f735104p-33, 0x1.581794f6c1706p-33,
    0x1.52c1e917fbba1p-33, 0x1.52c1e9178ba8ep-33, 0x1.4d8169738eb11p-33, 0x1.4d81697322129p-33,
    0x1.4855c20183a43p-33, 0x1.4855c2011a5d4p-33, 0x1.433ea006f5255p-33, 0x1.433ea0068f1b8p-33,
    0x1.3e3bb21156f3ap-33, 0x1.3e3bb210f40d8p-33, 0x1.394ca7f15ecc7p-33, 0x1.394ca7f0fef15p-33,
    0x1.347132b6016fdp-33, 0x1.347132b5a487bp-33, 0x1.2fa904a783892p-33, 0x1.2fa904a7297ccp-33,
    0x1.2af3d1429e2d0p-33, 0x1.2af3d14246e5ep-33, 0x1.26514d33b69e7p-33, 0x1.26514d336206cp-33,
    0x1.21c12e52290efp-33, 0x1.21c12e51d7118p-33, 0x1.1d432b9ba60e1p-33, 0x1.1d432b9b56967p-33,
    0x1.18d6fd2fa25e5p-33, 0x1.18d6fd2f55589p-33, 0x1.147c5c4ad8e68p-33, 0x1.147c5c4a8e3f6p-33,
    0x1.10330342de778p-33, 0x1.10330342961c7p-33, 0x1.0bfaad81c71ffp-33, 0x1.0bfaad8180fecp-33,
    0x1.07d31781dcc76p-33, 0x1.07d3178198ce8p-33, 0x1.03bbfec966cd9p-33, 0x1.03bbfec924ec1p-33,
    0x1.ff6a43cd04d27p-34, 0x1.ff6a43cc851d4p-34, 0x1.f77c80d617092p-34, 0x1.f77c80d59b41dp-34,
    0x1.efae35d12bab4p-34, 0x1.efae35d0b3b2ep-34, 0x1.e7fee5d8ebe41p-34, 0x1.e7fee5d8779cap-34,
    0x1.e06e15f7b43ebp-34, 0x1.e06e15f7438b1p-34, 0x1.d8fb4d1fe5415p-34, 0x1.d8fb4d1f78055p-34,
    0x1.d1a6142452893p-34, 0x1.d1a61423e8a99p-34, 0x1.ca6df5b0cfee1p-34, 0x1.ca6df5b069506p-34,
    0x1.c3527e42dc35ap-34, 0x1.c3527e4278c02p-34, 0x1.bc533c2268e17p-34, 0x1.bc533c22087b6p-34,
    0x1.b56fbf5abea54p-34, 0x1.b56fbf5a61366p-34, 0x1.aea799b37e117p-34, 0x1.aea799b323828p-34,
    0x1.a7fa5ea9bc048p-34, 0x1.a7fa5ea9643eep-34, 0x1.a167a3693972fp-34, 0x1.a167a368e460ap-34,
    0x1.9aeefec5b61a8p-34, 0x1.9aeefec563a63p-34, 0x1.949009345db58p-34, 0x1.949009340dcaap-34,
    0x1.8e4a5cc54f44cp-34, 0x1.8e4a5cc501cf5p-34, 0x1.881d951d3e093p-34, 0x1.881d951cf2f5ep-34,
    0x1.82094f6f2bc6bp-34, 0x1.82094f6ee302ap-34, 0x1.7c0d2a763bebap-34, 0x1.7c0d2a75f564cp-34,
    0x1.7628c66f9f3b9p-34, 0x1.7628c66f5ae03p-34, 0x1.705bc5149799dp-34, 0x1.705bc5145558dp-34,
    0x1.6aa5c9949395ep-34, 0x1.6aa5c994535ebp-34, 0x1.6506788f615abp-34, 0x1.6506788f231d5p-34,
    0x1.5f7d780f78a3ep-34, 0x1.5f7d780f3c50cp-34, 0x1.5a0a6f845b5d9p-34, 0x1.5a0a6f8420e59p-34,
    0x1.54ad07bd0c956p-34, 0x1.54ad07bcd3e9ep-34, 0x1.4f64eae29d631p-34, 0x1.4f64eae26675fp-34,
    0x1.4a31c472cf72dp-34, 0x1.4a31c4729a364p-34, 0x1.4513413accd9fp-34, 0x1.4513413a9940bp-34,
    0x1.40090f51f4e2bp-34, 0x1.40090f51c2dfep-34, 0x1.3b12de14bd7b9p-34, 0x1.3b12de148d02ap-34,
    0x1.36305e1fa8f7bp-34, 0x1.36305e1f79fc9p-34, 0x1.3161414a4fd09p-34, 0x1.3161414a22477p-34,
    0x1.2ca53aa27e18ep-34, 0x1.2ca53aa251f67p-34, 0x1.27fbfe6764531p-34, 0x1.27fbfe67398c3p-34,
    0x1.23654204db5ddp-34, 0x1.23654204b1e7ep-34, 0x1.1ee0bc0ebb2bap-34, 0x1.1ee0bc0e92fc4p-34,
    0x1.1a6e243c43fa1p-34, 0x1.1a6e243c1d073p-34, 0x1.160d336399bfap-34, 0x1.160d336373ff9p-34,
    0x1.11bda37551886p-34, 0x1.11bda3752cf1ap-34, 0x1.0d7f2f7810793p-34, 0x1.0d7f2f77ed02ap-34,
    0x1.095193843c345p-34, 0x1.0951938419d51p-34, 0x1.05348cbfbc5a2p-34, 0x1.05348cbf9b09ap-34,
    0x1.0127d959cce23p-34, 0x1.0127d959ac980p-34, 0x1.fa56710dc2125p-35, 0x1.fa56710d837abp-35,
    0x1.f27cd4f92d25fp-35, 0x1.f27cd4f8f07b5p-35, 0x1.eac260db723e4p-35, 0x1.eac260db37717p-35,
    0x1.e326990caaa09p-35, 0x1.e326990c71a2ep-35, 0x1.dba903cfb70fcp-35, 0x1.dba903cf7fd2fp-35,
    0x1.d449294aa3f02p-35, 0x1.d449294a6e667p-35, 0x1.cd06937f2b9e5p-35, 0x1.cd06937ef7ba5p-35,
    0x1.c5e0ce435680fp-35, 0x1.c5e0ce432435ap-35, 0x1.bed7673a385f9p-35, 0x1.bed7673a07a06p-35,
    0x1.b7e9edccca8a6p-35, 0x1.b7e9edcc9b4b2p-35, 0x1.b117f322e2606p-35, 0x1.b117f322b4954p-35,
    0x1.aa610a1c43c37p-35, 0x1.aa610a1c17610p-35, 0x1.a3c4c749cf0b8p-35, 0x1.a3c4c749a406ap-35,
    0x1.9d42c0e6ca0bcp-35, 0x1.9d42c0e6a059bp-35, 0x1.96da8ed243bdep-35, 0x1.96da8ed21b544p-35,
    0x1.908bca88922abp-35, 0x1.908bca886aff5p-35, 0x1.8a560f1cea269p-35, 0x1.8a560f1cc42fcp-35,
    0x1.8438f933107cdp-35, 0x1.8438f932ebb10p-35, 0x1.7e3426f924233p-35, 0x1.7e3426f900793p-35,
    0x1.7847382181140p-35, 0x1.784738215e82fp-35, 0x1.7271cddcbb6bep-35, 0x1.7271cddc99eb0p-35,
    0x1.6cb38ad3b26acp-35, 0x1.6cb38ad391f1dp-35, 0x1.670c1321bafa7p-35, 0x1.670c13219b814p-35,
    0x1.617b0c4ee15c3p-35, 0x1.617b0c4ec2daep-35, 0x1.5c001d4a41a1bp-35, 0x1.5c001d4a2410ap-35,
    0x1.569aee647697ap-35, 0x1.569aee6459ef8p-35, 0x1.514b294a1ec81p-35, 0x1.514b294a0301ap-35,
    0x1.4c1078fe773cfp-35, 0x1.4c1078fe5c515p-35, 0x1.46ea89d60bad2p-35, 0x1.46ea89d5f1958p-35,
    0x1.41d909717bbdcp-35, 0x1.41d909716273ap-35, 0x1.3cdba6b85505ep-35, 0x1.3cdba6b83c82fp-35,
    0x1.37f211d4017ffp-35, 0x1.37f211d3e9be1p-35, 0x1.331bfc2aca1a6p-35, 0x1.331bfc2ab313ap-35,
    0x1.2e59185aed152p-35, 0x1.2e59185ad6c3cp-35, 0x1.29a91a35c7df5p-35, 0x1.29a91a35b23dbp-35,
    0x1.250bb6bb1426bp-35, 0x1.250bb6baff2f7p-35, 0x1.2080a41437ccfp-35, 0x1.2080a414237aep-35,
    0x1.1c07998fa7781p-35, 0x1.1c07998f93c60p-35, 0x1.17a04f9c5b736p-35, 0x1.17a04f9c485c7p-35,
    0x1.134a7fc556993p-35, 0x1.134a7fc54418ap-35, 0x1.0f05e4ad3efd3p-35, 0x1.0f05e4ad2d0e6p-35,
    0x1.0ad23a0a0810ep-35, 0x1.0ad23a09f6af4p-35, 0x1.06af3ca0adfd3p-35, 0x1.06af3ca09d247p-35,
    0x1.029caa4101ec9p-35, 0x1.029caa40f1989p-35, 0x1.fd3483830e056p-36, 0x1.fd348382ee5e9p-36,
    0x1.f54f85f6bf7e2p-36, 0x1.f54f85f6a0d0ap-36, 0x1.ed89dd8c9713fp-36, 0x1.ed89dd8c79581p-36,
    0x1.e5e30de96855fp-36, 0x1.e5e30de94b844p-36, 0x1.de5a9c9f95d53p-36, 0x1.de5a9c9f79e68p-36,
    0x1.d6f011276a404p-36, 0x1.d6f011274f2d9p-36, 0x1.cfa2f4d78fddep-36, 0x1.cfa2f4d775a06p-36,
    0x1.c872d2dda5edep-36, 0x1.c872d2dd8c7f1p-36, 0x1.c15f3836f3796p-36, 0x1.c15f3836dad2ep-36,
    0x1.ba67b3a9371d7p-36, 0x1.ba67b3a91f392p-36, 0x1.b38bd5bb935dcp-36, 0x1.b38bd5bb7c35ap-36,
    0x1.accb30af970d8p-36, 0x1.accb30af809bcp-36, 0x1.a625587a615eep-36, 0x1.a625587a4b9dep-36,
    0x1.9f99e2bde12c6p-36, 0x1.9f99e2bdcc16cp-36, 0x1.992866c22f0ecp-36, 0x1.992866c21a9f3p-36,
    0x1.92d07d6f01d5ap-36, 0x1.92d07d6eee070p-36, 0x1.8c91c1453cfa9p-36, 0x1.8c91c14529c80p-36,
    0x1.866bce5898a6dp-36, 0x1.866bce58860b7p-36, 0x1.805e424962e65p-36, 0x1.805e424950dd8p-36,
    0x1.7a68bc3e59a49p-36, 0x1.7a68bc3e4829cp-36, 0x1.748adcde9d105p-36, 0x1.748adcde8c1f3p-36,
    0x1.6ec4464bba05bp-36, 0x1.6ec4464ba99a0p-36, 0x1.69149c1bcc1f1p-36, 0x1.69149c1bbc34bp-36,
    0x1.637b8353b70f4p-36, 0x1.637b8353a7a24p-36, 0x1.5df8a26176e82p-36, 0x1.5df8a26167f4ap-36,
    0x1.588ba11686f2ap-36, 0x1.588ba1167874fp-36, 0x1.533428a25ebfap-36, 0x1.533428a250b41p-36,
    0x1.4df1e38d0517cp-36, 0x1.4df1e38cf77acp-36, 0x1.48c47db1b874cp-36, 0x1.48c47db1ab430p-36,
    0x1.43aba439acae9p-36, 0x1.43aba4399fe4bp-36, 0x1.3ea70596dd878p-36, 0x1.3ea70596d1226p-36,
    0x1.39b6517ef5c54p-36, 0x1.39b6517ee9c1cp-36, 0x1.34d938e64a84dp-36, 0x1.34d938e63edffp-36,
    0x1.300f6dfaea796p-36, 0x1.300f6dfadf303p-36, 0x1.2b58a41fc0c67p-36, 0x1.2b58a41fb5d63p-36,
    0x1.26b48fe7cb288p-36, 0x1.26b48fe7c08e6p-36, 0x1.2222e711631e6p-36, 0x1.2222e71158d7cp-36,
    0x1.1da3608199c8ap-36, 0x1.1da360818fd30p-36, 0x1.1935b43fa634cp-36, 0x1.1935b43f9c8d8p-36,
    0x1.14d99b7065ca4p-36, 0x1.14d99b705c6f1p-36, 0x1.108ed051ee930p-36, 0x1.108ed051e5818p-36,
    0x1.0c550e3733166p-36, 0x1.0c550e372a4c5p-36, 0x1.082c1183b7832p-36, 0x1.082c1183aefe4p-36,
    0x1.041397a757e19p-36, 0x1.041397a74f9fep-36, 0x1.000b5f1a1f0c3p-36, 0x1.000b5f1a170b8p-36,
    0x1.f8264eb05c552p-37, 0x1.f8264eb04cd1cp-37, 0x1.f05561bb68dc5p-37, 0x1.f05561bb59d32p-37,
    0x1.e8a37a45eda02p-37, 0x1.e8a37a45df0d6p-37, 0x1.e1101d30cf1ffp-37, 0x1.e1101d30c1000p-37,
    0x1.d99ad1459a6c9p-37, 0x1.d99ad1458cbbep-37, 0x1.d2431f2ef1b6cp-37, 0x1.d2431f2ee471ep-37,
    0x1.cb08917116ef9p-37, 0x1.cb0891710a133p-37, 0x1.c3eab46294029p-37, 0x1.c3eab462878b7p-37,
    0x1.bce916250034ep-37, 0x1.bce91624f4200p-37, 0x1.b603469de2355p-37, 0x1.b603469dd67f9p-37,
    0x1.af38d76fae6b0p-37, 0x1.af38d76fa3118p-37, 0x1.a8895bf2e113ep-37, 0x1.a8895bf2d613dp-37,
    0x1.a1f4692f33c36p-37, 0x1.a1f4692f2919ep-37, 0x1.9b7995d4edd4bp-37, 0x1.9b7995d4e37f4p-37,
    0x1.95187a364f672p-37, 0x1.95187a3645630p-37, 0x1.8ed0b0411678cp-37, 0x1.8ed0b0410cc39p-37,
    0x1.88a1d3781dba7p-37, 0x1.88a1d3781451bp-37, 0x1.828b80ed14b4ap-37, 0x1.828b80ed0b960p-37,
    0x1.7c8d573a50da5p-37, 0x1.7c8d573a48038p-37, 0x1.76a6f67cb7263p-37, 0x1.76a6f67cae950p-37,
    0x1.70d8004dbde12p-37, 0x1.70d8004db5937p-37, 0x1.6b2017bd86318p-37, 0x1.6b2017bd7e253p-37,
    0x1.657ee14d0d158p-37, 0x1.657ee14d05489p-37, 0x1.5ff402e8736b9p-37, 0x1.5ff402e86bdc1p-37,
    0x1.5a7f23e15cac9p-37, 0x1.5a7f23e15558ap-37, 0x1.551fece963ff1p-37, 0x1.551fece95ce4ep-37,
    0x1.4fd6080ca7497p-37, 0x1.4fd6080ca0672p-37, 0x1.4aa120ac67ec8p-37, 0x1.4aa120ac61407p-37,
    0x1.4580e379c0d0fp-37, 0x1.4580e379ba597p-37, 0x1.4074fe707171ap-37, 0x1.4074fe706b2d1p-37,
    0x1.3b7d20d1bd910p-37, 0x1.3b7d20d1b77ddp-37, 0x1.3698fb1f61469p-37, 0x1.3698fb1f5b633p-37,
    0x1.31c83f169913cp-37, 0x1.31c83f16935ecp-37, 0x1.2d0a9fab3db1bp-37, 0x1.2d0a9fab3829ap-37,
    0x1.285fd102f347cp-37, 0x1.285fd102edeb4p-37, 0x1.23c788706bbffp-37, 0x1.23c78870668dbp-37,
    0x1.1f417c6ebbeb9p-37, 0x1.1f417c6eb6e24p-37, 0x1.1acd649cc32e7p-37, 0x1.1acd649cbe4cdp-37,
    0x1.166af9b8a566fp-37, 0x1.166af9b8a0abbp-37, 0x1.1219f59b56ca0p-37, 0x1.1219f59b52341p-37,
    0x1.0dda1334396d0p-37, 0x1.0dda133434fb3p-37, 0x1.09ab0e84cc35ap-37, 0x1.09ab0e84c7e6ep-37,
    0x1.058ca49c6aecap-37, 0x1.058ca49c66bfcp-37, 0x1.017e93941f2d8p-37, 0x1.017e93941b218p-37,
    0x1.fb01351503e3fp-38, 0x1.fb013514fc0bbp-38, 0x1.f324f33f5aebfp-38, 0x1.f324f33f53518p-38,
    0x1.eb67e3e27e680p-38, 0x1.eb67e3e277097p-38, 0x1.e3c98b2cd3737p-38, 0x1.e3c98b2ccc4efp-38,
    0x1.dc496f382c2bdp-38, 0x1.dc496f38253f9p-38, 0x1.d4e7180229442p-38, 0x1.d4e71802228e6p-38,
    0x1.cda20f64b9d49p-38, 0x1.cda20f64b353bp-38, 0x1.c679e10eb8efep-38, 0x1.c679e10eb2a23p-38,
    0x1.bf6e1a7ca8873p-38, 0x1.bf6e1a7ca26b3p-38, 0x1.b87e4af18928ap-38, 0x1.b87e4af1833ccp-38,
    0x1.b1aa036fce260p-38, 0x1.b1aa036fc868cp-38, 0x1.aaf0d6b26db2dp-38, 0x1.aaf0d6b26822cp-38,
    0x1.a45259260c8a4p-38, 0x1.a452592607260p-38, 0x1.9dce20e244b0fp-38, 0x1.9dce20e23f772p-38,
    0x1.9763c5a306e56p-38, 0x1.9763c5a301d4cp-38, 0x1.9112e0c216569p-38, 0x1.9112e0c2116ddp-38,
    0x1.8adb0d309e377p-38, 0x1.8adb0d3099756p-38, 0x1.84bbe770e0c94p-38, 0x1.84bbe770dc2cbp-38,
    0x1.7eb50d8fff778p-38, 0x1.7eb50d8ffaff4p-38, 0x1.78c61f1fdba1bp-38, 0x1.78c61f1fd74cbp-38,
    0x1.72eebd310fb18p-38, 0x1.72eebd310b7e9p-38, 0x1.6d2e8a4d001c6p-38, 0x1.6d2e8a4cfc0a9p-38,
    0x1.67852a7003f25p-38, 0x1.67852a7000008p-38, 0x1.61f24303a49b3p-38, 0x1.61f24303a0c88p-38,
    0x1.5c757ad8f4686p-38, 0x1.5c757ad8f0b3cp-38, 0x1.570e7a22fb9ddp-38, 0x1.570e7a22f8066p-38,
    0x1.51bcea713b9bbp-38, 0x1.51bcea7138209p-38, 0x1.4c8076aa47cf4p-38, 0x1.4c8076aa446f8p-38,
    0x1.4758cb067414ap-38, 0x1.4758cb0670cf8p-38, 0x1.4245950a98358p-38, 0x1.4245950a950a1p-38,
    0x1.3d468382e82f5p-38, 0x1.3d468382e51cep-38, 0x1.385b467de0f02p-38, 0x1.385b467dddf5fp-38,
    0x1.33838f4749379p-38, 0x1.33838f474654cp-38, 0x1.2ebf1063464cap-38, 0x1.2ebf106343809p-38,
    0x1.2a0d7d898439bp-38, 0x1.2a0d7d898183bp-38, 0x1.256e8ba07140fp-38, 0x1.256e8ba06ea04p-38,
    0x1.20e1f0b88c3ccp-38, 0x1.20e1f0b889b0cp-38, 0x1.1c676407c5a1cp-38, 0x1.1c676407c329dp-38,
    0x1.17fe9de4f2d7ap-38, 0x1.17fe9de4f0732p-38, 0x1.13a757c353a07p-38, 0x1.13a757c3514edp-38,
    0x1.0f614c2e29470p-38, 0x1.0f614c2e2707ap-38, 0x1.0b2c36c45f4cdp-38, 0x1.0b2c36c45d1f2p-38,
    0x1.0707d43445534p-38, 0x1.0707d4344336cp-38, 0x1.02f3e23759fb0p-38, 0x1.02f3e23757ef2p-38,
    0x1.fde03f1c4cecbp-39, 0x1.fde03f1c48f53p-39, 0x1.f5f897f85518bp-39, 0x1.f5f897f851407p-39,
    0x1.ee305087b1970p-39, 0x1.ee305087addd0p-39, 0x1.e686ec4545570p-39, 0x1.e686ec4541ba5p-39,
    0x1.defbf09a28beap-39, 0x1.defbf09a253e7p-39, 0x1.d78ee4d600318p-39, 0x1.d78ee4d5fcccep-39,
    0x1.d03f522771011p-39, 0x1.d03f52276db73p-39, 0x1.c90cc394b44d4p-39, 0x1.c90cc394b11d4p-39,
    0x1.c1f6c5f4475e1p-39, 0x1.c1f6c5f444473p-39, 0x1.bafce7e5b901fp-39, 0x1.bafce7e5b6036p-39,
    0x1.b41eb9ca937d2p-39, 0x1.b41eb9ca90963p-39, 0x1.ad5bcdbf62993p-39, 0x1.ad5bcdbf5fc92p-39,
    0x1.a6b3b794d5648p-39, 0x1.a6b3b794d2aa8p-39, 0x1.a0260cc8fb340p-39, 0x1.a0260cc8f88f8p-39,
    0x1.99b264809b7bap-39, 0x1.99b2648098ebfp-39, 0x1.93585780a811bp-39, 0x1.93585780a5963p-39,
    0x1.8d178027c975cp-39, 0x1.8d178027c70ddp-39, 0x1.86ef7a6804b24p-39, 0x1.86ef7a68025d4p-39,
    0x1.80dfe3c07a74dp-39, 0x1.80dfe3c078323p-39, 0x1.7ae85b373ef81p-39, 0x1.7ae85b373cc74p-39,
    0x1.750881534a5cap-39, 0x1.75088153483d1p-39, 0x1.6f3ff8168110cp-39, 0x1.6f3ff8167f01ep-39,
    0x1.698e62f7d3e6ep-39, 0x1.698e62f7d1e84p-39, 0x1.63f366dd777cfp-39, 0x1.63f366dd758e0p-39,
    0x1.5e6eaa173297cp-39, 0x1.5e6eaa1730b81p-39, 0x1.58ffd458c3188p-39, 0x1.58ffd458c1479p-39,
    0x1.53a68eb45930cp-39, 0x1.53a68eb4576e2p-39, 0x1.4e628395287eap-39, 0x1.4e62839526c9ep-39,
    0x1.49335eba0eb88p-39, 0x1.49335eba0d113p-39, 0x1.4418cd304f943p-39, 0x1.4418cd304df9ep-39,
    0x1.3f127d4e65941p-39, 0x1.3f127d4e64066p-39, 0x1.3a201eaee767fp-39, 0x1.3a201eaee5e68p-39,
    0x1.3541622b818fdp-39, 0x1.3541622b801a4p-39, 0x1.3075f9d803f03p-39, 0x1.3075f9d802861p-39,
    0x1.2bbd98fd83082p-39, 0x1.2bbd98fd81a93p-39, 0x1.2717f4158c7cdp-39, 0x1.2717f4158b28bp-39,
    0x1.2284c0c56eab7p-39, 0x1.2284c0c56d61cp-39, 0x1.1e03b5d992f87p-39, 0x1.1e03b5d991b8ep-39,
    0x1.19948b40ea8f9p-39, 0x1.19948b40e959dp-39, 0x1.1536fa086d4d4p-39, 0x1.1536fa086c211p-39,
    0x1.10eabc56aa880p-39, 0x1.10eabc56a9651p-39, 0x1.0caf8d676b73bp-39, 0x1.0caf8d676a59bp-39,
    0x1.0885298766d85p-39, 0x1.0885298765c70p-39, 0x1.046b4e1005d7bp-39, 0x1.046b4e1004cedp-39,
    0x1.0061b963397ebp-39, 0x1.0061b963387dep-39, 0x1.f8d055cec1bd2p-40, 0x1.f8d055cebfcb6p-40,
    0x1.f0fcc6067edb9p-40, 0x1.f0fcc6067cf92p-40, 0x1.e948463406dd8p-40, 0x1.e94846340509fp-40,
    0x1.e1b25b0eb83b2p-40, 0x1.e1b25b0eb675fp-40, 0x1.da3a8b373ecb9p-40, 0x1.da3a8b373d145p-40,
    0x1.d2e05f2ffdc5bp-40, 0x1.d2e05f2ffc1bfp-40, 0x1.cba3615597dc0p-40, 0x1.cba36155963f5p-40,
    0x1.c4831dd794fd6p-40, 0x1.c4831dd7936d7p-40, 0x1.bd7f22b12543bp-40, 0x1.bd7f22b123c01p-40,
    0x1.b696ffa2009d6p-40, 0x1.b696ffa1ff25bp-40, 0x1.afca462762bfbp-40, 0x1.afca462761539p-40,
    0x1.a918897522f0fp-40, 0x1.a918897521900p-40, 0x1.a2815e6ee73d1p-40, 0x1.a2815e6ee5e70p-40,
    0x1.9c045ba172a74p-40, 0x1.9c045ba1715bbp-40, 0x1.95a1193c0decfp-40, 0x1.95a1193c0cabap-40,
    0x1.8f57310a0a722p-40, 0x1.8f57310a093aap-40, 0x1.89263e6c5eed8p-40, 0x1.89263e6c5dbfap-40,
    0x1.830dde535d700p-40, 0x1.830dde535c4b6p-40, 0x1.7d0daf3882612p-40, 0x1.7d0daf3881458p-40,
    0x1.772551185c0f1p-40, 0x1.772551185afc3p-40, 0x1.7154656c8a6f6p-40, 0x1.7154656c8964fp-40,
    0x1.6b9a8f25d6b0fp-40, 0x1.6b9a8f25d5aecp-40, 0x1.65f772a662413p-40, 0x1.65f772a66146fp-40,
    0x1.606ab5bbece63p-40, 0x1.606ab5bbebf3ap-40, 0x1.5af3ff9a31935p-40, 0x1.5af3ff9a30a83p-40,
    0x1.5592f8d5599d6p-40, 0x1.5592f8d558b98p-40, 0x1.50474b5c85f63p-40, 0x1.50474b5c85195p-40,
    0x1.4b10a2746e171p-40, 0x1.4b10a2746d410p-40, 0x1.45eeaab214459p-40, 0x1.45eeaab213761p-40,
    0x1.40e111f58edc9p-40, 0x1.40e111f58e138p-40, 0x1.3be78764e646dp-40, 0x1.3be78764e583ep-40,
    0x1.3701bb6707589p-40, 0x1.3701bb67069bbp-40, 0x1.322f5f9ec9b82p-40, 0x1.322f5f9ec9010p-40,
    0x1.2d7026e60a046p-40, 0x1.2d7026e60952fp-40, 0x1.28c3c548d76c7p-40, 0x1.28c3c548d6c07p-40,
    0x1.2429f000b46a3p-40, 0x1.2429f000b3c37p-40, 0x1.1fa25d6fea540p-40, 0x1.1fa25d6fe9b27p-40,
    0x1.1b2cc51cef7bap-40, 0x1.1b2cc51ceedf0p-40, 0x1.16c8dfaddf8f1p-40, 0x1.16c8dfaddef75p-40,
    0x1.127666e405f4cp-40, 0x1.127666e40561ap-40, 0x1.0e35159779da3p-40, 0x1.0e351597794b9p-40,
    0x1.0a04a7b2cbaf9p-40, 0x1.0a04a7b2cb256p-40, 0x1.05e4da2ec3cb6p-40, 0x1.05e4da2ec3457p-40,
    0x1.01d56b0e31f12p-40, 0x1.01d56b0e316f5p-40, 0x1.fbac32b39af20p-41, 0x1.fbac32b399f65p-41,
    0x1.f3cd4a384bab5p-41, 0x1.f3cd4a384ab76p-41, 0x1.ec0d9ebb46704p-41, 0x1.ec0d9ebb4583dp-41,
    0x1.e46cb4412e21dp-41, 0x1.e46cb4412d3cbp-41, 0x1.dcea10bab8600p-41, 0x1.dcea10bab781ep-41,
    0x1.d5853bfd0c8adp-41, 0x1.d5853bfd0bb39p-41, 0x1.ce3dbfba410adp-41, 0x1.ce3dbfba403a2p-41,
    0x1.c7132779f6688p-41, 0x1.c7132779f59e5p-41, 0x1.c00500920fbd0p-41, 0x1.c00500920ef90p-41,
    0x1.b912da1f88065p-41, 0x1.b912da1f87486p-41, 0x1.b23c44ff63edcp-41, 0x1.b23c44ff6335ap-41,
    0x1.ab80d3c7bf8f1p-41, 0x1.ab80d3c7bedc9p-41, 0x1.a4e01ac0f7d0dp-41, 0x1.a4e01ac0f723dp-41,
    0x1.9e59afdeeee19p-41, 0x1.9e59afdeee39ep-41, 0x1.97ed2aba6b6cdp-41, 0x1.97ed2aba6aca5p-41,
    0x1.919a248a921f0p-41, 0x1.919a248a91818p-41, 0x1.8b60381e790f3p-41, 0x1.8b60381e78768p-41,
    0x1.853f01d6d4a7bp-41, 0x1.853f01d6d413bp-41, 0x1.7f361f9fbda98p-41, 0x1.7f361f9fbd1a1p-41,
    0x1.794530ea8fe56p-41, 0x1.794530ea8f5a6p-41, 0x1.736bd6a7e149ap-41, 0x1.736bd6a7e0c2fp-41,
    0x1.6da9b34190e3ap-41, 0x1.6da9b34190611p-41, 0x1.67fe6a94ed75dp-41, 0x1.67fe6a94ecf74p-41,
    0x1.6269a1ecf344fp-41, 0x1.6269a1ecf2ca4p-41, 0x1.5ceafffca0c06p-41, 0x1.5ceafffca0498p-41,
    0x1.57822cd961aabp-41, 0x1.57822cd961377p-41, 0x1.522ed1f59068ap-41, 0x1.522ed1f58ff8fp-41,
    0x1.4cf09a1b0d201p-41, 0x1.4cf09a1b0cb3dp-41, 0x1.47c73165ea4e9p-41, 0x1.47c73165e9e5ap-41,
    0x1.42b2453f2e83ap-41, 0x1.42b2453f2e1dfp-41, 0x1.3db18457aaea5p-41, 0x1.3db18457aa87cp-41,
    0x1.38c49ea2e64f7p-41, 0x1.38c49ea2e5efep-41, 0x1.33eb45521c535p-41, 0x1.33eb45521bf6bp-41,
    0x1.2f252acf50770p-41, 0x1.2f252acf501d4p-41, 0x1.2a7202b874b61p-41, 0x1.2a7202b8745f1p-41,
    0x1.25d181daa35f3p-41, 0x1.25d181daa30aep-41, 0x1.21435e2d6bdfap-41, 0x1.21435e2d6b8dfp-41,
    0x1.1cc74ece32363p-41, 0x1.1cc74ece31e70p-41, 0x1.185d0bfba0c30p-41, 0x1.185d0bfba0764p-41,
    0x1.14044f112c2cap-41, 0x1.14044f112be23p-41, 0x1.0fbcd282a9112p-41, 0x1.0fbcd282a8c90p-41,
    0x1.0b8651d7f33dcp-41, 0x1.0b8651d7f2f7ep-41, 0x1.076089a8a626fp-41, 0x1.076089a8a5e33p-41,
    0x1.034b3797e65c4p-41, 0x1.034b3797e61aap-41, 0x1.fe8c34a0776afp-42, 0x1.fe8c34a076ebap-42,
    0x1.f6a1e2fef7ea7p-42, 0x1.f6a1e2fef76f1p-42, 0x1.eed6fba58b429p-42, 0x1.eed6fba58acb0p-42,
    0x1.e72b01e5159e5p-42, 0x1.e72b01e5152a7p-42, 0x1.df9d7afd574bcp-42, 0x1.df9d7afd56db7p-42,
    0x1.d82dee1540ae3p-42, 0x1.d82dee1540415p-42, 0x1.d0dbe43364a2bp-42, 0x1.d0dbe43364393p-42,
    0x1.c9a6e83688dfdp-42, 0x1.c9a6e83688799p-42, 0x1.c28e86ce53d7cp-42, 0x1.c28e86ce5374ap-42,
    0x1.bb924e7417a97p-42, 0x1.bb924e7417496p-42, 0x1.b4b1cf63b9ac2p-42, 0x1.b4b1cf63b94f0p-42,
    0x1.adec9b94b6246p-42, 0x1.adec9b94b5ca2p-42, 0x1.a74246b33fb2ap-42, 0x1.a74246b33f5b3p-42,
    0x1.a0b266197a0d9p-42, 0x1.a0b2661979b8dp-42, 0x1.9a3c90c8cf9b1p-42, 0x1.9a3c90c8cf48fp-42,
    0x1.93e05f63617e8p-42, 0x1.93e05f63612edp-42, 0x1.8d9d6c2591b1dp-42, 0x1.8d9d6c259164ap-42,
    0x1.877352dfa6c39p-42, 0x1.877352dfa678bp-42, 0x1.8161b0ef88d2ap-42, 0x1.8161b0ef888a1p-42,
    0x1.7b68253a9764bp-42, 0x1.7b68253a971e7p-42, 0x1.7586502797b43p-42, 0x1.7586502797701p-42,
    0x1.6fbbd398bb146p-42, 0x1.6fbbd398bad26p-42, 0x1.6a0852e5bd0cep-42, 0x1.6a0852e5bcccep-42,
    0x1.646b72d618cd7p-42, 0x1.646b72d6188f7p-42, 0x1.5ee4d99b559e4p-42, 0x1.5ee4d99b55623p-42,
    0x1.59742ecb69f0dp-42, 0x1.59742ecb69b69p-42, 0x1.54191b5b34b7dp-42, 0x1.54191b5b347f6p-42,
    0x1.4ed349990cae3p-42, 0x1.4ed349990c777p-42, 0x1.49a2652765350p-42, 0x1.49a2652764fffp-42,
    0x1.44861af78873dp-42, 0x1.44861af788406p-42, 0x1.3f7e194466667p-42, 0x1.3f7e194466349p-42,
    0x1.3a8a0f8d78851p-42, 0x1.3a8a0f8d7854cp-42, 0x1.35a9ae91b9b52p-42, 0x1.35a9ae91b9865p-42,
    0x1.30dca84ab2327p-42, 0x1.30dca84ab2051p-42, 0x1.2c22afe797212p-42, 0x1.2c22afe796f52p-42,
    0x1.277b79c87d7a8p-42, 0x1.277b79c87d4fep-42, 0x1.22e6bb79a0085p-42, 0x1.22e6bb799fdf0p-42,
    0x1.1e642baeb8220p-42, 0x1.1e642baeb7f9fp-42, 0x1.19f3823e68e23p-42, 0x1.19f3823e68bb5p-42,
    0x1.1594781dbc8afp-42, 0x1.1594781dbc655p-42, 0x1.1146c75bb3d07p-42, 0x1.1146c75bb3ac0p-42,
    0x1.0d0a2b1ce6c35p-42, 0x1.0d0a2b1ce69ffp-42, 0x1.08de5f9737141p-42, 0x1.08de5f9736f1dp-42,
    0x1.04c3220d936c0p-42, 0x1.04c3220d934adp-42, 0x1.00b830cbcb964p-42, 0x1.00b830cbcb761p-42,
    0x1.f97a9644ea6eap-43, 0x1.f97a9644ea304p-43, 0x1.f1a462c5c1a25p-43, 0x1.f1a462c5c165ep-43,
    0x1.e9ed49b63da5dp-43, 0x1.e9ed49b63d6b3p-43, 0x1.e254cfa428e90p-43, 0x1.e254cfa428b03p-43,
    0x1.dada7b0740402p-43, 0x1.dada7b0740091p-43, 0x1.d37dd4399a554p-43, 0x1.d37dd4399a1fep-43,
    0x1.cc3e65702d3fcp-43, 0x1.cc3e65702d0c1p-43, 0x1.c51bbab371ca0p-43, 0x1.c51bbab37197ep-43,
    0x1.be1561d823eefp-43, 0x1.be1561d823be6p-43, 0x1.b72aea78201cdp-43, 0x1.b72aea781fedcp-43,
    0x1.b05be5eb5cc90p-43, 0x1.b05be5eb5c9b6p-43, 0x1.a9a7e740ffe6bp-43, 0x1.a9a7e740ffba8p-43,
    0x1.a30e83388fcfep-43, 0x1.a30e83388fa50p-43, 0x1.9c8f503b3f34ep-43, 0x1.9c8f503b3f0b5p-43,
    0x1.9629e65553a6ep-43, 0x1.9629e655537e9p-43, 0x1.8fdddf2fa6534p-43, 0x1.8fdddf2fa62c4p-43,
    0x1.89aad6093e891p-43, 0x1.89aad6093e634p-43, 0x1.839067b105a0cp-43, 0x1.839067b1057c1p-43,
    0x1.7d8e327f93e2ap-43, 0x1.7d8e327f93bf2p-43, 0x1.77a3d65116084p-43, 0x1.77a3d65115e5dp-43,
    0x1.71d0f47f4af71p-43, 0x1.71d0f47f4ad5bp-43, 0x1.6c152fdb9954cp-43, 0x1.6c152fdb99346p-43,
    0x1.66702ca93c957p-43, 0x1.66702ca93c761p-43, 0x1.60e1909789283p-43, 0x1.60e190978909dp-43,
    0x1.5b6902bc4764ap-43, 0x1.5b6902bc47472p-43, 0x1.56062b8e24dfdp-43, 0x1.56062b8e24c34p-43,
    0x1.50b8b4df3bd02p-43, 0x1.50b8b4df3bb47p-43, 0x1.4b8049d7b0278p-43, 0x1.4b8049d7b00cap-43,
    0x1.465c96f0620ecp-43, 0x1.465c96f061f4cp-43, 0x1.414d49edb56c8p-43, 0x1.414d49edb5535p-43,
    0x1.3c5211da6e24cp-43, 0x1.3c5211da6e0c5p-43, 0x1.376a9f02a0be1p-43, 0x1.376a9f02a0a66p-43,
    0x1.3296a2eeb71c7p-43, 0x1.3296a2eeb7058p-43, 0x1.2dd5d05e89018p-43, 0x1.2dd5d05e88eb4p-43,
    0x1.2927db4488033p-43, 0x1.2927db4487edap-43, 0x1.248c78c0feacep-43, 0x1.248c78c0fe980p-43,
    0x1.20035f1d627d8p-43, 0x1.20035f1d62694p-43, 0x1.1b8c45c7b8790p-43, 0x1.1b8c45c7b8656p-43,
    0x1.1726e54e0c027p-43, 0x1.1726e54e0bef7p-43, 0x1.12d2f759f7b6dp-43, 0x1.12d2f759f7a46p-43,
    0x1.0e9036ac4000dp-43, 0x1.0e9036ac3feefp-43, 0x1.0a5e5f187f1f6p-43, 0x1.0a5e5f187f0e0p-43,
    0x1.063d2d80e259ap-43, 0x1.063d2d80e248dp-43, 0x1.022c5fd1f81c2p-43, 0x1.022c5fd1f80bdp-43,
    0x1.fc5769fd1d787p-44, 0x1.fc5769fd1d58ep-44, 0x1.f475d9f7473f4p-44, 0x1.f475d9f74720bp-44,
    0x1.ecb39178c50d9p-44, 0x1.ecb39178c4effp-44, 0x1.e510145c6974ep-44, 0x1.e510145c69582p-44,
    0x1.dd8ae869bfba0p-44, 0x1.dd8ae869bf9e2p-44, 0x1.d623954d6843bp-44, 0x1.d623954d6828bp-44,
    0x1.ced9a491935a8p-44, 0x1.ced9a49193406p-44, 0x1.c7aca19699c23p-44, 0x1.c7aca19699a8dp-44,
    0x1.c09c198bb2b52p-44, 0x1.c09c198bb29c9p-44, 0x1.b9a79b67c6ceap-44, 0x1.b9a79b67c6b6dp-44,
    0x1.b2ceb7e25f6fdp-44, 0x1.b2ceb7e25f58cp-44, 0x1.ac11016cb22efp-44, 0x1.ac11016cb2189p-44,
    0x1.a56e0c2ac7e1ap-44, 0x1.a56e0c2ac7cbfp-44, 0x1.9ee56decbed49p-44, 0x1.9ee56decbebf8p-44,
    0x1.9876be2827c45p-44, 0x1.9876be2827affp-44, 0x1.922195f17d2dep-44, 0x1.922195f17d1a2p-44,
    0x1.8be58ff5b48dap-44, 0x1.8be58ff5b47a8p-44, 0x1.85c24873e9264p-44, 0x1.85c24873e913bp-44,
    0x1.7fb75d371fea1p-44, 0x1.7fb75d371fd82p-44, 0x1.79c46d9024237p-44, 0x1.79c46d9024120p-44,
    0x1.73e91a4f7c78fp-44, 0x1.73e91a4f7c680p-44, 0x1.6e2505bf77ee4p-44, 0x1.6e2505bf77ddep-44,
    0x1.6877d39e52812p-44, 0x1.6877d39e52714p-44, 0x1.62e1291871058p-44, 0x1.62e1291870f62p-44,
    0x1.5d60acc2b3e41p-44, 0x1.5d60acc2b3d53p-44, 0x1.57f60694e0613p-44, 0x1.57f60694e052cp-44,
    0x1.52a0dfe420117p-44, 0x1.52a0dfe420037p-44, 0x1.4d60e35d96257p-44, 0x1.4d60e35d9617ep-44,
    0x1.4835bd010a349p-44, 0x1.4835bd010a276p-44, 0x1.431f1a1ba832ap-44, 0x1.431f1a1ba825ep-44,
    0x1.3e1ca942d53bcp-44, 0x1.3e1ca942d52f6p-44, 0x1.392e1a4f18e3cp-44, 0x1.392e1a4f18d7dp-44,
    0x1.34531e571ab82p-44, 0x1.34531e571aac8p-44, 0x1.2f8b67aab3a3bp-44, 0x1.2f8b67aab3987p-44,
    0x1.2ad6a9ce12e5fp-44, 0x1.2ad6a9ce12db1p-44, 0x1.26349974f64f7p-44, 0x1.26349974f644ep-44,
    0x1.21a4ec7df5779p-44, 0x1.21a4ec7df56d5p-44, 0x1.1d2759eddf9f9p-44, 0x1.1d2759eddf95bp-44,
    0x1.18bb99eb2bf9cp-44, 0x1.18bb99eb2bf02p-44, 0x1.146165b97c0aap-44, 0x1.146165b97c015p-44,
    0x1.101877b52fdd5p-44, 0x1.101877b52fd45p-44, 0x1.0be08b4f0bc3cp-44, 0x1.0be08b4f0bbb0p-44,
    0x1.07b95d07ef5d2p-44, 0x1.07b95d07ef54ap-44, 0x1.03a2aa6c9d9e3p-44, 0x1.03a2aa6c9d960p-44,
    0x1.ff3864232b307p-45, 0x1.ff3864232b208p-45, 0x1.f74b671df7764p-45, 0x1.f74b671df766dp-45,
    0x1.ef7ddef926a52p-45, 0x1.ef7ddef926962p-45, 0x1.e7cf4edb8ff9bp-45, 0x1.e7cf4edb8feb3p-45,
    0x1.e03f3bdb8db8dp-45, 0x1.e03f3bdb8daacp-45, 0x1.d8cd2cf74e8b2p-45, 0x1.d8cd2cf74e7d8p-45,
    0x1.d178ab0d4555cp-45, 0x1.d178ab0d45489p-45, 0x1.ca4140d4b717bp-45, 0x1.ca4140d4b70aep-45,
    0x1.c3267ad666542p-45, 0x1.c3267ad66647bp-45, 0x1.bc27e7655b954p-45, 0x1.bc27e7655b893p-45,
    0x1.b5451697ca931p-45, 0x1.b5451697ca876p-45, 0x1.ae7d9a40138d9p-45, 0x1.ae7d9a4013824p-45,
    0x1.a7d105e5e0694p-45, 0x1.a7d105e5e05e5p-45, 0x1.a13eeebf5d20fp-45, 0x1.a13eeebf5d165p-45,
    0x1.9ac6ebaa8b1f9p-45, 0x1.9ac6ebaa8b154p-45, 0x1.94689526af177p-45, 0x1.94689526af0d7p-45,
    0x1.8e23854dd8ee0p-45, 0x1.8e23854dd8e45p-45, 0x1.87f757ce85543p-45, 0x1.87f757ce854adp-45,
    0x1.81e3a9e558a63p-45, 0x1.81e3a9e5589d1p-45, 0x1.7be81a56f2acfp-45, 0x1.7be81a56f2a43p-45,
    0x1.76044969dae0bp-45, 0x1.76044969dad82p-45, 0x1.7037d8e084c8dp-45, 0x1.7037d8e084c08p-45,
    0x1.6a826bf36c1bbp-45, 0x1.6a826bf36c13ap-45, 0x1.64e3a74b483e6p-45, 0x1.64e3a74b4836ap-45,
    0x1.5f5b30fb56c8cp-45, 0x1.5f5b30fb56c13p-45, 0x1.59e8b07bbcb19p-45, 0x1.59e8b07bbcaa4p-45,
    0x1.548bcea3fdc99p-45, 0x1.548bcea3fdc28p-45, 0x1.4f4435a58a2c7p-45, 0x1.4f4435a58a259p-45,
    0x1.4a1191066150bp-45, 0x1.4a119106614a0p-45, 0x1.44f38d9bca606p-45, 0x1.44f38d9bca59fp-45,
    0x1.3fe9d98521870p-45, 0x1.3fe9d9852180cp-45, 0x1.3af42426b9e01p-45, 0x1.3af42426b9da0p-45,
    0x1.36121e24d3b5cp-45, 0x1.36121e24d3afep-45, 0x1.3143795ea6be4p-45, 0x1.3143795ea6b89p-45,
    0x1.2c87e8e98008ep-45, 0x1.2c87e8e980036p-45, 0x1.27df210bf34c4p-45, 0x1.27df210bf346fp-45,
    0x1.2348d7391f497p-45, 0x1.2348d7391f444p-45, 0x1.1ec4c20c04f77p-45, 0x1.1ec4c20c04f26p-45,
    0x1.1a529942f12d5p-45, 0x1.1a529942f1287p-45, 0x1.15f215baf880fp-45, 0x1.15f215baf87c3p-45,
    0x1.11a2f16b85123p-45, 0x1.11a2f16b850dap-45, 0x1.0d64e761f5fc2p-45, 0x1.0d64e761f5f7bp-45,
    0x1.0937b3bd5024ap-45, 0x1.0937b3bd50205p-45, 0x1.051b13aa00279p-45, 0x1.051b13aa00237p-45,
    0x1.010ec55dad17dp-45, 0x1.010ec55dad13cp-45, 0x1.fa25102637a80p-46, 0x1.fa25102637a03p-46,
    0x1.f24c380c455bdp-46, 0x1.f24c380c45543p-46, 0x1.ea9284df5a441p-46, 0x1.ea9284df5a3cbp-46,
    0x1.e2f77b039ec2dp-46, 0x1.e2f77b039ebbbp-46, 0x1.db7aa0c7d2db3p-46, 0x1.db7aa0c7d2d45p-46,
    0x1.d41b7e5db3135p-46, 0x1.d41b7e5db30cap-46, 0x1.ccd99dd27b85ep-46, 0x1.ccd99dd27b7f7p-46,
    0x1.c5b48b0788ac9p-46, 0x1.c5b48b0788a64p-46, 0x1.beabd3ab156b7p-46, 0x1.beabd3ab15656p-46,
    0x1.b7bf073115ebep-46, 0x1.b7bf073115e60p-46, 0x1.b0edb6cc2ed1dp-46, 0x1.b0edb6cc2ecc1p-46,
    0x1.aa377566c85d2p-46, 0x1.aa377566c8579p-46, 0x1.a39bd79c3d071p-46, 0x1.a39bd79c3d01bp-46,
    0x1.9d1a73b2232ebp-46, 0x1.9d1a73b223298p-46, 0x1.96b2e191b169ep-46, 0x1.96b2e191b164dp-46,
    0x1.9064bac13d0fbp-46, 0x1.9064bac13d0adp-46, 0x1.8a2f9a5dd2956p-46, 0x1.8a2f9a5dd290ap-46,
    0x1.84131d14e7569p-46, 0x1.84131d14e751fp-46, 0x1.7e0ee11e24649p-46, 0x1.7e0ee11e24601p-46,
    0x1.7822863549f89p-46, 0x1.7822863549f44p-46, 0x1.724dad942b27cp-46, 0x1.724dad942b239p-46,
    0x1.6c8ff9ecc1789p-46, 0x1.6c8ff9ecc1748p-46, 0x1.66e90f6357fa7p-46, 0x1.66e90f6357f68p-46,
    0x1.61589388cd832p-46, 0x1.61589388cd7f5p-46, 0x1.5bde2d54edb4ap-46, 0x1.5bde2d54edb0fp-46,
    0x1.56798520e072ep-46, 0x1.56798520e06f5p-46, 0x1.512a44a1af6edp-46, 0x1.512a44a1af6b5p-46,
    0x1.4bf016e2e16fbp-46, 0x1.4bf016e2e16c6p-46, 0x1.46caa8412b04cp-46, 0x1.46caa8412b017p-46,
    0x1.41b9a6653448fp-46, 0x1.41b9a6653445dp-46, 0x1.3cbcc03e73675p-46, 0x1.3cbcc03e73644p-46,
    0x1.37d3a5fe1b8afp-46, 0x1.37d3a5fe1b880p-46, 0x1.32fe09121fec0p-46, 0x1.32fe09121fe92p-46,
    0x1.2e3b9c204aa82p-46, 0x1.2e3b9c204aa55p-46, 0x1.298c13016718bp-46, 0x1.298c130167160p-46,
    0x1.24ef22bc7f592p-46, 0x1.24ef22bc7f568p-46, 0x1.206481822cb18p-46, 0x1.206481822caefp-46,
    0x1.1bebe6a7fa999p-46, 0x1.1bebe6a7fa972p-46, 0x1.17850aa3dc0bdp-46, 0x1.17850aa3dc097p-46,
    0x1.132fa707b2de7p-46, 0x1.132fa707b2dc2p-46, 0x1.0eeb767ce8dbcp-46, 0x1.0eeb767ce8d98p-46,
    0x1.0ab834c01a52ep-46, 0x1.0ab834c01a50bp-46, 0x1.06959e9cd1dbep-46, 0x1.06959e9cd1d9cp-46,
    0x1.028371e9550aep-46, 0x1.028371e95508dp-46, 0x1.fd02db05039dap-47, 0x1.fd02db050399bp-47,
    0x1.f51ea28f78740p-47, 0x1.f51ea28f78702p-47, 0x1.ed59bc2dd8e5bp-47, 0x1.ed59bc2dd8e1fp-47,
    0x1.e5b3ab91191a8p-47, 0x1.e5b3ab911916fp-47, 0x1.de2bf6578c1a3p-47, 0x1.de2bf6578c16bp-47,
    0x1.d6c224053da70p-47, 0x1.d6c224053da3ap-47, 0x1.cf75bdfc6a74fp-47, 0x1.cf75bdfc6a71bp-47,
    0x1.c8464f7616435p-47, 0x1.c8464f7616402p-47, 0x0.0p+0, 0x0.0p+0,
};
// Signed Softplus table (tools/gen_fp64_tables.py): {g(c_j), 1/2 - sigmoid(c_j)} with
// g(h) = softplus(h) - h/2, c_j = j * kSgStep, j = -1280..799, and two linear end entries (h >= 20:
// g = h/2, torch's threshold; h < -32.03: g = -h/2) (softplus_sg, the fp64 decoder_v2_4 forward)
__constant__ static const double kSgTab[4164] = {
    0x1.005c37b6fe8f3p+4, 0x1.0000000000000p-1, 0x1.0028fc5154b1ap+4, 0x1.fffffffffff20p-2,
    0x1.ffeb81d755a7dp+3, 0x1.fffffffffff1bp-2, 0x1.ff850b0c01ec6p+3, 0x1.fffffffffff15p-2,
    0x1.ff1e9440ae30ep+3, 0x1.fffffffffff0fp-2, 0x1.feb81d755a757p+3, 0x1.fffffffffff09p-2,
    0x1.fe51a6aa06b9fp+3, 0x1.fffffffffff03p-2, 0x1.fdeb2fdeb2fe8p+3, 0x1.ffffffffffefcp-2,
    0x1.fd84b9135f431p+3, 0x1.ffffffffffef6p-2, 0x1.fd1e42480b879p+3, 0x1.ffffffffffeefp-2,
    0x1.fcb7cb7cb7cc2p+3, 0x1.ffffffffffee8p-2, 0x1.fc5154b16410ap+3, 0x1.ffffffffffee1p-2,
    0x1.fbeadde610553p+3, 0x1.ffffffffffedap-2, 0x1.fb84671abc99cp+3, 0x1.ffffffffffed2p-2,
    0x1.fb1df04f68de4p+3, 0x1.ffffffffffecap-2, 0x1.fab779841522dp+3, 0x1.ffffffffffec3p-2,
    0x1.fa5102b8c1675p+3, 0x1.ffffffffffebbp-2, 0x1.f9ea8bed6dabep+3, 0x1.ffffffffffeb2p-2,
    0x1.f984152219f07p+3, 0x1.ffffffffffeaap-2, 0x1.f91d9e56c634fp+3, 0x1.ffffffffffea1p-2,
    0x1.f8b7278b72798p+3, 0x1.ffffffffffe98p-2, 0x1.f850b0c01ebe1p+3, 0x1.ffffffffffe8fp-2,
    0x1.f7ea39f4cb029p+3, 0x1.ffffffffffe86p-2, 0x1.f783c32977472p+3, 0x1.ffffffffffe7cp-2,
    0x1.f71d4c5e238bbp+3, 0x1.ffffffffffe72p-2, 0x1.f6b6d592cfd03p+3, 0x1.ffffffffffe68p-2,
    0x1.f6505ec77c14cp+3, 0x1.ffffffffffe5ep-2, 0x1.f5e9e7fc28595p+3, 0x1.ffffffffffe53p-2,
    0x1.f5837130d49ddp+3, 0x1.ffffffffffe49p-2, 0x1.f51cfa6580e26p+3, 0x1.ffffffffffe3dp-2,
    0x1.f4b6839a2d26fp+3, 0x1.ffffffffffe32p-2, 0x1.f4500cced96b7p+3, 0x1.ffffffffffe26p-2,
    0x1.f3e9960385b00p+3, 0x1.ffffffffffe1ap-2, 0x1.f3831f3831f49p+3, 0x1.ffffffffffe0ep-2,
    0x1.f31ca86cde392p+3, 0x1.ffffffffffe01p-2, 0x1.f2b631a18a7dap+3, 0x1.ffffffffffdf5p-2,
    0x1.f24fbad636c23p+3, 0x1.ffffffffffde7p-2, 0x1.f1e9440ae306cp+3, 0x1.ffffffffffddap-2,
    0x1.f182cd3f8f4b5p+3, 0x1.ffffffffffdccp-2, 0x1.f11c56743b8fep+3, 0x1.ffffffffffdbdp-2,
    0x1.f0b5dfa8e7d46p+3, 0x1.ffffffffffdafp-2, 0x1.f04f68dd9418fp+3, 0x1.ffffffffffda0p-2,
    0x1.efe8f212405d8p+3, 0x1.ffffffffffd90p-2, 0x1.ef827b46eca21p+3, 0x1.ffffffffffd81p-2,
    0x1.ef1c047b98e6ap+3, 0x1.ffffffffffd70p-2, 0x1.eeb58db0452b3p+3, 0x1.ffffffffffd60p-2,
    0x1.ee4f16e4f16fcp+3, 0x1.ffffffffffd4fp-2, 0x1.ede8a0199db45p+3, 0x1.ffffffffffd3dp-2,
    0x1.ed82294e49f8ep+3, 0x1.ffffffffffd2bp-2, 0x1.ed1bb282f63d6p+3, 0x1.ffffffffffd19p-2,
    0x1.ecb53bb7a281fp+3, 0x1.ffffffffffd06p-2, 0x1.ec4ec4ec4ec68p+3, 0x1.ffffffffffcf3p-2,
    0x1.ebe84e20fb0b1p+3, 0x1.ffffffffffcdfp-2, 0x1.eb81d755a74fap+3, 0x1.ffffffffffccbp-2,
    0x1.eb1b608a53943p+3, 0x1.ffffffffffcb6p-2, 0x1.eab4e9beffd8cp+3, 0x1.ffffffffffca1p-2,
    0x1.ea4e72f3ac1d5p+3, 0x1.ffffffffffc8bp-2, 0x1.e9e7fc285861fp+3, 0x1.ffffffffffc74p-2,
    0x1.e981855d04a68p+3, 0x1.ffffffffffc5dp-2, 0x1.e91b0e91b0eb1p+3, 0x1.ffffffffffc46p-2,
    0x1.e8b497c65d2fap+3, 0x1.ffffffffffc2ep-2, 0x1.e84e20fb09743p+3, 0x1.ffffffffffc15p-2,
    0x1.e7e7aa2fb5b8cp+3, 0x1.ffffffffffbfbp-2, 0x1.e781336461fd5p+3, 0x1.ffffffffffbe1p-2,
    0x1.e71abc990e41ep+3, 0x1.ffffffffffbc7p-2, 0x1.e6b445cdba868p+3, 0x1.ffffffffffbabp-2,
    0x1.e64dcf0266cb1p+3, 0x1.ffffffffffb8fp-2, 0x1.e5e75837130fap+3, 0x1.ffffffffffb72p-2,
    0x1.e580e16bbf544p+3, 0x1.ffffffffffb55p-2, 0x1.e51a6aa06b98dp+3, 0x1.ffffffffffb37p-2,
    0x1.e4b3f3d517dd6p+3, 0x1.ffffffffffb18p-2, 0x1.e44d7d09c4220p+3, 0x1.ffffffffffaf8p-2,
    0x1.e3e7063e70669p+3, 0x1.ffffffffffad7p-2, 0x1.e3808f731cab2p+3, 0x1.ffffffffffab6p-2,
    0x1.e31a18a7c8efcp+3, 0x1.ffffffffffa93p-2, 0x1.e2b3a1dc75345p+3, 0x1.ffffffffffa70p-2,
    0x1.e24d2b112178fp+3, 0x1.ffffffffffa4cp-2, 0x1.e1e6b445cdbd8p+3, 0x1.ffffffffffa27p-2,
    0x1.e1803d7a7a022p+3, 0x1.ffffffffffa01p-2, 0x1.e119c6af2646bp+3, 0x1.ffffffffff9dap-2,
    0x1.e0b34fe3d28b5p+3, 0x1.ffffffffff9b2p-2, 0x1.e04cd9187ecffp+3, 0x1.ffffffffff98ap-2,
    0x1.dfe6624d2b148p+3, 0x1.ffffffffff960p-2, 0x1.df7feb81d7592p+3, 0x1.ffffffffff935p-2,
    0x1.df1974b6839dcp+3, 0x1.ffffffffff909p-2, 0x1.deb2fdeb2fe25p+3, 0x1.ffffffffff8dcp-2,
    0x1.de4c871fdc26fp+3, 0x1.ffffffffff8adp-2, 0x1.dde61054886b9p+3, 0x1.ffffffffff87ep-2,
    0x1.dd7f998934b03p+3, 0x1.ffffffffff84dp-2, 0x1.dd1922bde0f4dp+3, 0x1.ffffffffff81bp-2,
    0x1.dcb2abf28d397p+3, 0x1.ffffffffff7e8p-2, 0x1.dc4c3527397e1p+3, 0x1.ffffffffff7b3p-2,
    0x1.dbe5be5be5c2bp+3, 0x1.ffffffffff77ep-2, 0x1.db7f479092075p+3, 0x1.ffffffffff746p-2,
    0x1.db18d0c53e4bfp+3, 0x1.ffffffffff70ep-2, 0x1.dab259f9ea909p+3, 0x1.ffffffffff6d4p-2,
    0x1.da4be32e96d54p+3, 0x1.ffffffffff698p-2, 0x1.d9e56c634319ep+3, 0x1.ffffffffff65bp-2,
    0x1.d97ef597ef5e8p+3, 0x1.ffffffffff61dp-2, 0x1.d9187ecc9ba33p+3, 0x1.ffffffffff5ddp-2,
    0x1.d8b2080147e7dp+3, 0x1.ffffffffff59bp-2, 0x1.d84b9135f42c7p+3, 0x1.ffffffffff558p-2,
    0x1.d7e51a6aa0712p+3, 0x1.ffffffffff512p-2, 0x1.d77ea39f4cb5dp+3, 0x1.ffffffffff4ccp-2,
    0x1.d7182cd3f8fa7p+3, 0x1.ffffffffff483p-2, 0x1.d6b1b608a53f2p+3, 0x1.ffffffffff438p-2,
    0x1.d64b3f3d5183dp+3, 0x1.ffffffffff3ecp-2, 0x1.d5e4c871fdc87p+3, 0x1.ffffffffff39ep-2,
    0x1.d57e51a6aa0d2p+3, 0x1.ffffffffff34dp-2, 0x1.d517dadb5651dp+3, 0x1.ffffffffff2fbp-2,
    0x1.d4b1641002968p+3, 0x1.ffffffffff2a7p-2, 0x1.d44aed44aedb3p+3, 0x1.ffffffffff250p-2,
    0x1.d3e476795b1fep+3, 0x1.ffffffffff1f7p-2, 0x1.d37dffae0764ap+3, 0x1.ffffffffff19cp-2,
    0x1.d31788e2b3a95p+3, 0x1.ffffffffff13fp-2, 0x1.d2b112175fee0p+3, 0x1.ffffffffff0dfp-2,
    0x1.d24a9b4c0c32cp+3, 0x1.ffffffffff07dp-2, 0x1.d1e42480b8777p+3, 0x1.ffffffffff019p-2,
    0x1.d17dadb564bc3p+3, 0x1.fffffffffefb1p-2, 0x1.d11736ea1100ep+3, 0x1.fffffffffef48p-2,
    0x1.d0b0c01ebd45ap+3, 0x1.fffffffffeedbp-2, 0x1.d04a4953698a6p+3, 0x1.fffffffffee6cp-2,
    0x1.cfe3d28815cf2p+3, 0x1.fffffffffedfap-2, 0x1.cf7d5bbcc213ep+3, 0x1.fffffffffed85p-2,
    0x1.cf16e4f16e58ap+3, 0x1.fffffffffed0dp-2, 0x1.ceb06e261a9d6p+3, 0x1.fffffffffec93p-2,
    0x1.ce49f75ac6e23p+3, 0x1.fffffffffec15p-2, 0x1.cde3808f7326fp+3, 0x1.fffffffffeb93p-2,
    0x1.cd7d09c41f6bcp+3, 0x1.fffffffffeb0fp-2, 0x1.cd1692f8cbb08p+3, 0x1.fffffffffea87p-2,
    0x1.ccb01c2d77f55p+3, 0x1.fffffffffe9fcp-2, 0x1.cc49a562243a2p+3, 0x1.fffffffffe96dp-2,
    0x1.cbe32e96d07efp+3, 0x1.fffffffffe8dbp-2, 0x1.cb7cb7cb7cc3cp+3, 0x1.fffffffffe845p-2,
    0x1.cb16410029089p+3, 0x1.fffffffffe7abp-2, 0x1.caafca34d54d6p+3, 0x1.fffffffffe70dp-2,
    0x1.ca49536981924p+3, 0x1.fffffffffe66bp-2, 0x1.c9e2dc9e2dd71p+3, 0x1.fffffffffe5c5p-2,
    0x1.c97c65d2da1bfp+3, 0x1.fffffffffe51bp-2, 0x1.c915ef078660dp+3, 0x1.fffffffffe46dp-2,
    0x1.c8af783c32a5bp+3, 0x1.fffffffffe3bap-2, 0x1.c8490170deea9p+3, 0x1.fffffffffe303p-2,
    0x1.c7e28aa58b2f7p+3, 0x1.fffffffffe247p-2, 0x1.c77c13da37745p+3, 0x1.fffffffffe186p-2,
    0x1.c7159d0ee3b94p+3, 0x1.fffffffffe0c0p-2, 0x1.c6af26438ffe3p+3, 0x1.fffffffffdff6p-2,
    0x1.c648af783c431p+3, 0x1.fffffffffdf26p-2, 0x1.c5e238ace8880p+3, 0x1.fffffffffde51p-2,
    0x1.c57bc1e194cd0p+3, 0x1.fffffffffdd76p-2, 0x1.c5154b164111fp+3, 0x1.fffffffffdc96p-2,
    0x1.c4aed44aed56fp+3, 0x1.fffffffffdbb1p-2, 0x1.c4485d7f999bep+3, 0x1.fffffffffdac5p-2,
    0x1.c3e1e6b445e0ep+3, 0x1.fffffffffd9d4p-2, 0x1.c37b6fe8f225ep+3, 0x1.fffffffffd8dcp-2,
    0x1.c314f91d9e6afp+3, 0x1.fffffffffd7dep-2, 0x1.c2ae82524aaffp+3, 0x1.fffffffffd6dap-2,
    0x1.c2480b86f6f50p+3, 0x1.fffffffffd5cfp-2, 0x1.c1e194bba33a1p+3, 0x1.fffffffffd4bep-2,
    0x1.c17b1df04f7f2p+3, 0x1.fffffffffd3a5p-2, 0x1.c114a724fbc43p+3, 0x1.fffffffffd286p-2,
    0x1.c0ae3059a8095p+3, 0x1.fffffffffd15fp-2, 0x1.c047b98e544e7p+3, 0x1.fffffffffd030p-2,
    0x1.bfe142c300939p+3, 0x1.fffffffffcefap-2, 0x1.bf7acbf7acd8bp+3, 0x1.fffffffffcdbcp-2,
    0x1.bf14552c591ddp+3, 0x1.fffffffffcc76p-2, 0x1.beadde6105630p+3, 0x1.fffffffffcb28p-2,
    0x1.be476795b1a83p+3, 0x1.fffffffffc9d2p-2, 0x1.bde0f0ca5ded7p+3, 0x1.fffffffffc872p-2,
    0x1.bd7a79ff0a32ap+3, 0x1.fffffffffc70ap-2, 0x1.bd140333b677ep+3, 0x1.fffffffffc599p-2,
    0x1.bcad8c6862bd2p+3, 0x1.fffffffffc41ep-2, 0x1.bc47159d0f027p+3, 0x1.fffffffffc29ap-2,
    0x1.bbe09ed1bb47cp+3, 0x1.fffffffffc10bp-2, 0x1.bb7a2806678d1p+3, 0x1.fffffffffbf73p-2,
    0x1.bb13b13b13d26p+3, 0x1.fffffffffbdd0p-2, 0x1.baad3a6fc017cp+3, 0x1.fffffffffbc23p-2,
    0x1.ba46c3a46c5d2p+3, 0x1.fffffffffba6bp-2, 0x1.b9e04cd918a29p+3, 0x1.fffffffffb8a8p-2,
    0x1.b979d60dc4e7fp+3, 0x1.fffffffffb6d9p-2, 0x1.b9135f42712d7p+3, 0x1.fffffffffb4ffp-2,
    0x1.b8ace8771d72ep+3, 0x1.fffffffffb319p-2, 0x1.b84671abc9b86p+3, 0x1.fffffffffb126p-2,
    0x1.b7dffae075fdep+3, 0x1.fffffffffaf27p-2, 0x1.b779841522437p+3, 0x1.fffffffffad1ap-2,
    0x1.b7130d49ce890p+3, 0x1.fffffffffab01p-2, 0x1.b6ac967e7aceap+3, 0x1.fffffffffa8dap-2,
    0x1.b6461fb327144p+3, 0x1.fffffffffa6a4p-2, 0x1.b5dfa8e7d359ep+3, 0x1.fffffffffa461p-2,
    0x1.b579321c7f9f9p+3, 0x1.fffffffffa20fp-2, 0x1.b512bb512be55p+3, 0x1.fffffffff9faep-2,
    0x1.b4ac4485d82b1p+3, 0x1.fffffffff9d3dp-2, 0x1.b445cdba8470dp+3, 0x1.fffffffff9abcp-2,
    0x1.b3df56ef30b6ap+3, 0x1.fffffffff982cp-2, 0x1.b378e023dcfc7p+3, 0x1.fffffffff958bp-2,
    0x1.b312695889425p+3, 0x1.fffffffff92d8p-2, 0x1.b2abf28d35884p+3, 0x1.fffffffff9014p-2,
    0x1.b2457bc1e1ce3p+3, 0x1.fffffffff8d3fp-2, 0x1.b1df04f68e142p+3, 0x1.fffffffff8a56p-2,
    0x1.b1788e2b3a5a3p+3, 0x1.fffffffff875bp-2, 0x1.b112175fe6a03p+3, 0x1.fffffffff844dp-2,
    0x1.b0aba09492e65p+3, 0x1.fffffffff812bp-2, 0x1.b04529c93f2c7p+3, 0x1.fffffffff7df4p-2,
    0x1.afdeb2fdeb72ap+3, 0x1.fffffffff7aa9p-2, 0x1.af783c3297b8dp+3, 0x1.fffffffff7748p-2,
    0x1.af11c56743ff1p+3, 0x1.fffffffff73d2p-2, 0x1.aeab4e9bf0456p+3, 0x1.fffffffff7045p-2,
    0x1.ae44d7d09c8bbp+3, 0x1.fffffffff6ca1p-2, 0x1.adde610548d22p+3, 0x1.fffffffff68e5p-2,
    0x1.ad77ea39f5189p+3, 0x1.fffffffff6511p-2, 0x1.ad11736ea15f0p+3, 0x1.fffffffff6124p-2,
    0x1.acaafca34da59p+3, 0x1.fffffffff5d1ep-2, 0x1.ac4485d7f9ec2p+3, 0x1.fffffffff58fep-2,
    0x1.abde0f0ca632dp+3, 0x1.fffffffff54c3p-2, 0x1.ab77984152798p+3, 0x1.fffffffff506dp-2,
    0x1.ab112175fec04p+3, 0x1.fffffffff4bfap-2, 0x1.aaaaaaaaab070p+3, 0x1.fffffffff476bp-2,
    0x1.aa4433df574dep+3, 0x1.fffffffff42bep-2, 0x1.a9ddbd140394dp+3, 0x1.fffffffff3df2p-2,
    0x1.a9774648afdbdp+3, 0x1.fffffffff3908p-2, 0x1.a910cf7d5c22dp+3, 0x1.fffffffff33fep-2,
    0x1.a8aa58b20869fp+3, 0x1.fffffffff2ed3p-2, 0x1.a843e1e6b4b12p+3, 0x1.fffffffff2986p-2,
    0x1.a7dd6b1b60f86p+3, 0x1.fffffffff2417p-2, 0x1.a776f4500d3fap+3, 0x1.fffffffff1e85p-2,
    0x1.a7107d84b9871p+3, 0x1.fffffffff18cfp-2, 0x1.a6aa06b965ce8p+3, 0x1.fffffffff12f4p-2,
    0x1.a6438fee12160p+3, 0x1.fffffffff0cf3p-2, 0x1.a5dd1922be5dap+3, 0x1.fffffffff06cbp-2,
    0x1.a576a2576aa55p+3, 0x1.fffffffff007ap-2, 0x1.a5102b8c16ed1p+3, 0x1.ffffffffefa01p-2,
    0x1.a4a9b4c0c334ep+3, 0x1.ffffffffef35fp-2, 0x1.a4433df56f7cdp+3, 0x1.ffffffffeec90p-2,
    0x1.a3dcc72a1bc4dp+3, 0x1.ffffffffee596p-2, 0x1.a376505ec80cfp+3, 0x1.ffffffffede6fp-2,
    0x1.a30fd99374552p+3, 0x1.ffffffffed719p-2, 0x1.a2a962c8209d6p+3, 0x1.ffffffffecf94p-2,
    0x1.a242ebfccce5cp+3, 0x1.ffffffffec7dep-2, 0x1.a1dc7531792e4p+3, 0x1.ffffffffebff6p-2,
    0x1.a175fe662576dp+3, 0x1.ffffffffeb7dap-2, 0x1.a10f879ad1bf8p+3, 0x1.ffffffffeaf8ap-2,
    0x1.a0a910cf7e085p+3, 0x1.ffffffffea704p-2, 0x1.a0429a042a513p+3, 0x1.ffffffffe9e47p-2,
    0x1.9fdc2338d69a3p+3, 0x1.ffffffffe9551p-2, 0x1.9f75ac6d82e35p+3, 0x1.ffffffffe8c22p-2,
    0x1.9f0f35a22f2c9p+3, 0x1.ffffffffe82b6p-2, 0x1.9ea8bed6db75ep+3, 0x1.ffffffffe790dp-2,
    0x1.9e42480b87bf6p+3, 0x1.ffffffffe6f26p-2, 0x1.9ddbd1403408fp+3, 0x1.ffffffffe64ffp-2,
    0x1.9d755a74e052bp+3, 0x1.ffffffffe5a96p-2, 0x1.9d0ee3a98c9c9p+3, 0x1.ffffffffe4fe9p-2,
    0x1.9ca86cde38e69p+3, 0x1.ffffffffe44f7p-2, 0x1.9c41f612e530bp+3, 0x1.ffffffffe39bep-2,
    0x1.9bdb7f47917afp+3, 0x1.ffffffffe2e3cp-2, 0x1.9b75087c3dc56p+3, 0x1.ffffffffe2270p-2,
    0x1.9b0e91b0ea0ffp+3, 0x1.ffffffffe1657p-2, 0x1.9aa81ae5965abp+3, 0x1.ffffffffe09efp-2,
    0x1.9a41a41a42a59p+3, 0x1.ffffffffdfd38p-2, 0x1.99db2d4eeef0ap+3, 0x1.ffffffffdf02dp-2,
    0x1.9974b6839b3bdp+3, 0x1.ffffffffde2cfp-2, 0x1.990e3fb847873p+3, 0x1.ffffffffdd519p-2,
    0x1.98a7c8ecf3d2cp+3, 0x1.ffffffffdc70bp-2, 0x1.98415221a01e7p+3, 0x1.ffffffffdb8a1p-2,
    0x1.97dadb564c6a6p+3, 0x1.ffffffffda9dap-2, 0x1.9774648af8b68p+3, 0x1.ffffffffd9ab3p-2,
    0x1.970dedbfa502cp+3, 0x1.ffffffffd8b2ap-2, 0x1.96a776f4514f4p+3, 0x1.ffffffffd7b3cp-2,
    0x1.96410028fd9bfp+3, 0x1.ffffffffd6ae7p-2, 0x1.95da895da9e8dp+3, 0x1.ffffffffd5a28p-2,
    0x1.957412925635fp+3, 0x1.ffffffffd48fcp-2, 0x1.950d9bc702834p+3, 0x1.ffffffffd3761p-2,
    0x1.94a724fbaed0dp+3, 0x1.ffffffffd2554p-2, 0x1.9440ae305b1eap+3, 0x1.ffffffffd12d2p-2,
    0x1.93da3765076cap+3, 0x1.ffffffffcffd8p-2, 0x1.9373c099b3baep+3, 0x1.ffffffffcec62p-2,
    0x1.930d49ce60096p+3, 0x1.ffffffffcd86fp-2, 0x1.92a6d3030c582p+3, 0x1.ffffffffcc3fap-2,
    0x1.92405c37b8a72p+3, 0x1.ffffffffcaf00p-2, 0x1.91d9e56c64f66p+3, 0x1.ffffffffc997fp-2,
    0x1.91736ea11145fp+3, 0x1.ffffffffc8372p-2, 0x1.910cf7d5bd95cp+3, 0x1.ffffffffc6cd6p-2,
    0x1.90a6810a69e5ep+3, 0x1.ffffffffc55a7p-2, 0x1.90400a3f16365p+3, 0x1.ffffffffc3de2p-2,
    0x1.8fd99373c2870p+3, 0x1.ffffffffc2583p-2, 0x1.8f731ca86ed80p+3, 0x1.ffffffffc0c86p-2,
    0x1.8f0ca5dd1b296p+3, 0x1.ffffffffbf2e7p-2, 0x1.8ea62f11c77b0p+3, 0x1.ffffffffbd8a1p-2,
    0x1.8e3fb84673cd0p+3, 0x1.ffffffffbbdb2p-2, 0x1.8dd9417b201f5p+3, 0x1.ffffffffba213p-2,
    0x1.8d72caafcc720p+3, 0x1.ffffffffb85c2p-2, 0x1.8d0c53e478c51p+3, 0x1.ffffffffb68b9p-2,
    0x1.8ca5dd1925187p+3, 0x1.ffffffffb4af3p-2, 0x1.8c3f664dd16c4p+3, 0x1.ffffffffb2c6dp-2,
    0x1.8bd8ef827dc07p+3, 0x1.ffffffffb0d20p-2, 0x1.8b7278b72a150p+3, 0x1.ffffffffaed09p-2,
    0x1.8b0c01ebd669fp+3, 0x1.ffffffffacc21p-2, 0x1.8aa58b2082bf6p+3, 0x1.ffffffffaaa65p-2,
    0x1.8a3f14552f153p+3, 0x1.ffffffffa87cdp-2, 0x1.89d89d89db6b7p+3, 0x1.ffffffffa6455p-2,
    0x1.897226be87c22p+3, 0x1.ffffffffa3ff7p-2, 0x1.890baff334195p+3, 0x1.ffffffffa1aadp-2,
    0x1.88a53927e070fp+3, 0x1.ffffffff9f472p-2, 0x1.883ec25c8cc91p+3, 0x1.ffffffff9cd3ep-2,
    0x1.87d84b913921bp+3, 0x1.ffffffff9a50cp-2, 0x1.8771d4c5e57adp+3, 0x1.ffffffff97bd6p-2,
    0x1.870b5dfa91d47p+3, 0x1.ffffffff95194p-2, 0x1.86a4e72f3e2eap+3, 0x1.ffffffff92640p-2,
    0x1.863e7063ea896p+3, 0x1.ffffffff8f9d4p-2, 0x1.85d7f99896e4bp+3, 0x1.ffffffff8cc47p-2,
    0x1.857182cd43409p+3, 0x1.ffffffff89d93p-2, 0x1.850b0c01ef9d0p+3, 0x1.ffffffff86db0p-2,
    0x1.84a495369bfa2p+3, 0x1.ffffffff83c96p-2, 0x1.843e1e6b4857dp+3, 0x1.ffffffff80a3ep-2,
    0x1.83d7a79ff4b62p+3, 0x1.ffffffff7d6a0p-2, 0x1.837130d4a1152p+3, 0x1.ffffffff7a1b3p-2,
    0x1.830aba094d74cp+3, 0x1.ffffffff76b6fp-2, 0x1.82a4433df9d52p+3, 0x1.ffffffff733cap-2,
    0x1.823dcc72a6363p+3, 0x1.ffffffff6fabdp-2, 0x1.81d755a75297fp+3, 0x1.ffffffff6c03ep-2,
    0x1.8170dedbfefa7p+3, 0x1.ffffffff68444p-2, 0x1.810a6810ab5dbp+3, 0x1.ffffffff646c5p-2,
    0x1.80a3f14557c1cp+3, 0x1.ffffffff607b6p-2, 0x1.803d7a7a0426ap+3, 0x1.ffffffff5c70fp-2,
    0x1.7fd703aeb08c5p+3, 0x1.ffffffff584c5p-2, 0x1.7f708ce35cf2dp+3, 0x1.ffffffff540cdp-2,
    0x1.7f0a1618095a3p+3, 0x1.ffffffff4fb1cp-2, 0x1.7ea39f4cb5c27p+3, 0x1.ffffffff4b3a7p-2,
    0x1.7e3d2881622b9p+3, 0x1.ffffffff46a63p-2, 0x1.7dd6b1b60e95ap+3, 0x1.ffffffff41f44p-2,
    0x1.7d703aeabb00bp+3, 0x1.ffffffff3d23dp-2, 0x1.7d09c41f676cbp+3, 0x1.ffffffff38343p-2,
    0x1.7ca34d5413d9bp+3, 0x1.ffffffff33249p-2, 0x1.7c3cd688c047cp+3, 0x1.ffffffff2df42p-2,
    0x1.7bd65fbd6cb6dp+3, 0x1.ffffffff28a20p-2, 0x1.7b6fe8f219270p+3, 0x1.ffffffff232d6p-2,
    0x1.7b097226c5984p+3, 0x1.ffffffff1d957p-2, 0x1.7aa2fb5b720abp+3, 0x1.ffffffff17d93p-2,
    0x1.7a3c84901e7e4p+3, 0x1.ffffffff11f7bp-2, 0x1.79d60dc4caf30p+3, 0x1.ffffffff0bf02p-2,
    0x1.796f96f977690p+3, 0x1.ffffffff05c17p-2, 0x1.7909202e23e04p+3, 0x1.fffffffeff6abp-2,
    0x1.78a2a962d058cp+3, 0x1.fffffffef8eacp-2, 0x1.783c32977cd29p+3, 0x1.fffffffef240cp-2,
    0x1.77d5bbcc294dcp+3, 0x1.fffffffeeb6b8p-2, 0x1.776f4500d5ca5p+3, 0x1.fffffffee469fp-2,
    0x1.7708ce3582485p+3, 0x1.fffffffedd3afp-2, 0x1.76a2576a2ec7cp+3, 0x1.fffffffed5dd6p-2,
    0x1.763be09edb48bp+3, 0x1.fffffffece500p-2, 0x1.75d569d387cb3p+3, 0x1.fffffffec691bp-2,
    0x1.756ef308344f4p+3, 0x1.fffffffebea13p-2, 0x1.75087c3ce0d4ep+3, 0x1.fffffffeb67d3p-2,
    0x1.74a205718d5c3p+3, 0x1.fffffffeae246p-2, 0x1.743b8ea639e53p+3, 0x1.fffffffea5957p-2,
    0x1.73d517dae66fep+3, 0x1.fffffffe9ccf0p-2, 0x1.736ea10f92fc6p+3, 0x1.fffffffe93cfbp-2,
    0x1.73082a443f8abp+3, 0x1.fffffffe8a960p-2, 0x1.72a1b378ec1aep+3, 0x1.fffffffe81207p-2,
    0x1.723b3cad98ad0p+3, 0x1.fffffffe776dap-2, 0x1.71d4c5e245411p+3, 0x1.fffffffe6d7bep-2,
    0x1.716e4f16f1d73p+3, 0x1.fffffffe6349bp-2, 0x1.7107d84b9e6f5p+3, 0x1.fffffffe58d55p-2,
    0x1.70a161804b09ap+3, 0x1.fffffffe4e1d3p-2, 0x1.703aeab4f7a61p+3, 0x1.fffffffe431f8p-2,
    0x1.6fd473e9a444cp+3, 0x1.fffffffe37da9p-2, 0x1.6f6dfd1e50e5bp+3, 0x1.fffffffe2c4c9p-2,
    0x1.6f078652fd890p+3, 0x1.fffffffe2073ap-2, 0x1.6ea10f87aa2ebp+3, 0x1.fffffffe144dep-2,
    0x1.6e3a98bc56d6ep+3, 0x1.fffffffe07d96p-2, 0x1.6dd421f103819p+3, 0x1.fffffffdfb141p-2,
    0x1.6d6dab25b02edp+3, 0x1.fffffffdedfbfp-2, 0x1.6d07345a5cdecp+3, 0x1.fffffffde08eep-2,
    0x1.6ca0bd8f09917p+3, 0x1.fffffffdd2cadp-2, 0x1.6c3a46c3b646ep+3, 0x1.fffffffdc4ad7p-2,
    0x1.6bd3cff862ff3p+3, 0x1.fffffffdb6348p-2, 0x1.6b6d592d0fba6p+3, 0x1.fffffffda75dcp-2,
    0x1.6b06e261bc78ap+3, 0x1.fffffffd9826dp-2, 0x1.6aa06b966939fp+3, 0x1.fffffffd888d3p-2,
    0x1.6a39f4cb15fe7p+3, 0x1.fffffffd788e6p-2, 0x1.69d37dffc2c63p+3, 0x1.fffffffd6827dp-2,
    0x1.696d07346f914p+3, 0x1.fffffffd5756fp-2, 0x1.690690691c5fbp+3, 0x1.fffffffd46190p-2,
    0x1.68a0199dc931ap+3, 0x1.fffffffd346b5p-2, 0x1.6839a2d276073p+3, 0x1.fffffffd224afp-2,
    0x1.67d32c0722e06p+3, 0x1.fffffffd0fb50p-2, 0x1.676cb53bcfbd6p+3, 0x1.fffffffcfca69p-2,
    0x1.67063e707c9e3p+3, 0x1.fffffffce91c8p-2, 0x1.669fc7a529830p+3, 0x1.fffffffcd513cp-2,
    0x1.663950d9d66bdp+3, 0x1.fffffffcc0892p-2, 0x1.65d2da0e8358ep+3, 0x1.fffffffcab794p-2,
    0x1.656c6343304a2p+3, 0x1.fffffffc95e0dp-2, 0x1.6505ec77dd3fdp+3, 0x1.fffffffc7fbc5p-2,
    0x1.649f75ac8a39fp+3, 0x1.fffffffc69084p-2, 0x1.6438fee13738bp+3, 0x1.fffffffc51c0fp-2,
    0x1.63d28815e43c3p+3, 0x1.fffffffc39e2bp-2, 0x1.636c114a91448p+3, 0x1.fffffffc2169bp-2,
    0x1.63059a7f3e51cp+3, 0x1.fffffffc0851fp-2, 0x1.629f23b3eb642p+3, 0x1.fffffffbee978p-2,
    0x1.6238ace8987bbp+3, 0x1.fffffffbd4363p-2, 0x1.61d2361d45989p+3, 0x1.fffffffbb929dp-2,
    0x1.616bbf51f2bafp+3, 0x1.fffffffb9d6e1p-2, 0x1.610548869fe30p+3, 0x1.fffffffb80fe7p-2,
    0x1.609ed1bb4d10cp+3, 0x1.fffffffb63d67p-2, 0x1.60385aeffa447p+3, 0x1.fffffffb45f15p-2,
    0x1.5fd1e424a77e3p+3, 0x1.fffffffb274a6p-2, 0x1.5f6b6d5954be2p+3, 0x1.fffffffb07dcbp-2,
    0x1.5f04f68e02047p+3, 0x1.fffffffae7a32p-2, 0x1.5e9e7fc2af515p+3, 0x1.fffffffac698ap-2,
    0x1.5e3808f75ca4dp+3, 0x1.fffffffaa4b7ep-2, 0x1.5dd1922c09ff4p+3, 0x1.fffffffa81fb7p-2,
    0x1.5d6b1b60b760bp+3, 0x1.fffffffa5e5dbp-2, 0x1.5d04a49564c96p+3, 0x1.fffffffa39d91p-2,
    0x1.5c9e2dca12397p+3, 0x1.fffffffa14679p-2, 0x1.5c37b6febfb11p+3, 0x1.fffffff9ee034p-2,
    0x1.5bd140336d308p+3, 0x1.fffffff9c6a60p-2, 0x1.5b6ac9681ab7fp+3, 0x1.fffffff99e498p-2,
    0x1.5b04529cc8479p+3, 0x1.fffffff974e73p-2, 0x1.5a9ddbd175df8p+3, 0x1.fffffff94a789p-2,
    0x1.5a37650623802p+3, 0x1.fffffff91ef6dp-2, 0x1.59d0ee3ad1298p+3, 0x1.fffffff8f25aep-2,
    0x1.596a776f7edbfp+3, 0x1.fffffff8c49dbp-2, 0x1.590400a42c97ap+3, 0x1.fffffff895b7ep-2,
    0x1.589d89d8da5cdp+3, 0x1.fffffff865a1fp-2, 0x1.5837130d882bdp+3, 0x1.fffffff834543p-2,
    0x1.57d09c423604cp+3, 0x1.fffffff801c6bp-2, 0x1.576a2576e3e7fp+3, 0x1.fffffff7cdf17p-2,
    0x1.5703aeab91d5ap+3, 0x1.fffffff798cc0p-2, 0x1.569d37e03fce1p+3, 0x1.fffffff7624dfp-2,
    0x1.5636c114edd19p+3, 0x1.fffffff72a6e8p-2, 0x1.55d04a499be07p+3, 0x1.fffffff6f124bp-2,
    0x1.5569d37e49faep+3, 0x1.fffffff6b6677p-2, 0x1.55035cb2f8213p+3, 0x1.fffffff67a2d4p-2,
    0x1.549ce5e7a653cp+3, 0x1.fffffff63c6c9p-2, 0x1.54366f1c5492dp+3, 0x1.fffffff5fd1b6p-2,
    0x1.53cff85102debp+3, 0x1.fffffff5bc2f9p-2, 0x1.53698185b137cp+3, 0x1.fffffff5799edp-2,
    0x1.53030aba5f9e4p+3, 0x1.fffffff5355e6p-2, 0x1.529c93ef0e12ap+3, 0x1.fffffff4ef635p-2,
    0x1.52361d23bc953p+3, 0x1.fffffff4a7a27p-2, 0x1.51cfa6586b264p+3, 0x1.fffffff45e105p-2,
    0x1.51692f8d19c64p+3, 0x1.fffffff412a11p-2, 0x1.5102b8c1c8759p+3, 0x1.fffffff3c548ap-2,
    0x1.509c41f677348p+3, 0x1.fffffff375faap-2, 0x1.5035cb2b26039p+3, 0x1.fffffff324aa6p-2,
    0x1.4fcf545fd4e31p+3, 0x1.fffffff2d14adp-2, 0x1.4f68dd9483d37p+3, 0x1.fffffff27bceap-2,
    0x1.4f0266c932d53p+3, 0x1.fffffff224280p-2, 0x1.4e9beffde1e8bp+3, 0x1.fffffff1ca491p-2,
    0x1.4e357932910e6p+3, 0x1.fffffff16e235p-2, 0x1.4dcf02674046cp+3, 0x1.fffffff10fa80p-2,
    0x1.4d688b9bef925p+3, 0x1.fffffff0aec80p-2, 0x1.4d0214d09ef17p+3, 0x1.fffffff04b73cp-2,
    0x1.4c9b9e054e64cp+3, 0x1.ffffffefe59b6p-2, 0x1.4c352739fdecap+3, 0x1.ffffffef7d2eap-2,
    0x1.4bceb06ead89cp+3, 0x1.ffffffef121cap-2, 0x1.4b6839a35d3c8p+3, 0x1.ffffffeea4546p-2,
    0x1.4b01c2d80d059p+3, 0x1.ffffffee33c43p-2, 0x1.4a9b4c0cbce56p+3, 0x1.ffffffedc05a0p-2,
    0x1.4a34d5416cdcap+3, 0x1.ffffffed4a037p-2, 0x1.49ce5e761cebdp+3, 0x1.ffffffecd0ad7p-2,
    0x1.4967e7aacd13ap+3, 0x1.ffffffec5444ap-2, 0x1.490170df7d54ap+3, 0x1.ffffffebd4b51p-2,
    0x1.489afa142daf8p+3, 0x1.ffffffeb51ea4p-2, 0x1.48348348de24ep+3, 0x1.ffffffeacbcf5p-2,
    0x1.47ce0c7d8eb56p+3, 0x1.ffffffea424ebp-2, 0x1.476795b23f61dp+3, 0x1.ffffffe9b5527p-2,
    0x1.47011ee6f02acp+3, 0x1.ffffffe924c3fp-2, 0x1.469aa81ba1111p+3, 0x1.ffffffe8908c0p-2,
    0x1.4634315052156p+3, 0x1.ffffffe7f892ep-2, 0x1.45cdba8503387p+3, 0x1.ffffffe75cc04p-2,
    0x1.456743b9b47b2p+3, 0x1.ffffffe6bcfb3p-2, 0x1.4500ccee65de3p+3, 0x1.ffffffe6192a0p-2,
    0x1.449a562317627p+3, 0x1.ffffffe571329p-2, 0x1.4433df57c908cp+3, 0x1.ffffffe4c4f9dp-2,
    0x1.43cd688c7ad1fp+3, 0x1.ffffffe414645p-2, 0x1.4366f1c12cbefp+3, 0x1.ffffffe35f55bp-2,
    0x1.43007af5ded0ap+3, 0x1.ffffffe2a5b0fp-2, 0x1.429a042a9107ep+3, 0x1.ffffffe1e7586p-2,
    0x1.42338d5f4365cp+3, 0x1.ffffffe1242d6p-2, 0x1.41cd1693f5eb3p+3, 0x1.ffffffe05c10dp-2,
    0x1.41669fc8a8992p+3, 0x1.ffffffdf8ee29p-2, 0x1.410028fd5b70bp+3, 0x1.ffffffdebc81cp-2,
    0x1.4099b2320e72ep+3, 0x1.ffffffdde4cccp-2, 0x1.40333b66c1a0cp+3, 0x1.ffffffdd07a0ep-2,
    0x1.3fccc49b74fb8p+3, 0x1.ffffffdc24dacp-2, 0x1.3f664dd028842p+3, 0x1.ffffffdb3c561p-2,
    0x1.3effd704dc3bfp+3, 0x1.ffffffda4ded9p-2, 0x1.3e99603990241p+3, 0x1.ffffffd9597b0p-2,
    0x1.3e32e96e443dbp+3, 0x1.ffffffd85ed74p-2, 0x1.3dcc72a2f88a2p+3, 0x1.ffffffd75dda3p-2,
    0x1.3d65fbd7ad0aap+3, 0x1.ffffffd6565aap-2, 0x1.3cff850c61c08p+3, 0x1.ffffffd5482e5p-2,
    0x1.3c990e4116ad3p+3, 0x1.ffffffd4332a0p-2, 0x1.3c329775cbd20p+3, 0x1.ffffffd317214p-2,
    0x1.3bcc20aa81305p+3, 0x1.ffffffd1f3e6ap-2, 0x1.3b65a9df36c9bp+3, 0x1.ffffffd0c94b8p-2,
    0x1.3aff3313ec9f9p+3, 0x1.ffffffcf971ffp-2, 0x1.3a98bc48a2b38p+3, 0x1.ffffffce5d32fp-2,
    0x1.3a32457d59071p+3, 0x1.ffffffcd1b523p-2, 0x1.39cbceb20f9bdp+3, 0x1.ffffffcbd14a2p-2,
    0x1.396557e6c6738p+3, 0x1.ffffffca7ee5ep-2, 0x1.38fee11b7d8fcp+3, 0x1.ffffffc923ef4p-2,
    0x1.38986a5034f24p+3, 0x1.ffffffc7c02ebp-2, 0x1.3831f384ec9cep+3, 0x1.ffffffc6536b2p-2,
    0x1.37cb7cb9a4917p+3, 0x1.ffffffc4dd6a2p-2, 0x1.376505ee5cd1dp+3, 0x1.ffffffc35defdp-2,
    0x1.36fe8f23155fep+3, 0x1.ffffffc1d4becp-2, 0x1.36981857ce3d9p+3, 0x1.ffffffc04197ep-2,
    0x1.3631a18c876d0p+3, 0x1.ffffffbea43abp-2, 0x1.35cb2ac140f04p+3, 0x1.ffffffbcfc64fp-2,
    0x1.3564b3f5fac95p+3, 0x1.ffffffbb49d2bp-2, 0x1.34fe3d2ab4fa8p+3, 0x1.ffffffb98c3e6p-2,
    0x1.3497c65f6f85fp+3, 0x1.ffffffb7c3609p-2, 0x1.34314f942a6e0p+3, 0x1.ffffffb5eef01p-2,
    0x1.33cad8c8e5b4fp+3, 0x1.ffffffb40ea1dp-2, 0x1.336461fda15d4p+3, 0x1.ffffffb22228fp-2,
    0x1.32fdeb325d695p+3, 0x1.ffffffb029368p-2, 0x1.3297746719dbcp+3, 0x1.ffffffae23799p-2,
    0x1.3230fd9bd6b72p+3, 0x1.ffffffac109f3p-2, 0x1.31ca86d093fe1p+3, 0x1.ffffffa9f0526p-2,
    0x1.3164100551b34p+3, 0x1.ffffffa7c23bfp-2, 0x1.30fd993a0fd99p+3, 0x1.ffffffa586026p-2,
    0x1.3097226ece73ep+3, 0x1.ffffffa33b4a1p-2, 0x1.3030aba38d851p+3, 0x1.ffffffa0e1b51p-2,
    0x1.2fca34d84d102p+3, 0x1.ffffff9e78e2ep-2, 0x1.2f63be0d0d184p+3, 0x1.ffffff9c0070dp-2,
    0x1.2efd4741cda08p+3, 0x1.ffffff9977f97p-2, 0x1.2e96d0768eac2p+3, 0x1.ffffff96df14ep-2,
    0x1.2e3059ab503e9p+3, 0x1.ffffff943558bp-2, 0x1.2dc9e2e0125b2p+3, 0x1.ffffff917a579p-2,
    0x1.2d636c14d5055p+3, 0x1.ffffff8eada19p-2, 0x1.2cfcf5499840cp+3, 0x1.ffffff8bcec3ep-2,
    0x1.2c967e7e5c112p+3, 0x1.ffffff88dd48bp-2, 0x1.2c3007b3207a3p+3, 0x1.ffffff85d8b76p-2,
    0x1.2bc990e7e57fdp+3, 0x1.ffffff82c0943p-2, 0x1.2b631a1cab25fp+3, 0x1.ffffff7f94602p-2,
    0x1.2afca3517170bp+3, 0x1.ffffff7c53992p-2, 0x1.2a962c8638643p+3, 0x1.ffffff78fdb9bp-2,
    0x1.2a2fb5bb0004cp+3, 0x1.ffffff7592392p-2, 0x1.29c93eefc856bp+3, 0x1.ffffff72108b2p-2,
    0x1.2962c824915e9p+3, 0x1.ffffff6e781fep-2, 0x1.28fc51595b210p+3, 0x1.ffffff6ac863fp-2,
    0x1.2895da8e25a2ap+3, 0x1.ffffff6700c01p-2, 0x1.282f63c2f0e86p+3, 0x1.ffffff6320995p-2,
    0x1.27c8ecf7bcf73p+3, 0x1.ffffff5f2750ap-2, 0x1.2762762c89d42p+3, 0x1.ffffff5b14432p-2,
    0x1.26fbff6157847p+3, 0x1.ffffff56e6c9ap-2, 0x1.26958896260d8p+3, 0x1.ffffff529e38dp-2,
    0x1.262f11caf574cp+3, 0x1.ffffff4e39e11p-2, 0x1.25c89affc5bfep+3, 0x1.ffffff49b90e3p-2,
    0x1.2562243496f49p+3, 0x1.ffffff451b078p-2, 0x1.24fbad696918ep+3, 0x1.ffffff405f0fbp-2,
    0x1.2495369e3c32cp+3, 0x1.ffffff3b84647p-2, 0x1.242ebfd310487p+3, 0x1.ffffff368a3eep-2,
    0x1.23c84907e5605p+3, 0x1.ffffff316fd2bp-2, 0x1.2361d23cbb810p+3, 0x1.ffffff2c344eap-2,
    0x1.22fb5b7192b11p+3, 0x1.ffffff26d6dc2p-2, 0x1.2294e4a66af78p+3, 0x1.ffffff21569f3p-2,
    0x1.222e6ddb445b5p+3, 0x1.ffffff1bb2b61p-2, 0x1.21c7f7101ee3cp+3, 0x1.ffffff15ea399p-2,
    0x1.21618044fa982p+3, 0x1.ffffff0ffc3c7p-2, 0x1.20fb0979d7803p+3, 0x1.ffffff09e7cb7p-2,
    0x1.209492aeb5a3bp+3, 0x1.ffffff03abed5p-2, 0x1.202e1be3950a9p+3, 0x1.fffffefd47a25p-2,
    0x1.1fc7a51875bd0p+3, 0x1.fffffef6b9e46p-2, 0x1.1f612e4d57c37p+3, 0x1.fffffef001a6ap-2,
    0x1.1efab7823b268p+3, 0x1.fffffee91dd58p-2, 0x1.1e9440b71fef0p+3, 0x1.fffffee20d567p-2,
    0x1.1e2dc9ec06260p+3, 0x1.fffffedacf07bp-2, 0x1.1dc75320edd4cp+3, 0x1.fffffed361c02p-2,
    0x1.1d60dc55d704dp+3, 0x1.fffffecbc44f4p-2, 0x1.1cfa658ac1bfep+3, 0x1.fffffec3f57cap-2,
    0x1.1c93eebfae101p+3, 0x1.fffffebbf4082p-2, 0x1.1c2d77f49bff9p+3, 0x1.fffffeb3bea96p-2,
    0x1.1bc701298b98ep+3, 0x1.fffffeab540fcp-2, 0x1.1b608a5e7ce6dp+3, 0x1.fffffea2b2e1fp-2,
    0x1.1afa13936ff48p+3, 0x1.fffffe99d9be3p-2, 0x1.1a939cc864cd2p+3, 0x1.fffffe90c7398p-2,
    0x1.1a2d25fd5b7c7p+3, 0x1.fffffe8779dfcp-2, 0x1.19c6af32540e6p+3, 0x1.fffffe7df0338p-2,
    0x1.196038674e8f1p+3, 0x1.fffffe7428ad9p-2, 0x1.18f9c19c4b0b2p+3, 0x1.fffffe6a21bcep-2,
    0x1.18934ad1498f6p+3, 0x1.fffffe5fd9c62p-2, 0x1.182cd4064a28fp+3, 0x1.fffffe554f23bp-2,
    0x1.17c65d3b4ce57p+3, 0x1.fffffe4a80253p-2, 0x1.175fe67051d2ap+3, 0x1.fffffe3f6b0f6p-2,
    0x1.16f96fa558fecp+3, 0x1.fffffe340e1bcp-2, 0x1.1692f8da62787p+3, 0x1.fffffe2867783p-2,
    0x1.162c820f6e4e8p+3, 0x1.fffffe1c7546ep-2, 0x1.15c60b447c904p+3, 0x1.fffffe10359dep-2,
    0x1.155f94798d4d8p+3, 0x1.fffffe03a686ep-2, 0x1.14f91daea0965p+3, 0x1.fffffdf6c5febp-2,
    0x1.1492a6e3b67b2p+3, 0x1.fffffde991f54p-2, 0x1.142c3018cf0cep+3, 0x1.fffffddc084d1p-2,
    0x1.13c5b94dea5d0p+3, 0x1.fffffdce26dadp-2, 0x1.135f4283087d3p+3, 0x1.fffffdbfeb655p-2,
    0x1.12f8cbb8297fcp+3, 0x1.fffffdb153a4dp-2, 0x1.129254ed4d775p+3, 0x1.fffffda25d42cp-2,
    0x1.122bde2274772p+3, 0x1.fffffd9305d99p-2, 0x1.11c567579e92dp+3, 0x1.fffffd834af40p-2,
    0x1.115ef08ccbde9p+3, 0x1.fffffd732a0cep-2, 0x1.10f879c1fc6f1p+3, 0x1.fffffd62a08edp-2,
    0x1.109202f730597p+3, 0x1.fffffd51abd38p-2, 0x1.102b8c2c67b37p+3, 0x1.fffffd4049238p-2,
    0x1.0fc51561a2936p+3, 0x1.fffffd2e75b5cp-2, 0x1.0f5e9e96e1102p+3, 0x1.fffffd1c2eaf4p-2,
    0x1.0ef827cc23411p+3, 0x1.fffffd0971226p-2, 0x1.0e91b101693e3p+3, 0x1.fffffcf63a0e6p-2,
    0x1.0e2b3a36b3203p+3, 0x1.fffffce2865f5p-2, 0x1.0dc4c36c01005p+3, 0x1.fffffcce52ed2p-2,
    0x1.0d5e4ca152f86p+3, 0x1.fffffcb99c7b4p-2, 0x1.0cf7d5d6a9230p+3, 0x1.fffffca45fb83p-2,
    0x1.0c915f0c039b6p+3, 0x1.fffffc8e993d0p-2, 0x1.0c2ae841627d6p+3, 0x1.fffffc78458c8p-2,
    0x1.0bc47176c5e5cp+3, 0x1.fffffc6161132p-2, 0x1.0b5dfaac2df1bp+3, 0x1.fffffc49e825dp-2,
    0x1.0af783e19abf5p+3, 0x1.fffffc31d7021p-2, 0x1.0a910d170c6d8p+3, 0x1.fffffc1929ccap-2,
    0x1.0a2a964c831bep+3, 0x1.fffffbffdc919p-2, 0x1.09c41f81feeaep+3, 0x1.fffffbe5eb432p-2,
    0x1.095da8b77ffbbp+3, 0x1.fffffbcb51b95p-2, 0x1.08f731ed06707p+3, 0x1.fffffbb00bb13p-2,
    0x1.0890bb22926c2p+3, 0x1.fffffb9414cc3p-2, 0x1.082a445824129p+3, 0x1.fffffb77688f5p-2,
    0x1.07c3cd8dbb888p+3, 0x1.fffffb5a0262bp-2, 0x1.075d56c358f39p+3, 0x1.fffffb3bdd909p-2,
    0x1.06f6dff8fc7a8p+3, 0x1.fffffb1cf5449p-2, 0x1.0690692ea644dp+3, 0x1.fffffafd448b2p-2,
    0x1.0629f264567b3p+3, 0x1.fffffadcc6508p-2, 0x1.05c37b9a0d474p+3, 0x1.fffffabb75600p-2,
    0x1.055d04cfcad3ap+3, 0x1.fffffa994c635p-2, 0x1.04f68e058f4c4p+3, 0x1.fffffa7645e15p-2,
    0x1.0490173b5addep+3, 0x1.fffffa525c3d9p-2, 0x1.0429a0712db6ap+3, 0x1.fffffa2d89b73p-2,
    0x1.03c329a70805ap+3, 0x1.fffffa07c867ep-2, 0x1.035cb2dce9fb5p+3, 0x1.fffff9e112434p-2,
    0x1.02f63c12d3c94p+3, 0x1.fffff9b961159p-2, 0x1.028fc548c5a26p+3, 0x1.fffff990ae82fp-2,
    0x1.02294e7ebfbadp+3, 0x1.fffff966f4064p-2, 0x1.01c2d7b4c2480p+3, 0x1.fffff93c2af01p-2,
    0x1.015c60eacd80ep+3, 0x1.fffff9104c659p-2, 0x1.00f5ea20e19dap+3, 0x1.fffff8e3515f9p-2,
    0x1.008f7356fed7dp+3, 0x1.fffff8b532a94p-2, 0x1.0028fc8d256abp+3, 0x1.fffff885e8df1p-2,
    0x1.ff850b86ab258p+2, 0x1.fffff8556c6dap-2, 0x1.feb81df31f1c7p+2, 0x1.fffff823b5904p-2,
    0x1.fdeb305fa7398p+2, 0x1.fffff7f0bc501p-2, 0x1.fd1e42cc43ff7p+2, 0x1.fffff7bc78827p-2,
    0x1.fc515538f5f43p+2, 0x1.fffff786e1c7ep-2, 0x1.fb8467a5bda11p+2, 0x1.fffff74fef8a6p-2,
    0x1.fab77a129b930p+2, 0x1.fffff71798fc9p-2, 0x1.f9ea8c7f905a6p+2, 0x1.fffff6ddd517cp-2,
    0x1.f91d9eec9c8b4p+2, 0x1.fffff6a29a9adp-2, 0x1.f850b159c0bd8p+2, 0x1.fffff665e008ap-2,
    0x1.f783c3c6fd8cbp+2, 0x1.fffff6279ba66p-2, 0x1.f6b6d63453989p+2, 0x1.fffff5e7c37a7p-2,
    0x1.f5e9e8a1c384ap+2, 0x1.fffff5a64d4a3p-2, 0x1.f51cfb0f4df8dp+2, 0x1.fffff5632e98fp-2,
    0x1.f4500d7cf3a12p+2, 0x1.fffff51e5ca5dp-2, 0x1.f3831feab52dfp+2, 0x1.fffff4d7cc6a5p-2,
    0x1.f2b6325893542p+2, 0x1.fffff48f72986p-2, 0x1.f1e944c68ecd3p+2, 0x1.fffff4454398ap-2,
    0x1.f11c5734a8575p+2, 0x1.fffff3f933889p-2, 0x1.f04f69a2e0b57p+2, 0x1.fffff3ab3638ap-2,
    0x1.ef827c1138af7p+2, 0x1.fffff35b3f2a3p-2, 0x1.eeb58e7fb1125p+2, 0x1.fffff309418dap-2,
    0x1.ede8a0ee4ab04p+2, 0x1.fffff2b530403p-2, 0x1.ed1bb35d0660cp+2, 0x1.fffff25efdca0p-2,
    0x1.ec4ec5cbe500dp+2, 0x1.fffff2069c5bep-2, 0x1.eb81d83ae772dp+2, 0x1.fffff1abfdccfp-2,
    0x1.eab4eaaa0e9f4p+2, 0x1.fffff14f1398bp-2, 0x1.e9e7fd195b742p+2, 0x1.fffff0efcedc5p-2,
    0x1.e91b0f88cee5cp+2, 0x1.fffff08e20549p-2, 0x1.e84e21f869ee8p+2, 0x1.fffff029f85b3p-2,
    0x1.e78134682d8f1p+2, 0x1.ffffefc346e46p-2, 0x1.e6b446d81acebp+2, 0x1.ffffef59fb7c7p-2,
    0x1.e5e7594832bb5p+2, 0x1.ffffeeee0544ep-2, 0x1.e51a6bb87669bp+2, 0x1.ffffee7f52f1cp-2,
    0x1.e44d7e28e6f58p+2, 0x1.ffffee0dd2c72p-2, 0x1.e38090998581cp+2, 0x1.ffffed997295ep-2,
    0x1.e2b3a30a5338cp+2, 0x1.ffffed221fb91p-2, 0x1.e1e6b57b514c5p+2, 0x1.ffffeca7c712dp-2,
    0x1.e119c7ec80f62p+2, 0x1.ffffec2a55096p-2, 0x1.e04cda5de377bp+2, 0x1.ffffeba9b583dp-2,
    0x1.df7feccf7a1abp+2, 0x1.ffffeb25d3e6cp-2, 0x1.deb2ff4146314p+2, 0x1.ffffea9e9b116p-2,
    0x1.dde611b34915fp+2, 0x1.ffffea13f559dp-2, 0x1.dd192425842c3p+2, 0x1.ffffe985cc89ap-2,
    0x1.dc4c3697f8e07p+2, 0x1.ffffe8f409da6p-2, 0x1.db7f490aa8a83p+2, 0x1.ffffe85e95f20p-2,
    0x1.dab25b7d9502ap+2, 0x1.ffffe7c558deep-2, 0x1.d9e56df0bf78ap+2, 0x1.ffffe7283a145p-2,
    0x1.d9188064299ccp+2, 0x1.ffffe68720662p-2, 0x1.d84b92d7d50c2p+2, 0x1.ffffe5e1f2053p-2,
    0x1.d77ea54bc36e2p+2, 0x1.ffffe538947adp-2, 0x1.d6b1b7bff674dp+2, 0x1.ffffe48aeca4cp-2,
    0x1.d5e4ca346fdd7p+2, 0x1.ffffe3d8deb0ep-2, 0x1.d517dca931705p+2, 0x1.ffffe3224e189p-2,
    0x1.d44aef1e3d017p+2, 0x1.ffffe2671d9c4p-2, 0x1.d37e01939470bp+2, 0x1.ffffe1a72f3eap-2,
    0x1.d2b1140939aa0p+2, 0x1.ffffe0e264400p-2, 0x1.d1e4267f2ea5ep+2, 0x1.ffffe0189d194p-2,
    0x1.d11738f575698p+2, 0x1.ffffdf49b976dp-2, 0x1.d04a4b6c10073p+2, 0x1.ffffde7598337p-2,
    0x1.cf7d5de3009ebp+2, 0x1.ffffdd9c17531p-2, 0x1.ceb0705a495d9p+2, 0x1.ffffdcbd13fd2p-2,
    0x1.cde382d1ec7f8p+2, 0x1.ffffdbd86a772p-2, 0x1.cd169549ec4e9p+2, 0x1.ffffdaedf61eep-2,
    0x1.cc49a7c24b23dp+2, 0x1.ffffd9fd9164bp-2, 0x1.cb7cba3b0b677p+2, 0x1.ffffd90715c52p-2,
    0x1.caafccb42f913p+2, 0x1.ffffd80a5bc34p-2, 0x1.c9e2df2dba28fp+2, 0x1.ffffd7073ae1ep-2,
    0x1.c915f1a7adc6fp+2, 0x1.ffffd5fd899d5p-2, 0x1.c84904220d144p+2, 0x1.ffffd4ed1d64bp-2,
    0x1.c77c169cdacb2p+2, 0x1.ffffd3d5ca930p-2, 0x1.c6af291819b7ap+2, 0x1.ffffd2b764685p-2,
    0x1.c5e23b93ccb7ep+2, 0x1.ffffd191bd027p-2, 0x1.c5154e0ff6bc9p+2, 0x1.ffffd064a555dp-2,
    0x1.c448608c9ac99p+2, 0x1.ffffcf2fed258p-2, 0x1.c37b7309bbf62p+2, 0x1.ffffcdf362fc1p-2,
    0x1.c2ae85875d6dcp+2, 0x1.ffffccaed4232p-2, 0x1.c1e1980582705p+2, 0x1.ffffcb620c9b8p-2,
    0x1.c114aa842e52ep+2, 0x1.ffffca0cd714fp-2, 0x1.c047bd0364801p+2, 0x1.ffffc8aefce54p-2,
    0x1.bf7acf832878bp+2, 0x1.ffffc74845fffp-2, 0x1.beade2037dd43p+2, 0x1.ffffc5d878ed0p-2,
    0x1.bde0f48468417p+2, 0x1.ffffc45f5abfbp-2, 0x1.bd140705eb871p+2, 0x1.ffffc2dcaf0d4p-2,
    0x1.bc4719880b844p+2, 0x1.ffffc15037e31p-2, 0x1.bb7a2c0acc314p+2, 0x1.ffffbfb9b5bcep-2,
    0x1.baad3e8e31a02p+2, 0x1.ffffbe18e77a7p-2, 0x1.b9e051123ffd3p+2, 0x1.ffffbc6d8a555p-2,
    0x1.b9136396fb901p+2, 0x1.ffffbab759d5ep-2, 0x1.b846761c68bbdp+2, 0x1.ffffb8f60fc8ap-2,
    0x1.b77988a28c004p+2, 0x1.ffffb7296432ep-2, 0x1.b6ac9b2969fa3p+2, 0x1.ffffb5510d470p-2,
    0x1.b5dfadb107646p+2, 0x1.ffffb36cbf58fp-2, 0x1.b512c03969183p+2, 0x1.ffffb17c2cd1ep-2,
    0x1.b445d2c2940e9p+2, 0x1.ffffaf7f0623cp-2, 0x1.b378e54c8d60bp+2, 0x1.ffffad74f9bcdp-2,
    0x1.b2abf7d75a48ap+2, 0x1.ffffab5db3fa3p-2, 0x1.b1df0a6300228p+2, 0x1.ffffa938df1acp-2,
    0x1.b1121cef846d2p+2, 0x1.ffffa70623312p-2, 0x1.b0452f7ceccb1p+2, 0x1.ffffa4c52615fp-2,
    0x1.af78420b3f034p+2, 0x1.ffffa2758b592p-2, 0x1.aeab549a81023p+2, 0x1.ffffa016f4333p-2,
    0x1.adde672ab8dacp+2, 0x1.ffff9da8ff760p-2, 0x1.ad1179bbecc73p+2, 0x1.ffff9b2b497d4p-2,
    0x1.ac448c4e232a4p+2, 0x1.ffff989d6c1e7p-2, 0x1.ab779ee1628ffp+2, 0x1.ffff95fefe98bp-2,
    0x1.aaaab175b1aedp+2, 0x1.ffff934f9583cp-2, 0x1.a9ddc40b1768ep+2, 0x1.ffff908ec2bedp-2,
    0x1.a910d6a19accep+2, 0x1.ffff8dbc155efp-2, 0x1.a843e93943175p+2, 0x1.ffff8ad7199d1p-2,
    0x1.a776fbd217b37p+2, 0x1.ffff87df58c34p-2, 0x1.a6aa0e6c203cep+2, 0x1.ffff84d45919bp-2,
    0x1.a5dd210764806p+2, 0x1.ffff81b59dd37p-2, 0x1.a51033a3ec7d7p+2, 0x1.ffff7e82a6fa3p-2,
    0x1.a4434641c0673p+2, 0x1.ffff7b3af159cp-2, 0x1.a37658e0e8a64p+2, 0x1.ffff77ddf66b4p-2,
    0x1.a2a96b816dd97p+2, 0x1.ffff746b2c3f6p-2, 0x1.a1dc7e2358d7cp+2, 0x1.ffff70e205686p-2,
    0x1.a10f90c6b2b15p+2, 0x1.ffff6d41f0e37p-2, 0x1.a042a36b84b12p+2, 0x1.ffff698a5a014p-2,
    0x1.9f75b611d85e6p+2, 0x1.ffff65baa84e8p-2, 0x1.9ea8c8b9b77e3p+2, 0x1.ffff61d23f7b4p-2,
    0x1.9ddbdb632c14ep+2, 0x1.ffff5dd07f41cp-2, 0x1.9d0eee0e4067cp+2, 0x1.ffff59b4c34d3p-2,
    0x1.9c4200bafefecp+2, 0x1.ffff557e631f0p-2, 0x1.9b75136972a62p+2, 0x1.ffff512cb1f40p-2,
    0x1.9aa82619a6702p+2, 0x1.ffff4cbefea8cp-2, 0x1.99db38cba5b6dp+2, 0x1.ffff4834939d1p-2,
    0x1.990e4b7f7c1dcp+2, 0x1.ffff438cb6970p-2, 0x1.98415e3535942p+2, 0x1.ffff3ec6a8a50p-2,
    0x1.977470ecde568p+2, 0x1.ffff39e1a5ff6p-2, 0x1.96a783a682f0bp+2, 0x1.ffff34dce5e8dp-2,
    0x1.95da9662303ffp+2, 0x1.ffff2fb79a8e5p-2, 0x1.950da91ff374ep+2, 0x1.ffff2a70f0e62p-2,
    0x1.9440bbdfda15bp+2, 0x1.ffff2508108e1p-2, 0x1.9373cea1f2005p+2, 0x1.ffff1f7c1ba8cp-2,
    0x1.92a6e166496c8p+2, 0x1.ffff19cc2eba2p-2, 0x1.91d9f42ceeee3p+2, 0x1.ffff13f76082fp-2,
    0x1.910d06f5f1781p+2, 0x1.ffff0dfcc1db8p-2, 0x1.904019c1605d7p+2, 0x1.ffff07db5d8d3p-2,
    0x1.8f732c8f4b555p+2, 0x1.ffff0192382b6p-2, 0x1.8ea63f5fc27c5p+2, 0x1.fffefb204feb1p-2,
    0x1.8dd95232d657cp+2, 0x1.fffef4849c797p-2, 0x1.8d0c650897d7fp+2, 0x1.fffeedbe0ed1dp-2,
    0x1.8c3f77e1185b2p+2, 0x1.fffee6cb91120p-2, 0x1.8b728abc69b02p+2, 0x1.fffedfac064dep-2,
    0x1.8aa59d9a9e194p+2, 0x1.fffed85e4a61ap-2, 0x1.89d8b07bc84f4p+2, 0x1.fffed0e131c34p-2,
    0x1.890bc35ffb843p+2, 0x1.fffec93389522p-2, 0x1.883ed6474b66bp+2, 0x1.fffec15416264p-2,
    0x1.8771e931cc24fp+2, 0x1.fffeb941955d8p-2, 0x1.86a4fc1f92702p+2, 0x1.fffeb0fabbe81p-2,
    0x1.85d80f10b37f8p+2, 0x1.fffea87e36534p-2, 0x1.850b22054513dp+2, 0x1.fffe9fcaa8936p-2,
    0x1.843e34fd5d7b1p+2, 0x1.fffe96deadcbbp-2, 0x1.837147f91393cp+2, 0x1.fffe8db8d8158p-2,
    0x1.82a45af87ed0cp+2, 0x1.fffe8457b0454p-2, 0x1.81d76dfbb73d0p+2, 0x1.fffe7ab9b5aeep-2,
    0x1.810a8102d57f4p+2, 0x1.fffe70dd5de7bp-2, 0x1.803d940df2de2p+2, 0x1.fffe66c114878p-2,
    0x1.7f70a71d29445p+2, 0x1.fffe5c633ae7bp-2, 0x1.7ea3ba3093445p+2, 0x1.fffe51c227e10p-2,
    0x1.7dd6cd484c1d3p+2, 0x1.fffe46dc27872p-2, 0x1.7d09e0646fbe8p+2, 0x1.fffe3baf7ae33p-2,
    0x1.7c3cf3851acd0p+2, 0x1.fffe303a57abdp-2, 0x1.7b7006aa6aa74p+2, 0x1.fffe247ae7fc3p-2,
    0x1.7aa319d47d6a2p+2, 0x1.fffe186f4a083p-2, 0x1.79d62d0371f60p+2, 0x1.fffe0c158fcfdp-2,
    0x1.7909403767f34p+2, 0x1.fffdff6bbecf9p-2, 0x1.783c53707fd79p+2, 0x1.fffdf26fcfaf9p-2,
    0x1.776f66aedaeb5p+2, 0x1.fffde51fadf07p-2, 0x1.76a279f29b4e6p+2, 0x1.fffdd7793795bp-2,
    0x1.75d58d3be3fe4p+2, 0x1.fffdc97a3ccebp-2, 0x1.7508a08ad8db1p+2, 0x1.fffdbb207f9cap-2,
    0x1.743bb3df9eadbp+2, 0x1.fffdac69b376cp-2, 0x1.736ec73a5b2dap+2, 0x1.fffd9d537cec1p-2,
    0x1.72a1da9b3506bp+2, 0x1.fffd8ddb7142ap-2, 0x1.71d4ee0253dfcp+2, 0x1.fffd7dff1614ap-2,
    0x1.7108016fe060ap+2, 0x1.fffd6dbbe0ea8p-2, 0x1.703b14e40438dp+2, 0x1.fffd5d0f36d2fp-2,
    0x1.6f6e285eea263p+2, 0x1.fffd4bf66bf7fp-2, 0x1.6ea13be0bdfb9p+2, 0x1.fffd3a6ec3318p-2,
    0x1.6dd44f69aca83p+2, 0x1.fffd28756d94fp-2, 0x1.6d0762f9e43e9p+2, 0x1.fffd16078a023p-2,
    0x1.6c3a769193fbfp+2, 0x1.fffd032224ad4p-2, 0x1.6b6d8a30ec4ffp+2, 0x1.fffcefc236a5bp-2,
    0x1.6aa09dd81ee44p+2, 0x1.fffcdbe4a55a0p-2, 0x1.69d3b1875ea49p+2, 0x1.fffcc7864218ap-2,
    0x1.6906c53edfc6cp+2, 0x1.fffcb2a3c98d8p-2, 0x1.6839d8fed7d35p+2, 0x1.fffc9d39e33c1p-2,
    0x1.676cecc77dadep+2, 0x1.fffc874520f64p-2, 0x1.66a00099099dep+2, 0x1.fffc70c1fe4fep-2,
    0x1.65d31473b557ep+2, 0x1.fffc59ace00e3p-2, 0x1.65062857bc066p+2, 0x1.fffc420213944p-2,
    0x1.64393c455a53ep+2, 0x1.fffc29bdce4b4p-2, 0x1.636c503cce73ep+2, 0x1.fffc10dc2d071p-2,
    0x1.629f643e582d8p+2, 0x1.fffbf7593366cp-2, 0x1.61d2784a38e55p+2, 0x1.fffbdd30cb316p-2,
    0x1.61058c60b3a7ep+2, 0x1.fffbc25ec3ae4p-2, 0x1.6038a0820d34ap+2, 0x1.fffba6ded0f96p-2,
    0x1.5f6bb4ae8c08bp+2, 0x1.fffb8aac8b52ep-2, 0x1.5e9ec8e6786a6p+2, 0x1.fffb6dc36e6aep-2,
    0x1.5dd1dd2a1c748p+2, 0x1.fffb501ed8a81p-2, 0x1.5d04f179c4227p+2, 0x1.fffb31ba0a69ep-2,
    0x1.5c3805d5bd5c7p+2, 0x1.fffb12902545bp-2, 0x1.5b6b1a3e5803ap+2, 0x1.fffaf29c2b3f8p-2,
    0x1.5a9e2eb3e5ff5p+2, 0x1.fffad1d8fdfd2p-2, 0x1.59d14336bb49dp+2, 0x1.fffab0415df45p-2,
    0x1.590457c72dfe0p+2, 0x1.fffa8dcfe993bp-2, 0x1.58376c659664fp+2, 0x1.fffa6a7f1c661p-2,
    0x1.576a81124f047p+2, 0x1.fffa46494e306p-2, 0x1.569d95cdb4acfp+2, 0x1.fffa2128b209bp-2,
    0x1.55d0aa9826890p+2, 0x1.fff9fb17556d9p-2, 0x1.5503bf72062c1p+2, 0x1.fff9d40f1f482p-2,
    0x1.5436d45bb7a26p+2, 0x1.fff9ac09cefc0p-2, 0x1.5369e955a180ep+2, 0x1.fff98300fb626p-2,
    0x1.529cfe602cf5ap+2, 0x1.fff958ee11c40p-2, 0x1.51d0137bc5d8cp+2, 0x1.fff92dca54cb9p-2,
    0x1.510328a8dabd9p+2, 0x1.fff9018edb71fp-2, 0x1.50363de7dd047p+2, 0x1.fff8d4348fe28p-2,
    0x1.4f69533940ecep+2, 0x1.fff8a5b42e58fp-2, 0x1.4e9c689d7da82p+2, 0x1.fff8760643f77p-2,
    0x1.4dcf7e150d6c4p+2, 0x1.fff845232d956p-2, 0x1.4d0293a06d87cp+2, 0x1.fff8130316866p-2,
    0x1.4c35a9401e75bp+2, 0x1.fff7df9df7594p-2, 0x1.4b68bef4a3f21p+2, 0x1.fff7aaeb948efp-2,
    0x1.4a9bd4be850f3p+2, 0x1.fff774e37d497p-2, 0x1.49ceea9e4c4b0p+2, 0x1.fff73d7d09f14p-2,
    0x1.4902009487a58p+2, 0x1.fff704af5ad36p-2, 0x1.483516a1c8b78p+2, 0x1.fff6ca7156b53p-2,
    0x1.47682cc6a4c9ap+2, 0x1.fff68eb9a95fbp-2, 0x1.469b4303b4ecap+2, 0x1.fff6517ec2217p-2,
    0x1.45ce595996118p+2, 0x1.fff612b6d2463p-2, 0x1.45016fc8e9232p+2, 0x1.fff5d257cb856p-2,
    0x1.44348652531f7p+2, 0x1.fff590575e65dp-2, 0x1.43679cf67d324p+2, 0x1.fff54caaf8975p-2,
    0x1.429ab3b614d06p+2, 0x1.fff50747c341bp-2, 0x1.41cdca91cbd2fp+2, 0x1.fff4c022a1483p-2,
    0x1.4100e18a58948p+2, 0x1.fff477302d82ap-2, 0x1.4033f8a0760ddp+2, 0x1.fff42c64b8ea2p-2,
    0x1.3f670fd4e3f3dp+2, 0x1.fff3dfb448bacp-2, 0x1.3e9a272866d68p+2, 0x1.fff3911294887p-2,
    0x1.3dcd3e9bc8403p+2, 0x1.fff340730447fp-2, 0x1.3d00562fd6d60p+2, 0x1.fff2edc8ae4adp-2,
    0x1.3c336de56678dp+2, 0x1.fff29906552e9p-2, 0x1.3b6685bd50671p+2, 0x1.fff2421e65be0p-2,
    0x1.3a999db8735fep+2, 0x1.fff1e902f4c59p-2, 0x1.39ccb5d7b3c67p+2, 0x1.fff18da5bcd8bp-2,
    0x1.38ffce1bfbc6ap+2, 0x1.fff12ff81c09cp-2, 0x1.3832e6863b7aap+2, 0x1.fff0cfeb11924p-2,
    0x1.3765ff1769113p+2, 0x1.fff06d6f3b6ccp-2, 0x1.369917d080f51p+2, 0x1.fff00874d3de6p-2,
    0x1.35cc30b285f5bp+2, 0x1.ffefa0ebaef15p-2, 0x1.34ff49be81704p+2, 0x1.ffef36c337de3p-2,
    0x1.343262f5837a6p+2, 0x1.ffeec9ea6e651p-2, 0x1.33657c58a30d9p+2, 0x1.ffee5a4fe4157p-2,
    0x1.329895e8fe341p+2, 0x1.ffede7e1b9843p-2, 0x1.31cbafa7ba367p+2, 0x1.ffed728d9b6fcp-2,
    0x1.30fec99603ca8p+2, 0x1.ffecfa40bfd21p-2, 0x1.3031e3b50f43dp+2, 0x1.ffec7ee7e2dedp-2,
    0x1.2f64fe0618c47p+2, 0x1.ffec006f43ef0p-2, 0x1.2e98188a64703p+2, 0x1.ffeb7ec2a2582p-2,
    0x1.2dcb33433e9ffp+2, 0x1.ffeaf9cd3a2f2p-2, 0x1.2cfe4e31fc175p+2, 0x1.ffea7179c0f62p-2,
    0x1.2c316957fa3acp+2, 0x1.ffe9e5b262353p-2, 0x1.2b6484b69f47ep+2, 0x1.ffe95660bbfc7p-2,
    0x1.2a97a04f5a8e8p+2, 0x1.ffe8c36ddb502p-2, 0x1.29cabc23a4abbp+2, 0x1.ffe82cc2387d2p-2,
    0x1.28fdd834ffc5ap+2, 0x1.ffe79245b3563p-2, 0x1.2830f484f7c9fp+2, 0x1.ffe6f3df8f586p-2,
    0x1.2764111522ac9p+2, 0x1.ffe651766fb6dp-2, 0x1.26972de720a92p+2, 0x1.ffe5aaf0534d0p-2,
    0x1.25ca4afc9c853p+2, 0x1.ffe5003290768p-2, 0x1.24fd68574bd4dp+2, 0x1.ffe45121d0cc3p-2,
    0x1.243085f8ef408p+2, 0x1.ffe39da20cc5fp-2, 0x1.2363a3e352ccdp+2, 0x1.ffe2e596873f7p-2,
    0x1.2296c2184e244p+2, 0x1.ffe228e1c8e10p-2, 0x1.21c9e099c4e28p+2, 0x1.ffe167659b6a3p-2,
    0x1.20fcff69a6e1fp+2, 0x1.ffe0a10304ddcp-2, 0x1.20301e89f08afp+2, 0x1.ffdfd59a428f0p-2,
    0x1.1f633dfcab252p+2, 0x1.ffdf050ac40ebp-2, 0x1.1e965dc3ed2adp+2, 0x1.ffde2f3325f79p-2,
    0x1.1dc97de1da9eap+2, 0x1.ffdd53f12c98ep-2, 0x1.1cfc9e58a562fp+2, 0x1.ffdc7321be7ecp-2,
    0x1.1c2fbf2a8d93fp+2, 0x1.ffdb8ca0ded73p-2, 0x1.1b62e059e1e3bp+2, 0x1.ffdaa049a7b2bp-2,
    0x1.1a9601e8fff89p+2, 0x1.ffd9adf644202p-2, 0x1.19c923da54ce4p+2, 0x1.ffd8b57fea222p-2,
    0x1.18fc46305d18fp+2, 0x1.ffd7b6bed47e2p-2, 0x1.182f68eda5ab4p+2, 0x1.ffd6b18a3c629p-2,
    0x1.17628c14cbde7p+2, 0x1.ffd5a5b852e4ep-2, 0x1.1695afa87dfddp+2, 0x1.ffd4931e3a552p-2,
    0x1.15c8d3ab7bb3fp+2, 0x1.ffd3798fff66cp-2, 0x1.14fbf820967bap+2, 0x1.ffd258e0922d0p-2,
    0x1.142f1d0ab2132p+2, 0x1.ffd130e1beea1p-2, 0x1.1362426cc4f23p+2, 0x1.ffd0016426b08p-2,
    0x1.12956849d8c3ap+2, 0x1.ffceca3737d3fp-2, 0x1.11c88ea50ae19p+2, 0x1.ffcd8b29262a6p-2,
    0x1.10fbb5818cd4bp+2, 0x1.ffcc4406e31a7p-2, 0x1.102edce2a4d73p+2, 0x1.ffcaf49c15773p-2,
    0x1.0f6204cbae5a9p+2, 0x1.ffc99cb311272p-2, 0x1.0e952d401a912p+2, 0x1.ffc83c14ce957p-2,
    0x1.0dc8564370fa9p+2, 0x1.ffc6d288e1ec1p-2, 0x1.0cfb7fd94ff4cp+2, 0x1.ffc55fd57215ap-2,
    0x1.0c2eaa056d4f5p+2, 0x1.ffc3e3bf2f84dp-2, 0x1.0b61d4cb96e3bp+2, 0x1.ffc25e094ac10p-2,
    0x1.0a95002fb330cp+2, 0x1.ffc0ce756ab59p-2, 0x1.09c82c35c1fa0p+2, 0x1.ffbf34c3a2c35p-2,
    0x1.08fb58e1dceb8p+2, 0x1.ffbd90b268916p-2, 0x1.082e863838416p+2, 0x1.ffbbe1fe899d3p-2,
    0x1.0761b43d23739p+2, 0x1.ffba286320871p-2, 0x1.0694e2f509e68p+2, 0x1.ffb863998a19cp-2,
    0x1.05c81264739f3p+2, 0x1.ffb693595a0bbp-2, 0x1.04fb429005fd2p+2, 0x1.ffb4b7584f782p-2,
    0x1.042e737c84778p+2, 0x1.ffb2cf4a490dfp-2, 0x1.0361a52ed1609p+2, 0x1.ffb0dae138f23p-2,
    0x1.0294d7abeeaccp+2, 0x1.ffaed9cd18559p-2, 0x1.01c80af8febfap+2, 0x1.ffaccbbbdab9cp-2,
    0x1.00fb3f1b453dap+2, 0x1.ffaab05960e4cp-2, 0x1.002e741827e2ep+2, 0x1.ffa8874f6b80ep-2,
    0x1.fec353ea5ec05p+1, 0x1.ffa650458d66cp-2, 0x1.fd29c17010795p+1, 0x1.ffa40ae11d8f7p-2,
    0x1.fb9030cd077bap+1, 0x1.ffa1b6c528ac0p-2, 0x1.f9f6a20d31a9fp+1, 0x1.ff9f539262616p-2,
    0x1.f85d153cca25cp+1, 0x1.ff9ce0e716250p-2, 0x1.f6c38a685b42ep+1, 0x1.ff9a5e5f17b8bp-2,
    0x1.f52a019cc087ap+1, 0x1.ff97cb93b342fp-2, 0x1.f3907ae728b96p+1, 0x1.ff95281b9d01ap-2,
    0x1.f1f6f65517f72p+1, 0x1.ff92738ae0942p-2, 0x1.f05d73f469e0ap+1, 0x1.ff8fad72cfda6p-2,
    0x1.eec3f3d353cc9p+1, 0x1.ff8cd561f166dp-2, 0x1.ed2a7600670bbp+1, 0x1.ff89eae3ee7f4p-2,
    0x1.eb90fa8a933b9p+1, 0x1.ff86ed8180ab9p-2, 0x1.e9f7818128a7ep+1, 0x1.ff83dcc05ecdcp-2,
    0x1.e85e0af3dabaep+1, 0x1.ff80b82329c1ap-2, 0x1.e6c496f2c27ddp+1, 0x1.ff7d7f295880dp-2,
    0x1.e52b258e61296p+1, 0x1.ff7a314f23c76p-2, 0x1.e391b6d7a2c69p+1, 0x1.ff76ce0d71374p-2,
    0x1.e1f84adfe0e08p+1, 0x1.ff7354d9bdf65p-2, 0x1.e05ee1b8e547bp+1, 0x1.ff6fc52608c3dp-2,
    0x1.dec57b74ece6fp+1, 0x1.ff6c1e60bb829p-2, 0x1.dd2c1826aaaa5p+1, 0x1.ff685ff49433dp-2,
    0x1.db92b7e14a791p+1, 0x1.ff6489488d5fap-2, 0x1.d9f95ab874428p+1, 0x1.ff6099bfc5e6dp-2,
    0x1.d86000c04f1e8p+1, 0x1.ff5c90b9683b8p-2, 0x1.d6c6aa0d84821p+1, 0x1.ff586d9090fbdp-2,
    0x1.d52d56b543887p+1, 0x1.ff542f9c34eb3p-2, 0x1.d39406cd44516p+1, 0x1.ff4fd62f06467p-2,
    0x1.d1faba6bcb750p+1, 0x1.ff4b6097596e6p-2, 0x1.d06171a7ad8dfp+1, 0x1.ff46ce1f08e52p-2,
    0x1.cec82c9852d9dp+1, 0x1.ff421e0b5899dp-2, 0x1.cd2eeb55baf15p+1, 0x1.ff3d4f9cd87e1p-2,
    0x1.cb95adf880983p+1, 0x1.ff38620f46616p-2, 0x1.c9fc7499dda51p+1, 0x1.ff3354996f0dfp-2,
    0x1.c8633f53af034p+1, 0x1.ff2e266d0ea15p-2, 0x1.c6ca0e4078cd1p+1, 0x1.ff28d6b6b01dap-2,
    0x1.c530e17b6a81ap+1, 0x1.ff23649d8c2dbp-2, 0x1.c397b92063547p+1, 0x1.ff1dcf4367172p-2,
    0x1.c1fe954bf6998p+1, 0x1.ff1815c46dd5ap-2, 0x1.c065761b704d3p+1, 0x1.ff123737125a8p-2,
    0x1.becc5bacd9b92p+1, 0x1.ff0c32abe6ea9p-2, 0x1.bd33461efe371p+1, 0x1.ff06072d7895ap-2,
    0x1.bb9a35917011ap+1, 0x1.feffb3c028c1cp-2, 0x1.ba012a248d84ep+1, 0x1.fef9376205c4fp-2,
    0x1.b86823f985de2p+1, 0x1.fef2910aa2874p-2, 0x1.b6cf23325ebd3p+1, 0x1.feebbfaaed276p-2,
    0x1.b53627f1f9766p+1, 0x1.fee4c22d049c4p-2, 0x1.b39d325c18977p+1, 0x1.fedd97740d4d2p-2,
    0x1.b2044295658f5p+1, 0x1.fed63e5c0499ep-2, 0x1.b06b58c3767a1p+1, 0x1.feceb5b9934d3p-2,
    0x1.aed2750cd411dp+1, 0x1.fec6fc59def26p-2, 0x1.ad399798ffc51p+1, 0x1.febf11025a07ap-2,
    0x1.aba0c09079f44p+1, 0x1.feb6f2709306dp-2, 0x1.aa07f01cc856ep+1, 0x1.feae9f5a023c6p-2,
    0x1.a86f26687c88dp+1, 0x1.fea6166bd6672p-2, 0x1.a6d6639f3ac20p+1, 0x1.fe9d564ac0180p-2,
    0x1.a53da7edc0b7fp+1, 0x1.fe945d92bbcb8p-2, 0x1.a3a4f381ecabbp+1, 0x1.fe8b2ad6dab4bp-2,
    0x1.a20c468ac4a3ep+1, 0x1.fe81bca10a32ap-2, 0x1.a073a1387dd50p+1, 0x1.fe781171d9e79p-2,
    0x1.9edb03bc84386p+1, 0x1.fe6e27c0406a8p-2, 0x1.9d426e4982532p+1, 0x1.fe63fdf95e8b5p-2,
    0x1.9ba9e113692ecp+1, 0x1.fe599280411fep-2, 0x1.9a115c4f78837p+1, 0x1.fe4ee3ada152cp-2,
    0x1.9878e03447169p+1, 0x1.fe43efcfa36b0p-2, 0x1.96e06cf9cb4dap+1, 0x1.fe38b5299402bp-2,
    0x1.954802d963f7bp+1, 0x1.fe2d31f3a3a54p-2, 0x1.93afa20de14dap+1, 0x1.fe21645aa0cb0p-2,
    0x1.92174ad38e2bap+1, 0x1.fe154a7fb028fp-2, 0x1.907efd6839849p+1, 0x1.fe08e278034bap-2,
    0x1.8ee6ba0b4010cp+1, 0x1.fdfc2a4c8d72ep-2, 0x1.8d4e80fd9639ap+1, 0x1.fdef1ff9b6a52p-2,
    0x1.8bb65281d243cp+1, 0x1.fde1c16f0ceffp-2, 0x1.8a1e2edc36b88p+1, 0x1.fdd40c8ef3cb4p-2,
    0x1.88861652bd115p+1, 0x1.fdc5ff2e51961p-2, 0x1.86ee092d20a55p+1, 0x1.fdb797143b205p-2,
    0x1.855607b4e9dbcp+1, 0x1.fda8d1f99d395p-2, 0x1.83be123579a44p+1, 0x1.fd99ad88e4356p-2,
    0x1.822628fc1536dp+1, 0x1.fd8a275da1624p-2, 0x1.808e4c57f21d0p+1, 0x1.fd7a3d042e5c8p-2,
    0x1.7ef67c9a42864p+1, 0x1.fd69ebf94e3c5p-2, 0x1.7d5eba1641e91p+1, 0x1.fd5931a9cc8d2p-2,
    0x1.7bc7052141f29p+1, 0x1.fd480b721a04ep-2, 0x1.7a2f5e12b7c6bp+1, 0x1.fd36769de6edep-2,
    0x1.7897c54449926p+1, 0x1.fd247067bb38dp-2, 0x1.77003b11dc722p+1, 0x1.fd11f5f88c28ep-2,
    0x1.7568bfd9a2ae8p+1, 0x1.fcff04674f8eap-2, 0x1.73d153fc2a50fp+1, 0x1.fceb98b88c84dp-2,
    0x1.7239f7dc6c122p+1, 0x1.fcd7afdde9a1bp-2, 0x1.70a2abdfdaa52p+1, 0x1.fcc346b5b890dp-2,
    0x1.6f0b706e72606p+1, 0x1.fcae5a0a7f078p-2, 0x1.6d7445f2c9472p+1, 0x1.fc98e6927d070p-2,
    0x1.6bdd2cda1f757p+1, 0x1.fc82e8ef305f1p-2, 0x1.6a4625946ff0fp+1, 0x1.fc6c5dacd562dp-2,
    0x1.68af309481e0bp+1, 0x1.fc554141e4c30p-2, 0x1.67184e4ffa2e5p+1, 0x1.fc3d900e8e7fbp-2,
    0x1.65817f3f6d92cp+1, 0x1.fc25465c31e29p-2, 0x1.63eac3de73118p+1, 0x1.fc0c605cd2755p-2,
    0x1.62541cabb6e3ap+1, 0x1.fbf2da2a89e4bp-2, 0x1.60bd8a290dd69p+1, 0x1.fbd8afc6f6c2cp-2,
    0x1.5f270cdb89202p+1, 0x1.fbbddd1aa819bp-2, 0x1.5d90a54b8aaa8p+1, 0x1.fba25df485c13p-2,
    0x1.5bfa5404d9db1p+1, 0x1.fb862e0935674p-2, 0x1.5a641996b8d6dp+1, 0x1.fb6948f27c3eep-2,
    0x1.58cdf693fa467p+1, 0x1.fb4baa2e9d458p-2, 0x1.5737eb93179ddp+1, 0x1.fb2d4d1fb410ep-2,
    0x1.55a1f92e47e89p+1, 0x1.fb0e2d0b0c16dp-2, 0x1.540c2003971f5p+1, 0x1.faee45187460dp-2,
    0x1.527660b4fe08bp+1, 0x1.facd90518f9bdp-2, 0x1.50e0bbe87aa83p+1, 0x1.faac09a12077dp-2,
    0x1.4f4b3248293e4p+1, 0x1.fa89abd252469p-2, 0x1.4db5c4825ddd3p+1, 0x1.fa66718ffdcd4p-2,
    0x1.4c207349be94fp+1, 0x1.fa425563ea39ep-2, 0x1.4a8b3f555e39cp+1, 0x1.fa1d51b60a2ebp-2,
    0x1.48f62960d7c81p+1, 0x1.f9f760cbb4d69p-2, 0x1.4761322c6a69ap+1, 0x1.f9d07cc6daf34p-2,
    0x1.45cc5a7d161e8p+1, 0x1.f9a89fa537da3p-2, 0x1.4437a31cb90d8p+1, 0x1.f97fc33f7e512p-2,
    0x1.42a30cda2d7f4p+1, 0x1.f955e148813f4p-2, 0x1.410e988968874p+1, 0x1.f92af34c58250p-2,
    0x1.3f7a4703995ebp+1, 0x1.f8fef2af7f4ffp-2, 0x1.3de6192749739p+1, 0x1.f8d1d8adf3be8p-2,
    0x1.3c520fd87d30bp+1, 0x1.f8a39e5a4aa85p-2, 0x1.3abe2c00d5813p+1, 0x1.f8743c9cc4a0ep-2,
    0x1.392a6e8fb213bp+1, 0x1.f843ac325c4adp-2, 0x1.3796d87a54601p+1, 0x1.f811e5abd0914p-2,
    0x1.36036abc03745p+1, 0x1.f7dee16caa604p-2, 0x1.34702656308abp+1, 0x1.f7aa97aa3dd26p-2,
    0x1.32dd0c509c6eap+1, 0x1.f775006aa6cdfp-2, 0x1.314a1db97db2bp+1, 0x1.f73e1383c10a4p-2,
    0x1.2fb75ba5a7bb4p+1, 0x1.f705c89a1b784p-2, 0x1.2e24c730b2a33p+1, 0x1.f6cc171fe7096p-2,
    0x1.2c92617d23fbbp+1, 0x1.f690f653e0d20p-2, 0x1.2b002bb4986dcp+1, 0x1.f6545d4037842p-2,
    0x1.296e2707ee3e8p+1, 0x1.f61642b96c42ap-2, 0x1.27dc54af70bc4p+1, 0x1.f5d69d5d2ecbep-2,
    0x1.264ab5eb04965p+1, 0x1.f595639134fe3p-2, 0x1.24b94c0255247p+1, 0x1.f5528b820db93p-2,
    0x1.2328184502a0ep+1, 0x1.f50e0b21ef202p-2, 0x1.21971c0ad1594p+1, 0x1.f4c7d82780447p-2,
    0x1.200658b3d9d99p+1, 0x1.f47fe80c9e3f9p-2, 0x1.1e75cfa8ba14fp+1, 0x1.f436300d1cc73p-2,
    0x1.1ce5825ac7905p+1, 0x1.f3eaa52582473p-2, 0x1.1b5572444291bp+1, 0x1.f39d3c11bf8f8p-2,
    0x1.19c5a0e88a583p+1, 0x1.f34de94be326bp-2, 0x1.18360fd452601p+1, 0x1.f2fca10ac853ep-2,
    0x1.16a6c09dd8b65p+1, 0x1.f2a95740c1f57p-2, 0x1.1517b4e51d5eep+1, 0x1.f253ff9a413c0p-2,
    0x1.1388ee541ad0cp+1, 0x1.f1fc8d7c78657p-2, 0x1.11fa6e9eff8b6p+1, 0x1.f1a2f403f9951p-2,
    0x1.106c378468c87p+1, 0x1.f147260351ea1p-2, 0x1.0ede4acd9e4c6p+1, 0x1.f0e91601a0f8bp-2,
    0x1.0d50aa4ecf594p+1, 0x1.f088b6392ccdap-2, 0x1.0bc357e750c62p+1, 0x1.f025f895f2a71p-2,
    0x1.0a365581dc3e1p+1, 0x1.efc0ceb43492dp-2, 0x1.08a9a514d0a81p+1, 0x1.ef5929df04244p-2,
    0x1.071d48a273bbap+1, 0x1.eeeefb0eca7acp-2, 0x1.0591423934c32p+1, 0x1.ee8232e7cdd2ap-2,
    0x1.040593f3f08d9p+1, 0x1.ee12c1b8b4e38p-2, 0x1.027a3ffa36928p+1, 0x1.eda09779084f8p-2,
    0x1.00ef48808f484p+1, 0x1.ed2ba3c7b26f4p-2, 0x1.fec95f91875d9p+0, 0x1.ecb3d5e97dc9ep-2,
    0x1.fbb4f0444c1e5p+0, 0x1.ec391cc7928eep-2, 0x1.f8a147d3b7e1ep+0, 0x1.ebbb66edf36cfp-2,
    0x1.f58e6b16528b5p+0, 0x1.eb3aa289fa275p-2, 0x1.f27c5eff79945p+0, 0x1.eab6bd68d4513p-2,
    0x1.ef6b289ffb3c1p+0, 0x1.ea2fa4f6009e1p-2, 0x1.ec5acd26b41fdp+0, 0x1.e9a54639cd3b7p-2,
    0x1.e94b51e12f3c7p+0, 0x1.e9178dd7d7b10p-2, 0x1.e63cbc3c4854ep+0, 0x1.e886680d8ecb0p-2,
    0x1.e32f11c4d0ba3p+0, 0x1.e7f1c0b0b719fp-2, 0x1.e022582836717p+0, 0x1.e759832df29c1p-2,
    0x1.dd1695352db08p+0, 0x1.e6bd9a874c2bep-2, 0x1.da0bcedc5cac2p+0, 0x1.e61df152c7586p-2,
    0x1.d7020b3109af8p+0, 0x1.e57a71b8f5556p-2, 0x1.d3f95069cb745p+0, 0x1.e4d305738fb9bp-2,
    0x1.d0f1a4e13bb20p+0, 0x1.e42795cc19cc8p-2, 0x1.cdeb0f16abd87p+0, 0x1.e3780b9a892b3p-2,
    0x1.cae595aedbe9ep+0, 0x1.e2c44f43f69dcp-2, 0x1.c7e13f74b3664p+0, 0x1.e20c48b957f74p-2,
    0x1.c4de1359fc396p+0, 0x1.e14fdf7643ecfp-2, 0x1.c1dc18781f99ep+0, 0x1.e08efa7fc0d9dp-2,
    0x1.bedb5610e4c7fp+0, 0x1.dfc980631f6dbp-2, 0x1.bbdbd38f31974p+0, 0x1.deff5734e2557p-2,
    0x1.b8dd9887ccaebp+0, 0x1.de30648fb3f47p-2, 0x1.b5e0acba21663p+0, 0x1.dd5c8d936b536p-2,
    0x1.b2e518110529ep+0, 0x1.dc83b6e421775p-2, 0x1.afeae2a37e467p+0, 0x1.dba5c4a9585e3p-2,
    0x1.acf214b58c02ap+0, 0x1.dac29a8d34ec8p-2, 0x1.a9fab6b8efe52p+0, 0x1.d9da1bbbcd263p-2,
    0x1.a704d14df8065p+0, 0x1.d8ec2ae28c186p-2, 0x1.a4106d444a49ap+0, 0x1.d7f8aa2face92p-2,
    0x1.a11d939bb057ap+0, 0x1.d6ff7b51ce8f9p-2, 0x1.9e2c4d84e4318p+0, 0x1.d6007f77a1c5fp-2,
    0x1.9b3ca4625d315p+0, 0x1.d4fb974fb2d45p-2, 0x1.984ea1c91d498p+0, 0x1.d3f0a30850e14p-2,
    0x1.95624f817e53cp+0, 0x1.d2df824f94867p-2, 0x1.9277b787ff3a6p+0, 0x1.d1c8145387720p-2,
    0x1.8f8ee40e10c75p+0, 0x1.d0aa37c26ef00p-2, 0x1.8ca7df7ae1ddbp+0, 0x1.cf85cacb3b423p-2,
    0x1.89c2b46c2ae34p+0, 0x1.ce5aab1e1dbe7p-2, 0x1.86df6db6f8186p+0, 0x1.cd28b5ed47b70p-2,
    0x1.83fe1668729cdp+0, 0x1.cbefc7edd43fdp-2, 0x1.811eb9c6a7da8p+0, 0x1.caafbd58def23p-2,
    0x1.7e4163514f0c0p+0, 0x1.c96871ecc9dc2p-2, 0x1.7b661ec28c92cp+0, 0x1.c819c0eeb4d6cp-2,
    0x1.788cf80fb2ca7p+0, 0x1.c6c3852c288bap-2, 0x1.75b5fb6a0006ap+0, 0x1.c56598fcf77d9p-2,
    0x1.72e1353f5960dp+0, 0x1.c3ffd64557728p-2, 0x1.700eb23b01fb7p+0, 0x1.c292167835aabp-2,
    0x1.6d3e7f464e5a3p+0, 0x1.c11c3299c8574p-2, 0x1.6a70a989536a3p+0, 0x1.bf9e03425fce4p-2,
    0x1.67a53e6b90d37p+0, 0x1.be1760a179fffp-2, 0x1.64dc4b949626bp+0, 0x1.bc8822811aba4p-2,
    0x1.6215deeca2775p+0, 0x1.baf020496b4a0p-2, 0x1.5f52069d3dedbp+0, 0x1.b94f3104a4110p-2,
    0x1.5c90d111ccd8fp+0, 0x1.b7a52b6342a76p-2, 0x1.59d24cf81bc32p+0, 0x1.b5f1e5c08f224p-2,
    0x1.57168940e4086p+0, 0x1.b435362773184p-2, 0x1.545d9520486a8p+0, 0x1.b26ef257a4f87p-2,
    0x1.51a7800e49190p+0, 0x1.b09eefcb2a461p-2, 0x1.4ef459c72ea02p+0, 0x1.aec503bc33429p-2,
    0x1.4c44324beb2d6p+0, 0x1.ace1032b52868p-2, 0x1.499719e271951p+0, 0x1.aaf2c2e612ff3p-2,
    0x1.46ed2116017f3p+0, 0x1.a8fa178deeb73p-2, 0x1.444658b7681ecp+0, 0x1.a6f6d59fa8bf5p-2,
    0x1.41a2d1dd34d41p+0, 0x1.a4e8d17b0c78dp-2, 0x1.3f029de3e1144p+0, 0x1.a2cfdf6b146afp-2,
    0x1.3c65ce6deaf02p+0, 0x1.a0abd3ae7ab21p-2, 0x1.39cc7563e18f2p+0, 0x1.9e7c8280b4f94p-2,
    0x1.3736a4f462effp+0, 0x1.9c41c0235dcc4p-2, 0x1.34a46f940a407p+0, 0x1.99fb60e80cebbp-2,
    0x1.3215e7fd4e175p+0, 0x1.97a9393aa020dp-2, 0x1.2f8b21304ddcdp+0, 0x1.954b1dabf5e36p-2,
    0x1.2d042e728da94p+0, 0x1.92e0e2fd1aef2p-2, 0x1.2a81234e9fe22p+0, 0x1.906a5e2aebb2ap-2,
    0x1.28021393bbdafp+0, 0x1.8de7647a2a42fp-2, 0x1.2587135540befp+0, 0x1.8b57cb840942dp-2,
    0x1.231036ea2408cp+0, 0x1.88bb69432be5cp-2, 0x1.209d92ec4acbap+0, 0x1.861214211aee3p-2,
    0x1.1e2f3c37cd14bp+0, 0x1.835ba3042e38cp-2, 0x1.1bc547ea22a87p+0, 0x1.8097ed5dea11fp-2,
    0x1.195fcb613865bp+0, 0x1.7dc6cb39cf3c9p-2, 0x1.16fedc3a6d95cp+0, 0x1.7ae8154c9c312p-2,
    0x1.14a290517877fp+0, 0x1.77fba503fdbddp-2, 0x1.124afdbf3155bp+0, 0x1.75015496acc4ap-2,
    0x1.0ff83ad843749p+0, 0x1.71f8ff14f66d7p-2, 0x1.0daa5e2bc33cep+0, 0x1.6ee28079abad1p-2,
    0x1.0b617e81a8f31p+0, 0x1.6bbdb5bb74903p-2, 0x1.091db2d92f66dp+0, 0x1.688a7cde833d1p-2,
    0x1.06df126716026p+0, 0x1.6548b506a2232p-2, 0x1.04a5b493c5ac1p+0, 0x1.61f83e89984bep-2,
    0x1.0271b0f957f4ep+0, 0x1.5e98fb01de3c3p-2, 0x1.00431f6180172p+0, 0x1.5b2acd619d4b9p-2,
    0x1.fc342f86aaa7ap-1, 0x1.57ad9a05f2cc3p-2, 0x1.f7ed6481fc8fep-1, 0x1.542146ca6fce7p-2,
    0x1.f3b20e4a79bcbp-1, 0x1.5085bb1ccdbcep-2, 0x1.ef825dc1b520fp-1, 0x1.4cdae010cf793p-2,
    0x1.eb5e840fe96b5p-1, 0x1.4920a0744611dp-2, 0x1.e746b29e515f7p-1, 0x1.4556e8e32f943p-2,
    0x1.e33b1b113fa55p-1, 0x1.417da7dbe5ec7p-2, 0x1.df3bef41f5ecfp-1, 0x1.3d94cdd35332ap-2,
    0x1.db4961383b665p-1, 0x1.399c4d4920352p-2, 0x1.d763a323b2b35p-1, 0x1.35941adbd182bp-2,
    0x1.d38ae754ef9e0p-1, 0x1.317c2d5cc6acfp-2, 0x1.cfbf60364d088p-1, 0x1.2d547de40ef74p-2,
    0x1.cc01404483b29p-1, 0x1.291d07e40624cp-2, 0x1.c850ba07029edp-1, 0x1.24d5c93cab9f3p-2,
    0x1.c4ae00080a0c4p-1, 0x1.207ec24ea5bd8p-2, 0x1.c11944cc8a291p-1, 0x1.1c17f60de2866p-2,
    0x1.bd92bacbc6d10p-1, 0x1.17a16a13c6e91p-2, 0x1.ba1a9466c1dcdp-1, 0x1.131b26b0dd111p-2,
    0x1.b6b103df6db67p-1, 0x1.0e8536fdf22c9p-2, 0x1.b3563b4faa1c6p-1, 0x1.09dfa8ec93bd4p-2,
    0x1.b00a6ca00d2e4p-1, 0x1.052a8d56dc5b1p-2, 0x1.accdc97e7b128p-1, 0x1.0065f80e7fa9bp-2,
    0x1.a9a083548eb86p-1, 0x1.f723ffd60a5e7p-3, 0x1.a682cb3dd66e6p-1, 0x1.ed5d7dae4369bp-3,
    0x1.a374d1fde7390p-1, 0x1.e378a3ba3dccdp-3, 0x1.a076c7f64a098p-1, 0x1.d975b264820a4p-3,
    0x1.9d88dd1c4628bp-1, 0x1.cf54f0823563fp-3, 0x1.9aab40ee8c5bdp-1, 0x1.c516ab657e31cp-3,
    0x1.97de226ac67b9p-1, 0x1.babb36ed863afp-3, 0x1.9521b0030f65fp-1, 0x1.b042ed93fd2edp-3,
    0x1.927617935762dp-1, 0x1.a5ae3077fe597p-3, 0x1.8fdb8656b93fdp-1, 0x1.9afd67663ddf2p-3,
    0x1.8d5228dcc4947p-1, 0x1.903100de631f7p-3, 0x1.8ada2afec1c74p-1, 0x1.854972157761ap-3,
    0x1.8873b7d4f494bp-1, 0x1.7a4736f551990p-3, 0x1.861ef9abe1fa1p-1, 0x1.6f2ad218e9e29p-3,
    0x1.83dc19f99e8a5p-1, 0x1.63f4ccc5815c4p-3, 0x1.81ab41532a4cdp-1, 0x1.58a5b6e08d1b6p-3,
    0x1.7f8c9761df626p-1, 0x1.4d3e26e25552ap-3, 0x1.7d8042d8f8c13p-1, 0x1.41beb9c53c26fp-3,
    0x1.7b86696b366b6p-1, 0x1.362812f1a246fp-3, 0x1.799f2fc0a490ep-1, 0x1.2a7adc2662074p-3,
    0x1.77cab96c8b170p-1, 0x1.1eb7c55ddc97bp-3, 0x1.760928e38b05ap-1, 0x1.12df84af97cbcp-3,
    0x1.745a9f71ef576p-1, 0x1.06f2d62e6df39p-3, 0x1.72bf3d3236a95p-1, 0x1.f5e4f786a8a56p-4,
    0x1.71372103db391p-1, 0x1.ddbe7a097fcd7p-4, 0x1.6fc268825e93cp-1, 0x1.c573ce1566b96p-4,
    0x1.6e612ffc9e438p-1, 0x1.ad06987f08932p-4, 0x1.6d13926c76afep-1, 0x1.9478885ad1e35p-4,
    0x1.6bd9a96eb947ap-1, 0x1.7bcb5691c6421p-4, 0x1.6ab38d3b7ae6fp-1, 0x1.6300c5703f8d5p-4,
    0x1.69a1549ebf444p-1, 0x1.4a1aa02ecc4e7p-4, 0x1.68a314f186016p-1, 0x1.311aba7569234p-4,
    0x1.67b8e2133dcaap-1, 0x1.1802efd956fc0p-4, 0x1.66e2ce63a1b92p-1, 0x1.fdaa46abab965p-5,
    0x1.6620eabd04ef0p-1, 0x1.cb267d8021a62p-5, 0x1.6573466f1026cp-1, 0x1.987e646d1e0bdp-5,
    0x1.64d9ef39f4a9bp-1, 0x1.65b5e718fdd09p-5, 0x1.6454f14a17d9ap-1, 0x1.32d0fb6274144p-5,
    0x1.63e457343a2f3p-1, 0x1.ffa7405181bd4p-6, 0x1.638829f21c3e6p-1, 0x1.9983b81bc0859p-6,
    0x1.634070dfa4028p-1, 0x1.333f7867025b5p-6, 0x1.630d31b8845dbp-1, 0x1.99c54bce64e3dp-7,
    0x1.62ee709668617p-1, 0x1.99d5b4ab7f73cp-8, 0x1.62e42fefa39efp-1, 0x0.0p+0,
    0x1.62ee709668617p-1, -0x1.99d5b4ab7f73cp-8, 0x1.630d31b8845dbp-1, -0x1.99c54bce64e3dp-7,
    0x1.634070dfa4028p-1, -0x1.333f7867025b5p-6, 0x1.638829f21c3e6p-1, -0x1.9983b81bc0859p-6,
    0x1.63e457343a2f3p-1, -0x1.ffa7405181bd4p-6, 0x1.6454f14a17d9ap-1, -0x1.32d0fb6274144p-5,
    0x1.64d9ef39f4a9bp-1, -0x1.65b5e718fdd09p-5, 0x1.6573466f1026cp-1, -0x1.987e646d1e0bdp-5,
    0x1.6620eabd04ef0p-1, -0x1.cb267d8021a62p-5, 0x1.66e2ce63a1b92p-1, -0x1.fdaa46abab965p-5,
    0x1.67b8e2133dcaap-1, -0x1.1802efd956fc0p-4, 0x1.68a314f186016p-1, -0x1.311aba7569234p-4,
    0x1.69a1549ebf444p-1, -0x1.4a1aa02ecc4e7p-4, 0x1.6ab38d3b7ae6fp-1, -0x1.6300c5703f8d5p-4,
    0x1.6bd9a96eb947ap-1, -0x1.7bcb5691c6421p-4, 0x1.6d13926c76afep-1, -0x1.9478885ad1e35p-4,
    0x1.6e612ffc9e438p-1, -0x1.ad06987f08932p-4, 0x1.6fc268825e93cp-1, -0x1.c573ce1566b96p-4,
    0x1.71372103db391p-1, -0x1.ddbe7a097fcd7p-4, 0x1.72bf3d3236a95p-1, -0x1.f5e4f786a8a56p-4,
    0x1.745a9f71ef576p-1, -0x1.06f2d62e6df39p-3, 0x1.760928e38b05ap-1, -0x1.12df84af97cbcp-3,
    0x1.77cab96c8b170p-1, -0x1.1eb7c55ddc97bp-3, 0x1.799f2fc0a490ep-1, -0x1.2a7adc2662074p-3,
    0x1.7b86696b366b6p-1, -0x1.362812f1a246fp-3, 0x1.7d8042d8f8c13p-1, -0x1.41beb9c53c26fp-3,
    0x1.7f8c9761df626p-1, -0x1.4d3e26e25552ap-3, 0x1.81ab41532a4cdp-1, -0x1.58a5b6e08d1b6p-3,
    0x1.83dc19f99e8a5p-1, -0x1.63f4ccc5815c4p-3, 0x1.861ef9abe1fa1p-1, -0x1.6f2ad218e9e29p-3,
    0x1.8873b7d4f494bp-1, -0x1.7a4736f551990p-3, 0x1.8ada2afec1c74p-1, -0x1.854972157761ap-3,
    0x1.8d5228dcc4947p-1, -0x1.903100de631f7p-3, 0x1.8fdb8656b93fdp-1, -0x1.9afd67663ddf2p-3,
    0x1.927617935762dp-1, -0x1.a5ae3077fe597p-3, 0x1.9521b0030f65fp-1, -0x1.b042ed93fd2edp-3,
    0x1.97de226ac67b9p-1, -0x1.babb36ed863afp-3, 0x1.9aab40ee8c5bdp-1, -0x1.c516ab657e31cp-3,
    0x1.9d88dd1c4628bp-1, -0x1.cf54f0823563fp-3, 0x1.a076c7f64a098p-1, -0x1.d975b264820a4p-3,
    0x1.a374d1fde7390p-1, -0x1.e378a3ba3dccdp-3, 0x1.a682cb3dd66e6p-1, -0x1.ed5d7dae4369bp-3,
    0x1.a9a083548eb86p-1, -0x1.f723ffd60a5e7p-3, 0x1.accdc97e7b128p-1, -0x1.0065f80e7fa9bp-2,
    0x1.b00a6ca00d2e4p-1, -0x1.052a8d56dc5b1p-2, 0x1.b3563b4faa1c6p-1, -0x1.09dfa8ec93bd4p-2,
    0x1.b6b103df6db67p-1, -0x1.0e8536fdf22c9p-2, 0x1.ba1a9466c1dcdp-1, -0x1.131b26b0dd111p-2,
    0x1.bd92bacbc6d10p-1, -0x1.17a16a13c6e91p-2, 0x1.c11944cc8a291p-1, -0x1.1c17f60de2866p-2,
    0x1.c4ae00080a0c4p-1, -0x1.207ec24ea5bd8p-2, 0x1.c850ba07029edp-1, -0x1.24d5c93cab9f3p-2,
    0x1.cc01404483b29p-1, -0x1.291d07e40624cp-2, 0x1.cfbf60364d088p-1, -0x1.2d547de40ef74p-2,
    0x1.d38ae754ef9e0p-1, -0x1.317c2d5cc6acfp-2, 0x1.d763a323b2b35p-1, -0x1.35941adbd182bp-2,
    0x1.db4961383b665p-1, -0x1.399c4d4920352p-2, 0x1.df3bef41f5ecfp-1, -0x1.3d94cdd35332ap-2,
    0x1.e33b1b113fa55p-1, -0x1.417da7dbe5ec7p-2, 0x1.e746b29e515f7p-1, -0x1.4556e8e32f943p-2,
    0x1.eb5e840fe96b5p-1, -0x1.4920a0744611dp-2, 0x1.ef825dc1b520fp-1, -0x1.4cdae010cf793p-2,
    0x1.f3b20e4a79bcbp-1, -0x1.5085bb1ccdbcep-2, 0x1.f7ed6481fc8fep-1, -0x1.542146ca6fce7p-2,
    0x1.fc342f86aaa7ap-1, -0x1.57ad9a05f2cc3p-2, 0x1.00431f6180172p+0, -0x1.5b2acd619d4b9p-2,
    0x1.0271b0f957f4ep+0, -0x1.5e98fb01de3c3p-2, 0x1.04a5b493c5ac1p+0, -0x1.61f83e89984bep-2,
    0x1.06df126716026p+0, -0x1.6548b506a2232p-2, 0x1.091db2d92f66dp+0, -0x1.688a7cde833d1p-2,
    0x1.0b617e81a8f31p+0, -0x1.6bbdb5bb74903p-2, 0x1.0daa5e2bc33cep+0, -0x1.6ee28079abad1p-2,
    0x1.0ff83ad843749p+0, -0x1.71f8ff14f66d7p-2, 0x1.124afdbf3155bp+0, -0x1.75015496acc4ap-2,
    0x1.14a290517877fp+0, -0x1.77fba503fdbddp-2, 0x1.16fedc3a6d95cp+0, -0x1.7ae8154c9c312p-2,
    0x1.195fcb613865bp+0, -0x1.7dc6cb39cf3c9p-2, 0x1.1bc547ea22a87p+0, -0x1.8097ed5dea11fp-2,
    0x1.1e2f3c37cd14bp+0, -0x1.835ba3042e38cp-2, 0x1.209d92ec4acbap+0, -0x1.861214211aee3p-2,
    0x1.231036ea2408cp+0, -0x1.88bb69432be5cp-2, 0x1.2587135540befp+0, -0x1.8b57cb840942dp-2,
    0x1.28021393bbdafp+0, -0x1.8de7647a2a42fp-2, 0x1.2a81234e9fe22p+0, -0x1.906a5e2aebb2ap-2,
    0x1.2d042e728da94p+0, -0x1.92e0e2fd1aef2p-2, 0x1.2f8b21304ddcdp+0, -0x1.954b1dabf5e36p-2,
    0x1.3215e7fd4e175p+0, -0x1.97a9393aa020dp-2, 0x1.34a46f940a407p+0, -0x1.99fb60e80cebbp-2,
    0x1.3736a4f462effp+0, -0x1.9c41c0235dcc4p-2, 0x1.39cc7563e18f2p+0, -0x1.9e7c8280b4f94p-2,
    0x1.3c65ce6deaf02p+0, -0x1.a0abd3ae7ab21p-2, 0x1.3f029de3e1144p+0, -0x1.a2cfdf6b146afp-2,
    0x1.41a2d1dd34d41p+0, -0x1.a4e8d17b0c78dp-2, 0x1.444658b7681ecp+0, -0x1.a6f6d59fa8bf5p-2,
    0x1.46ed2116017f3p+0, -0x1.a8fa178deeb73p-2, 0x1.499719e271951p+0, -0x1.aaf2c2e612ff3p-2,
    0x1.4c44324beb2d6p+0, -0x1.ace1032b52868p-2, 0x1.4ef459c72ea02p+0, -0x1.aec503bc33429p-2,
    0x1.51a7800e49190p+0, -0x1.b09eefcb2a461p-2, 0x1.545d9520486a8p+0, -0x1.b26ef257a4f87p-2,
    0x1.57168940e4086p+0, -0x1.b435362773184p-2, 0x1.59d24cf81bc32p+0, -0x1.b5f1e5c08f224p-2,
    0x1.5c90d111ccd8fp+0, -0x1.b7a52b6342a76p-2, 0x1.5f52069d3dedbp+0, -0x1.b94f3104a4110p-2,
    0x1.6215deeca2775p+0, -0x1.baf020496b4a0p-2, 0x1.64dc4b949626bp+0, -0x1.bc8822811aba4p-2,
    0x1.67a53e6b90d37p+0, -0x1.be1760a179fffp-2, 0x1.6a70a989536a3p+0, -0x1.bf9e03425fce4p-2,
    0x1.6d3e7f464e5a3p+0, -0x1.c11c3299c8574p-2, 0x1.700eb23b01fb7p+0, -0x1.c292167835aabp-2,
    0x1.72e1353f5960dp+0, -0x1.c3ffd64557728p-2, 0x1.75b5fb6a0006ap+0, -0x1.c56598fcf77d9p-2,
    0x1.788cf80fb2ca7p+0, -0x1.c6c3852c288bap-2, 0x1.7b661ec28c92cp+0, -0x1.c819c0eeb4d6cp-2,
    0x1.7e4163514f0c0p+0, -0x1.c96871ecc9dc2p-2, 0x1.811eb9c6a7da8p+0, -0x1.caafbd58def23p-2,
    0x1.83fe1668729cdp+0, -0x1.cbefc7edd43fdp-2, 0x1.86df6db6f8186p+0, -0x1.cd28b5ed47b70p-2,
    0x1.89c2b46c2ae34p+0, -0x1.ce5aab1e1dbe7p-2, 0x1.8ca7df7ae1ddbp+0, -0x1.cf85cacb3b423p-2,
    0x1.8f8ee40e10c75p+0, -0x1.d0aa37c26ef00p-2, 0x1.9277b787ff3a6p+0, -0x1.d1c8145387720p-2,
    0x1.95624f817e53cp+0, -0x1.d2df824f94867p-2, 0x1.984ea1c91d498p+0, -0x1.d3f0a30850e14p-2,
    0x1.9b3ca4625d315p+0, -0x1.d4fb974fb2d45p-2, 0x1.9e2c4d84e4318p+0, -0x1.d6007f77a1c5fp-2,
    0x1.a11d939bb057ap+0, -0x1.d6ff7b51ce8f9p-2, 0x1.a4106d444a49ap+0, -0x1.d7f8aa2face92p-2,
    0x1.a704d14df8065p+0, -0x1.d8ec2ae28c186p-2, 0x1.a9fab6b8efe52p+0, -0x1.d9da1bbbcd263p-2,
    0x1.acf214b58c02ap+0, -0x1.dac29a8d34ec8p-2, 0x1.afeae2a37e467p+0, -0x1.dba5c4a9585e3p-2,
    0x1.b2e518110529ep+0, -0x1.dc83b6e421775p-2, 0x1.b5e0acba21663p+0, -0x1.dd5c8d936b536p-2,
    0x1.b8dd9887ccaebp+0, -0x1.de30648fb3f47p-2, 0x1.bbdbd38f31974p+0, -0x1.deff5734e2557p-2,
    0x1.bedb5610e4c7fp+0, -0x1.dfc980631f6dbp-2, 0x1.c1dc18781f99ep+0, -0x1.e08efa7fc0d9dp-2,
    0x1.c4de1359fc396p+0, -0x1.e14fdf7643ecfp-2, 0x1.c7e13f74b3664p+0, -0x1.e20c48b957f74p-2,
    0x1.cae595aedbe9ep+0, -0x1.e2c44f43f69dcp-2, 0x1.cdeb0f16abd87p+0, -0x1.e3780b9a892b3p-2,
    0x1.d0f1a4e13bb20p+0, -0x1.e42795cc19cc8p-2, 0x1.d3f95069cb745p+0, -0x1.e4d305738fb9bp-2,
    0x1.d7020b3109af8p+0, -0x1.e57a71b8f5556p-2, 0x1.da0bcedc5cac2p+0, -0x1.e61df152c7586p-2,
    0x1.dd1695352db08p+0, -0x1.e6bd9a874c2bep-2, 0x1.e022582836717p+0, -0x1.e759832df29c1p-2,
    0x1.e32f11c4d0ba3p+0, -0x1.e7f1c0b0b719fp-2, 0x1.e63cbc3c4854ep+0, -0x1.e886680d8ecb0p-2,
    0x1.e94b51e12f3c7p+0, -0x1.e9178dd7d7b10p-2, 0x1.ec5acd26b41fdp+0, -0x1.e9a54639cd3b7p-2,
    0x1.ef6b289ffb3c1p+0, -0x1.ea2fa4f6009e1p-2, 0x1.f27c5eff79945p+0, -0x1.eab6bd68d4513p-2,
    0x1.f58e6b16528b5p+0, -0x1.eb3aa289fa275p-2, 0x1.f8a147d3b7e1ep+0, -0x1.ebbb66edf36cfp-2,
    0x1.fbb4f0444c1e5p+0, -0x1.ec391cc7928eep-2, 0x1.fec95f91875d9p+0, -0x1.ecb3d5e97dc9ep-2,
    0x1.00ef48808f484p+1, -0x1.ed2ba3c7b26f4p-2, 0x1.027a3ffa36928p+1, -0x1.eda09779084f8p-2,
    0x1.040593f3f08d9p+1, -0x1.ee12c1b8b4e38p-2, 0x1.0591423934c32p+1, -0x1.ee8232e7cdd2ap-2,
    0x1.071d48a273bbap+1, -0x1.eeeefb0eca7acp-2, 0x1.08a9a514d0a81p+1, -0x1.ef5929df04244p-2,
    0x1.0a365581dc3e1p+1, -0x1.efc0ceb43492dp-2, 0x1.0bc357e750c62p+1, -0x1.f025f895f2a71p-2,
    0x1.0d50aa4ecf594p+1, -0x1.f088b6392ccdap-2, 0x1.0ede4acd9e4c6p+1, -0x1.f0e91601a0f8bp-2,
    0x1.106c378468c87p+1, -0x1.f147260351ea1p-2, 0x1.11fa6e9eff8b6p+1, -0x1.f1a2f403f9951p-2,
    0x1.1388ee541ad0cp+1, -0x1.f1fc8d7c78657p-2, 0x1.1517b4e51d5eep+1, -0x1.f253ff9a413c0p-2,
    0x1.16a6c09dd8b65p+1, -0x1.f2a95740c1f57p-2, 0x1.18360fd452601p+1, -0x1.f2fca10ac853ep-2,
    0x1.19c5a0e88a583p+1, -0x1.f34de94be326bp-2, 0x1.1b5572444291bp+1, -0x1.f39d3c11bf8f8p-2,
    0x1.1ce5825ac7905p+1, -0x1.f3eaa52582473p-2, 0x1.1e75cfa8ba14fp+1, -0x1.f436300d1cc73p-2,
    0x1.200658b3d9d99p+1, -0x1.f47fe80c9e3f9p-2, 0x1.21971c0ad1594p+1, -0x1.f4c7d82780447p-2,
    0x1.2328184502a0ep+1, -0x1.f50e0b21ef202p-2, 0x1.24b94c0255247p+1, -0x1.f5528b820db93p-2,
    0x1.264ab5eb04965p+1, -0x1.f595639134fe3p-2, 0x1.27dc54af70bc4p+1, -0x1.f5d69d5d2ecbep-2,
    0x1.296e2707ee3e8p+1, -0x1.f61642b96c42ap-2, 0x1.2b002bb4986dcp+1, -0x1.f6545d4037842p-2,
    0x1.2c92617d23fbbp+1, -0x1.f690f653e0d20p-2, 0x1.2e24c730b2a33p+1, -0x1.f6cc171fe7096p-2,
    0x1.2fb75ba5a7bb4p+1, -0x1.f705c89a1b784p-2, 0x1.314a1db97db2bp+1, -0x1.f73e1383c10a4p-2,
    0x1.32dd0c509c6eap+1, -0x1.f775006aa6cdfp-2, 0x1.34702656308abp+1, -0x1.f7aa97aa3dd26p-2,
    0x1.36036abc03745p+1, -0x1.f7dee16caa604p-2, 0x1.3796d87a54601p+1, -0x1.f811e5abd0914p-2,
    0x1.392a6e8fb213bp+1, -0x1.f843ac325c4adp-2, 0x1.3abe2c00d5813p+1, -0x1.f8743c9cc4a0ep-2,
    0x1.3c520fd87d30bp+1, -0x1.f8a39e5a4aa85p-2, 0x1.3de6192749739p+1, -0x1.f8d1d8adf3be8p-2,
    0x1.3f7a4703995ebp+1, -0x1.f8fef2af7f4ffp-2, 0x1.410e988968874p+1, -0x1.f92af34c58250p-2,
    0x1.42a30cda2d7f4p+1, -0x1.f955e148813f4p-2, 0x1.4437a31cb90d8p+1, -0x1.f97fc33f7e512p-2,
    0x1.45cc5a7d161e8p+1, -0x1.f9a89fa537da3p-2, 0x1.4761322c6a69ap+1, -0x1.f9d07cc6daf34p-2,
    0x1.48f62960d7c81p+1, -0x1.f9f760cbb4d69p-2, 0x1.4a8b3f555e39cp+1, -0x1.fa1d51b60a2ebp-2,
    0x1.4c207349be94fp+1, -0x1.fa425563ea39ep-2, 0x1.4db5c4825ddd3p+1, -0x1.fa66718ffdcd4p-2,
    0x1.4f4b3248293e4p+1, -0x1.fa89abd252469p-2, 0x1.50e0bbe87aa83p+1, -0x1.faac09a12077dp-2,
    0x1.527660b4fe08bp+1, -0x1.facd90518f9bdp-2, 0x1.540c2003971f5p+1, -0x1.faee45187460dp-2,
    0x1.55a1f92e47e89p+1, -0x1.fb0e2d0b0c16dp-2, 0x1.5737eb93179ddp+1, -0x1.fb2d4d1fb410ep-2,
    0x1.58cdf693fa467p+1, -0x1.fb4baa2e9d458p-2, 0x1.5a641996b8d6dp+1, -0x1.fb6948f27c3eep-2,
    0x1.5bfa5404d9db1p+1, -0x1.fb862e0935674p-2, 0x1.5d90a54b8aaa8p+1, -0x1.fba25df485c13p-2,
    0x1.5f270cdb89202p+1, -0x1.fbbddd1aa819bp-2, 0x1.60bd8a290dd69p+1, -0x1.fbd8afc6f6c2cp-2,
    0x1.62541cabb6e3ap+1, -0x1.fbf2da2a89e4bp-2, 0x1.63eac3de73118p+1, -0x1.fc0c605cd2755p-2,
    0x1.65817f3f6d92cp+1, -0x1.fc25465c31e29p-2, 0x1.67184e4ffa2e5p+1, -0x1.fc3d900e8e7fbp-2,
    0x1.68af309481e0bp+1, -0x1.fc554141e4c30p-2, 0x1.6a4625946ff0fp+1, -0x1.fc6c5dacd562dp-2,
    0x1.6bdd2cda1f757p+1, -0x1.fc82e8ef305f1p-2, 0x1.6d7445f2c9472p+1, -0x1.fc98e6927d070p-2,
    0x1.6f0b706e72606p+1, -0x1.fcae5a0a7f078p-2, 0x1.70a2abdfdaa52p+1, -0x1.fcc346b5b890dp-2,
    0x1.7239f7dc6c122p+1, -0x1.fcd7afdde9a1bp-2, 0x1.73d153fc2a50fp+1, -0x1.fceb98b88c84dp-2,
    0x1.7568bfd9a2ae8p+1, -0x1.fcff04674f8eap-2, 0x1.77003b11dc722p+1, -0x1.fd11f5f88c28ep-2,
    0x1.7897c54449926p+1, -0x1.fd247067bb38dp-2, 0x1.7a2f5e12b7c6bp+1, -0x1.fd36769de6edep-2,
    0x1.7bc7052141f29p+1, -0x1.fd480b721a04ep-2, 0x1.7d5eba1641e91p+1, -0x1.fd5931a9cc8d2p-2,
    0x1.7ef67c9a42864p+1, -0x1.fd69ebf94e3c5p-2, 0x1.808e4c57f21d0p+1, -0x1.fd7a3d042e5c8p-2,
    0x1.822628fc1536dp+1, -0x1.fd8a275da1624p-2, 0x1.83be123579a44p+1, -0x1.fd99ad88e4356p-2,
    0x1.855607b4e9dbcp+1, -0x1.fda8d1f99d395p-2, 0x1.86ee092d20a55p+1, -0x1.fdb797143b205p-2,
    0x1.88861652bd115p+1, -0x1.fdc5ff2e51961p-2, 0x1.8a1e2edc36b88p+1, -0x1.fdd40c8ef3cb4p-2,
    0x1.8bb65281d243cp+1, -0x1.fde1c16f0ceffp-2, 0x1.8d4e80fd9639ap+1, -0x1.fdef1ff9b6a52p-2,
    0x1.8ee6ba0b4010cp+1, -0x1.fdfc2a4c8d72ep-2, 0x1.907efd6839849p+1, -0x1.fe08e278034bap-2,
    0x1.92174ad38e2bap+1, -0x1.fe154a7fb028fp-2, 0x1.93afa20de14dap+1, -0x1.fe21645aa0cb0p-2,
    0x1.954802d963f7bp+1, -0x1.fe2d31f3a3a54p-2, 0x1.96e06cf9cb4dap+1, -0x1.fe38b5299402bp-2,
    0x1.9878e03447169p+1, -0x1.fe43efcfa36b0p-2, 0x1.9a115c4f78837p+1, -0x1.fe4ee3ada152cp-2,
    0x1.9ba9e113692ecp+1, -0x1.fe599280411fep-2, 0x1.9d426e4982532p+1, -0x1.fe63fdf95e8b5p-2,
    0x1.9edb03bc84386p+1, -0x1.fe6e27c0406a8p-2, 0x1.a073a1387dd50p+1, -0x1.fe781171d9e79p-2,
    0x1.a20c468ac4a3ep+1, -0x1.fe81bca10a32ap-2, 0x1.a3a4f381ecabbp+1, -0x1.fe8b2ad6dab4bp-2,
    0x1.a53da7edc0b7fp+1, -0x1.fe945d92bbcb8p-2, 0x1.a6d6639f3ac20p+1, -0x1.fe9d564ac0180p-2,
    0x1.a86f26687c88dp+1, -0x1.fea6166bd6672p-2, 0x1.aa07f01cc856ep+1, -0x1.feae9f5a023c6p-2,
    0x1.aba0c09079f44p+1, -0x1.feb6f2709306dp-2, 0x1.ad399798ffc51p+1, -0x1.febf11025a07ap-2,
    0x1.aed2750cd411dp+1, -0x1.fec6fc59def26p-2, 0x1.b06b58c3767a1p+1, -0x1.feceb5b9934d3p-2,
    0x1.b2044295658f5p+1, -0x1.fed63e5c0499ep-2, 0x1.b39d325c18977p+1, -0x1.fedd97740d4d2p-2,
    0x1.b53627f1f9766p+1, -0x1.fee4c22d049c4p-2, 0x1.b6cf23325ebd3p+1, -0x1.feebbfaaed276p-2,
    0x1.b86823f985de2p+1, -0x1.fef2910aa2874p-2, 0x1.ba012a248d84ep+1, -0x1.fef9376205c4fp-2,
    0x1.bb9a35917011ap+1, -0x1.feffb3c028c1cp-2, 0x1.bd33461efe371p+1, -0x1.ff06072d7895ap-2,
    0x1.becc5bacd9b92p+1, -0x1.ff0c32abe6ea9p-2, 0x1.c065761b704d3p+1, -0x1.ff123737125a8p-2,
    0x1.c1fe954bf6998p+1, -0x1.ff1815c46dd5ap-2, 0x1.c397b92063547p+1, -0x1.ff1dcf4367172p-2,
    0x1.c530e17b6a81ap+1, -0x1.ff23649d8c2dbp-2, 0x1.c6ca0e4078cd1p+1, -0x1.ff28d6b6b01dap-2,
    0x1.c8633f53af034p+1, -0x1.ff2e266d0ea15p-2, 0x1.c9fc7499dda51p+1, -0x1.ff3354996f0dfp-2,
    0x1.cb95adf880983p+1, -0x1.ff38620f46616p-2, 0x1.cd2eeb55baf15p+1, -0x1.ff3d4f9cd87e1p-2,
    0x1.cec82c9852d9dp+1, -0x1.ff421e0b5899dp-2, 0x1.d06171a7ad8dfp+1, -0x1.ff46ce1f08e52p-2,
    0x1.d1faba6bcb750p+1, -0x1.ff4b6097596e6p-2, 0x1.d39406cd44516p+1, -0x1.ff4fd62f06467p-2,
    0x1.d52d56b543887p+1, -0x1.ff542f9c34eb3p-2, 0x1.d6c6aa0d84821p+1, -0x1.ff586d9090fbdp-2,
    0x1.d86000c04f1e8p+1, -0x1.ff5c90b9683b8p-2, 0x1.d9f95ab874428p+1, -0x1.ff6099bfc5e6dp-2,
    0x1.db92b7e14a791p+1, -0x1.ff6489488d5fap-2, 0x1.dd2c1826aaaa5p+1, -0x1.ff685ff49433dp-2,
    0x1.dec57b74ece6fp+1, -0x1.ff6c1e60bb829p-2, 0x1.e05ee1b8e547bp+1, -0x1.ff6fc52608c3dp-2,
    0x1.e1f84adfe0e08p+1, -0x1.ff7354d9bdf65p-2, 0x1.e391b6d7a2c69p+1, -0x1.ff76ce0d71374p-2,
    0x1.e52b258e61296p+1, -0x1.ff7a314f23c76p-2, 0x1.e6c496f2c27ddp+1, -0x1.ff7d7f295880dp-2,
    0x1.e85e0af3dabaep+1, -0x1.ff80b82329c1ap-2, 0x1.e9f7818128a7ep+1, -0x1.ff83dcc05ecdcp-2,
    0x1.eb90fa8a933b9p+1, -0x1.ff86ed8180ab9p-2, 0x1.ed2a7600670bbp+1, -0x1.ff89eae3ee7f4p-2,
    0x1.eec3f3d353cc9p+1, -0x1.ff8cd561f166dp-2, 0x1.f05d73f469e0ap+1, -0x1.ff8fad72cfda6p-2,
    0x1.f1f6f65517f72p+1, -0x1.ff92738ae0942p-2, 0x1.f3907ae728b96p+1, -0x1.ff95281b9d01ap-2,
    0x1.f52a019cc087ap+1, -0x1.ff97cb93b342fp-2, 0x1.f6c38a685b42ep+1, -0x1.ff9a5e5f17b8bp-2,
    0x1.f85d153cca25cp+1, -0x1.ff9ce0e716250p-2, 0x1.f9f6a20d31a9fp+1, -0x1.ff9f539262616p-2,
    0x1.fb9030cd077bap+1, -0x1.ffa1b6c528ac0p-2, 0x1.fd29c17010795p+1, -0x1.ffa40ae11d8f7p-2,
    0x1.fec353ea5ec05p+1, -0x1.ffa650458d66cp-2, 0x1.002e741827e2ep+2, -0x1.ffa8874f6b80ep-2,
    0x1.00fb3f1b453dap+2, -0x1.ffaab05960e4cp-2, 0x1.01c80af8febfap+2, -0x1.ffaccbbbdab9cp-2,
    0x1.0294d7abeeaccp+2, -0x1.ffaed9cd18559p-2, 0x1.0361a52ed1609p+2, -0x1.ffb0dae138f23p-2,
    0x1.042e737c84778p+2, -0x1.ffb2cf4a490dfp-2, 0x1.04fb429005fd2p+2, -0x1.ffb4b7584f782p-2,
    0x1.05c81264739f3p+2, -0x1.ffb693595a0bbp-2, 0x1.0694e2f509e68p+2, -0x1.ffb863998a19cp-2,
    0x1.0761b43d23739p+2, -0x1.ffba286320871p-2, 0x1.082e863838416p+2, -0x1.ffbbe1fe899d3p-2,
    0x1.08fb58e1dceb8p+2, -0x1.ffbd90b268916p-2, 0x1.09c82c35c1fa0p+2, -0x1.ffbf34c3a2c35p-2,
    0x1.0a95002fb330cp+2, -0x1.ffc0ce756ab59p-2, 0x1.0b61d4cb96e3bp+2, -0x1.ffc25e094ac10p-2,
    0x1.0c2eaa056d4f5p+2, -0x1.ffc3e3bf2f84dp-2, 0x1.0cfb7fd94ff4cp+2, -0x1.ffc55fd57215ap-2,
    0x1.0dc8564370fa9p+2, -0x1.ffc6d288e1ec1p-2, 0x1.0e952d401a912p+2, -0x1.ffc83c14ce957p-2,
    0x1.0f6204cbae5a9p+2, -0x1.ffc99cb311272p-2, 0x1.102edce2a4d73p+2, -0x1.ffcaf49c15773p-2,
    0x1.10fbb5818cd4bp+2, -0x1.ffcc4406e31a7p-2, 0x1.11c88ea50ae19p+2, -0x1.ffcd8b29262a6p-2,
    0x1.12956849d8c3ap+2, -0x1.ffceca3737d3fp-2, 0x1.1362426cc4f23p+2, -0x1.ffd0016426b08p-2,
    0x1.142f1d0ab2132p+2, -0x1.ffd130e1beea1p-2, 0x1.14fbf820967bap+2, -0x1.ffd258e0922d0p-2,
    0x1.15c8d3ab7bb3fp+2, -0x1.ffd3798fff66cp-2, 0x1.1695afa87dfddp+2, -0x1.ffd4931e3a552p-2,
    0x1.17628c14cbde7p+2, -0x1.ffd5a5b852e4ep-2, 0x1.182f68eda5ab4p+2, -0x1.ffd6b18a3c629p-2,
    0x1.18fc46305d18fp+2, -0x1.ffd7b6bed47e2p-2, 0x1.19c923da54ce4p+2, -0x1.ffd8b57fea222p-2,
    0x1.1a9601e8fff89p+2, -0x1.ffd9adf644202p-2, 0x1.1b62e059e1e3bp+2, -0x1.ffdaa049a7b2bp-2,
    0x1.1c2fbf2a8d93fp+2, -0x1.ffdb8ca0ded73p-2, 0x1.1cfc9e58a562fp+2, -0x1.ffdc7321be7ecp-2,
    0x1.1dc97de1da9eap+2, -0x1.ffdd53f12c98ep-2, 0x1.1e965dc3ed2adp+2, -0x1.ffde2f3325f79p-2,
    0x1.1f633dfcab252p+2, -0x1.ffdf050ac40ebp-2, 0x1.20301e89f08afp+2, -0x1.ffdfd59a428f0p-2,
    0x1.20fcff69a6e1fp+2, -0x1.ffe0a10304ddcp-2, 0x1.21c9e099c4e28p+2, -0x1.ffe167659b6a3p-2,
    0x1.2296c2184e244p+2, -0x1.ffe228e1c8e10p-2, 0x1.2363a3e352ccdp+2, -0x1.ffe2e596873f7p-2,
    0x1.243085f8ef408p+2, -0x1.ffe39da20cc5fp-2, 0x1.24fd68574bd4dp+2, -0x1.ffe45121d0cc3p-2,
    0x1.25ca4afc9c853p+2, -0x1.ffe5003290768p-2, 0x1.26972de720a92p+2, -0x1.ffe5aaf0534d0p-2,
    0x1.2764111522ac9p+2, -0x1.ffe651766fb6dp-2, 0x1.2830f484f7c9fp+2, -0x1.ffe6f3df8f586p-2,
    0x1.28fdd834ffc5ap+2, -0x1.ffe79245b3563p-2, 0x1.29cabc23a4abbp+2, -0x1.ffe82cc2387d2p-2,
    0x1.2a97a04f5a8e8p+2, -0x1.ffe8c36ddb502p-2, 0x1.2b6484b69f47ep+2, -0x1.ffe95660bbfc7p-2,
    0x1.2c316957fa3acp+2, -0x1.ffe9e5b262353p-2, 0x1.2cfe4e31fc175p+2, -0x1.ffea7179c0f62p-2,
    0x1.2dcb33433e9ffp+2, -0x1.ffeaf9cd3a2f2p-2, 0x1.2e98188a64703p+2, -0x1.ffeb7ec2a2582p-2,
    0x1.2f64fe0618c47p+2, -0x1.ffec006f43ef0p-2, 0x1.3031e3b50f43dp+2, -0x1.ffec7ee7e2dedp-2,
    0x1.30fec99603ca8p+2, -0x1.ffecfa40bfd21p-2, 0x1.31cbafa7ba367p+2, -0x1.ffed728d9b6fcp-2,
    0x1.329895e8fe341p+2, -0x1.ffede7e1b9843p-2, 0x1.33657c58a30d9p+2, -0x1.ffee5a4fe4157p-2,
    0x1.343262f5837a6p+2, -0x1.ffeec9ea6e651p-2, 0x1.34ff49be81704p+2, -0x1.ffef36c337de3p-2,
    0x1.35cc30b285f5bp+2, -0x1.ffefa0ebaef15p-2, 0x1.369917d080f51p+2, -0x1.fff00874d3de6p-2,
    0x1.3765ff1769113p+2, -0x1.fff06d6f3b6ccp-2, 0x1.3832e6863b7aap+2, -0x1.fff0cfeb11924p-2,
    0x1.38ffce1bfbc6ap+2, -0x1.fff12ff81c09cp-2, 0x1.39ccb5d7b3c67p+2, -0x1.fff18da5bcd8bp-2,
    0x1.3a999db8735fep+2, -0x1.fff1e902f4c59p-2, 0x1.3b6685bd50671p+2, -0x1.fff2421e65be0p-2,
    0x1.3c336de56678dp+2, -0x1.fff29906552e9p-2, 0x1.3d00562fd6d60p+2, -0x1.fff2edc8ae4adp-2,
    0x1.3dcd3e9bc8403p+2, -0x1.fff340730447fp-2, 0x1.3e9a272866d68p+2, -0x1.fff3911294887p-2,
    0x1.3f670fd4e3f3dp+2, -0x1.fff3dfb448bacp-2, 0x1.4033f8a0760ddp+2, -0x1.fff42c64b8ea2p-2,
    0x1.4100e18a58948p+2, -0x1.fff477302d82ap-2, 0x1.41cdca91cbd2fp+2, -0x1.fff4c022a1483p-2,
    0x1.429ab3b614d06p+2, -0x1.fff50747c341bp-2, 0x1.43679cf67d324p+2, -0x1.fff54caaf8975p-2,
    0x1.44348652531f7p+2, -0x1.fff590575e65dp-2, 0x1.45016fc8e9232p+2, -0x1.fff5d257cb856p-2,
    0x1.45ce595996118p+2, -0x1.fff612b6d2463p-2, 0x1.469b4303b4ecap+2, -0x1.fff6517ec2217p-2,
    0x1.47682cc6a4c9ap+2, -0x1.fff68eb9a95fbp-2, 0x1.483516a1c8b78p+2, -0x1.fff6ca7156b53p-2,
    0x1.4902009487a58p+2, -0x1.fff704af5ad36p-2, 0x1.49ceea9e4c4b0p+2, -0x1.fff73d7d09f14p-2,
    0x1.4a9bd4be850f3p+2, -0x1.fff774e37d497p-2, 0x1.4b68bef4a3f21p+2, -0x1.fff7aaeb948efp-2,
    0x1.4c35a9401e75bp+2, -0x1.fff7df9df7594p-2, 0x1.4d0293a06d87cp+2, -0x1.fff8130316866p-2,
    0x1.4dcf7e150d6c4p+2, -0x1.fff845232d956p-2, 0x1.4e9c689d7da82p+2, -0x1.fff8760643f77p-2,
    0x1.4f69533940ecep+2, -0x1.fff8a5b42e58fp-2, 0x1.50363de7dd047p+2, -0x1.fff8d4348fe28p-2,
    0x1.510328a8dabd9p+2, -0x1.fff9018edb71fp-2, 0x1.51d0137bc5d8cp+2, -0x1.fff92dca54cb9p-2,
    0x1.529cfe602cf5ap+2, -0x1.fff958ee11c40p-2, 0x1.5369e955a180ep+2, -0x1.fff98300fb626p-2,
    0x1.5436d45bb7a26p+2, -0x1.fff9ac09cefc0p-2, 0x1.5503bf72062c1p+2, -0x1.fff9d40f1f482p-2,
    0x1.55d0aa9826890p+2, -0x1.fff9fb17556d9p-2, 0x1.569d95cdb4acfp+2, -0x1.fffa2128b209bp-2,
    0x1.576a81124f047p+2, -0x1.fffa46494e306p-2, 0x1.58376c659664fp+2, -0x1.fffa6a7f1c661p-2,
    0x1.590457c72dfe0p+2, -0x1.fffa8dcfe993bp-2, 0x1.59d14336bb49dp+2, -0x1.fffab0415df45p-2,
    0x1.5a9e2eb3e5ff5p+2, -0x1.fffad1d8fdfd2p-2, 0x1.5b6b1a3e5803ap+2, -0x1.fffaf29c2b3f8p-2,
    0x1.5c3805d5bd5c7p+2, -0x1.fffb12902545bp-2, 0x1.5d04f179c4227p+2, -0x1.fffb31ba0a69ep-2,
    0x1.5dd1dd2a1c748p+2, -0x1.fffb501ed8a81p-2, 0x1.5e9ec8e6786a6p+2, -0x1.fffb6dc36e6aep-2,
    0x1.5f6bb4ae8c08bp+2, -0x1.fffb8aac8b52ep-2, 0x1.6038a0820d34ap+2, -0x1.fffba6ded0f96p-2,
    0x1.61058c60b3a7ep+2, -0x1.fffbc25ec3ae4p-2, 0x1.61d2784a38e55p+2, -0x1.fffbdd30cb316p-2,
    0x1.629f643e582d8p+2, -0x1.fffbf7593366cp-2, 0x1.636c503cce73ep+2, -0x1.fffc10dc2d071p-2,
    0x1.64393c455a53ep+2, -0x1.fffc29bdce4b4p-2, 0x1.65062857bc066p+2, -0x1.fffc420213944p-2,
    0x1.65d31473b557ep+2, -0x1.fffc59ace00e3p-2, 0x1.66a00099099dep+2, -0x1.fffc70c1fe4fep-2,
    0x1.676cecc77dadep+2, -0x1.fffc874520f64p-2, 0x1.6839d8fed7d35p+2, -0x1.fffc9d39e33c1p-2,
    0x1.6906c53edfc6cp+2, -0x1.fffcb2a3c98d8p-2, 0x1.69d3b1875ea49p+2, -0x1.fffcc7864218ap-2,
    0x1.6aa09dd81ee44p+2, -0x1.fffcdbe4a55a0p-2, 0x1.6b6d8a30ec4ffp+2, -0x1.fffcefc236a5bp-2,
    0x1.6c3a769193fbfp+2, -0x1.fffd032224ad4p-2, 0x1.6d0762f9e43e9p+2, -0x1.fffd16078a023p-2,
    0x1.6dd44f69aca83p+2, -0x1.fffd28756d94fp-2, 0x1.6ea13be0bdfb9p+2, -0x1.fffd3a6ec3318p-2,
    0x1.6f6e285eea263p+2, -0x1.fffd4bf66bf7fp-2, 0x1.703b14e40438dp+2, -0x1.fffd5d0f36d2fp-2,
    0x1.7108016fe060ap+2, -0x1.fffd6dbbe0ea8p-2, 0x1.71d4ee0253dfcp+2, -0x1.fffd7dff1614ap-2,
    0x1.72a1da9b3506bp+2, -0x1.fffd8ddb7142ap-2, 0x1.736ec73a5b2dap+2, -0x1.fffd9d537cec1p-2,
    0x1.743bb3df9eadbp+2, -0x1.fffdac69b376cp-2, 0x1.7508a08ad8db1p+2, -0x1.fffdbb207f9cap-2,
    0x1.75d58d3be3fe4p+2, -0x1.fffdc97a3ccebp-2, 0x1.76a279f29b4e6p+2, -0x1.fffdd7793795bp-2,
    0x1.776f66aedaeb5p+2, -0x1.fffde51fadf07p-2, 0x1.783c53707fd79p+2, -0x1.fffdf26fcfaf9p-2,
    0x1.7909403767f34p+2, -0x1.fffdff6bbecf9p-2, 0x1.79d62d0371f60p+2, -0x1.fffe0c158fcfdp-2,
    0x1.7aa319d47d6a2p+2, -0x1.fffe186f4a083p-2, 0x1.7b7006aa6aa74p+2, -0x1.fffe247ae7fc3p-2,
    0x1.7c3cf3851acd0p+2, -0x1.fffe303a57abdp-2, 0x1.7d09e0646fbe8p+2, -0x1.fffe3baf7ae33p-2,
    0x1.7dd6cd484c1d3p+2, -0x1.fffe46dc27872p-2, 0x1.7ea3ba3093445p+2, -0x1.fffe51c227e10p-2,
    0x1.7f70a71d29445p+2, -0x1.fffe5c633ae7bp-2, 0x1.803d940df2de2p+2, -0x1.fffe66c114878p-2,
    0x1.810a8102d57f4p+2, -0x1.fffe70dd5de7bp-2, 0x1.81d76dfbb73d0p+2, -0x1.fffe7ab9b5aeep-2,
    0x1.82a45af87ed0cp+2, -0x1.fffe8457b0454p-2, 0x1.837147f91393cp+2, -0x1.fffe8db8d8158p-2,
    0x1.843e34fd5d7b1p+2, -0x1.fffe96deadcbbp-2, 0x1.850b22054513dp+2, -0x1.fffe9fcaa8936p-2,
    0x1.85d80f10b37f8p+2, -0x1.fffea87e36534p-2, 0x1.86a4fc1f92702p+2, -0x1.fffeb0fabbe81p-2,
    0x1.8771e931cc24fp+2, -0x1.fffeb941955d8p-2, 0x1.883ed6474b66bp+2, -0x1.fffec15416264p-2,
    0x1.890bc35ffb843p+2, -0x1.fffec93389522p-2, 0x1.89d8b07bc84f4p+2, -0x1.fffed0e131c34p-2,
    0x1.8aa59d9a9e194p+2, -0x1.fffed85e4a61ap-2, 0x1.8b728abc69b02p+2, -0x1.fffedfac064dep-2,
    0x1.8c3f77e1185b2p+2, -0x1.fffee6cb91120p-2, 0x1.8d0c650897d7fp+2, -0x1.fffeedbe0ed1dp-2,
    0x1.8dd95232d657cp+2, -0x1.fffef4849c797p-2, 0x1.8ea63f5fc27c5p+2, -0x1.fffefb204feb1p-2,
    0x1.8f732c8f4b555p+2, -0x1.ffff0192382b6p-2, 0x1.904019c1605d7p+2, -0x1.ffff07db5d8d3p-2,
    0x1.910d06f5f1781p+2, -0x1.ffff0dfcc1db8p-2, 0x1.91d9f42ceeee3p+2, -0x1.ffff13f76082fp-2,
    0x1.92a6e166496c8p+2, -0x1.ffff19cc2eba2p-2, 0x1.9373cea1f2005p+2, -0x1.ffff1f7c1ba8cp-2,
    0x1.9440bbdfda15bp+2, -0x1.ffff2508108e1p-2, 0x1.950da91ff374ep+2, -0x1.ffff2a70f0e62p-2,
    0x1.95da9662303ffp+2, -0x1.ffff2fb79a8e5p-2, 0x1.96a783a682f0bp+2, -0x1.ffff34dce5e8dp-2,
    0x1.977470ecde568p+2, -0x1.ffff39e1a5ff6p-2, 0x1.98415e3535942p+2, -0x1.ffff3ec6a8a50p-2,
    0x1.990e4b7f7c1dcp+2, -0x1.ffff438cb6970p-2, 0x1.99db38cba5b6dp+2, -0x1.ffff4834939d1p-2,
    0x1.9aa82619a6702p+2, -0x1.ffff4cbefea8cp-2, 0x1.9b75136972a62p+2, -0x1.ffff512cb1f40p-2,
    0x1.9c4200bafefecp+2, -0x1.ffff557e631f0p-2, 0x1.9d0eee0e4067cp+2, -0x1.ffff59b4c34d3p-2,
    0x1.9ddbdb632c14ep+2, -0x1.ffff5dd07f41cp-2, 0x1.9ea8c8b9b77e3p+2, -0x1.ffff61d23f7b4p-2,
    0x1.9f75b611d85e6p+2, -0x1.ffff65baa84e8p-2, 0x1.a042a36b84b12p+2, -0x1.ffff698a5a014p-2,
    0x1.a10f90c6b2b15p+2, -0x1.ffff6d41f0e37p-2, 0x1.a1dc7e2358d7cp+2, -0x1.ffff70e205686p-2,
    0x1.a2a96b816dd97p+2, -0x1.ffff746b2c3f6p-2, 0x1.a37658e0e8a64p+2, -0x1.ffff77ddf66b4p-2,
    0x1.a4434641c0673p+2, -0x1.ffff7b3af159cp-2, 0x1.a51033a3ec7d7p+2, -0x1.ffff7e82a6fa3p-2,
    0x1.a5dd210764806p+2, -0x1.ffff81b59dd37p-2, 0x1.a6aa0e6c203cep+2, -0x1.ffff84d45919bp-2,
    0x1.a776fbd217b37p+2, -0x1.ffff87df58c34p-2, 0x1.a843e93943175p+2, -0x1.ffff8ad7199d1p-2,
    0x1.a910d6a19accep+2, -0x1.ffff8dbc155efp-2, 0x1.a9ddc40b1768ep+2, -0x1.ffff908ec2bedp-2,
    0x1.aaaab175b1aedp+2, -0x1.ffff934f9583cp-2, 0x1.ab779ee1628ffp+2, -0x1.ffff95fefe98bp-2,
    0x1.ac448c4e232a4p+2, -0x1.ffff989d6c1e7p-2, 0x1.ad1179bbecc73p+2, -0x1.ffff9b2b497d4p-2,
    0x1.adde672ab8dacp+2, -0x1.ffff9da8ff760p-2, 0x1.aeab549a81023p+2, -0x1.ffffa016f4333p-2,
    0x1.af78420b3f034p+2, -0x1.ffffa2758b592p-2, 0x1.b0452f7ceccb1p+2, -0x1.ffffa4c52615fp-2,
    0x1.b1121cef846d2p+2, -0x1.ffffa70623312p-2, 0x1.b1df0a6300228p+2, -0x1.ffffa938df1acp-2,
    0x1.b2abf7d75a48ap+2, -0x1.ffffab5db3fa3p-2, 0x1.b378e54c8d60bp+2, -0x1.ffffad74f9bcdp-2,
    0x1.b445d2c2940e9p+2, -0x1.ffffaf7f0623cp-2, 0x1.b512c03969183p+2, -0x1.ffffb17c2cd1ep-2,
    0x1.b5dfadb107646p+2, -0x1.ffffb36cbf58fp-2, 0x1.b6ac9b2969fa3p+2, -0x1.ffffb5510d470p-2,
    0x1.b77988a28c004p+2, -0x1.ffffb7296432ep-2, 0x1.b846761c68bbdp+2, -0x1.ffffb8f60fc8ap-2,
    0x1.b9136396fb901p+2, -0x1.ffffbab759d5ep-2, 0x1.b9e051123ffd3p+2, -0x1.ffffbc6d8a555p-2,
    0x1.baad3e8e31a02p+2, -0x1.ffffbe18e77a7p-2, 0x1.bb7a2c0acc314p+2, -0x1.ffffbfb9b5bcep-2,
    0x1.bc4719880b844p+2, -0x1.ffffc15037e31p-2, 0x1.bd140705eb871p+2, -0x1.ffffc2dcaf0d4p-2,
    0x1.bde0f48468417p+2, -0x1.ffffc45f5abfbp-2, 0x1.beade2037dd43p+2, -0x1.ffffc5d878ed0p-2,
    0x1.bf7acf832878bp+2, -0x1.ffffc74845fffp-2, 0x1.c047bd0364801p+2, -0x1.ffffc8aefce54p-2,
    0x1.c114aa842e52ep+2, -0x1.ffffca0cd714fp-2, 0x1.c1e1980582705p+2, -0x1.ffffcb620c9b8p-2,
    0x1.c2ae85875d6dcp+2, -0x1.ffffccaed4232p-2, 0x1.c37b7309bbf62p+2, -0x1.ffffcdf362fc1p-2,
    0x1.c448608c9ac99p+2, -0x1.ffffcf2fed258p-2, 0x1.c5154e0ff6bc9p+2, -0x1.ffffd064a555dp-2,
    0x1.c5e23b93ccb7ep+2, -0x1.ffffd191bd027p-2, 0x1.c6af291819b7ap+2, -0x1.ffffd2b764685p-2,
    0x1.c77c169cdacb2p+2, -0x1.ffffd3d5ca930p-2, 0x1.c84904220d144p+2, -0x1.ffffd4ed1d64bp-2,
    0x1.c915f1a7adc6fp+2, -0x1.ffffd5fd899d5p-2, 0x1.c9e2df2dba28fp+2, -0x1.ffffd7073ae1ep-2,
    0x1.caafccb42f913p+2, -0x1.ffffd80a5bc34p-2, 0x1.cb7cba3b0b677p+2, -0x1.ffffd90715c52p-2,
    0x1.cc49a7c24b23dp+2, -0x1.ffffd9fd9164bp-2, 0x1.cd169549ec4e9p+2, -0x1.ffffdaedf61eep-2,
    0x1.cde382d1ec7f8p+2, -0x1.ffffdbd86a772p-2, 0x1.ceb0705a495d9p+2, -0x1.ffffdcbd13fd2p-2,
    0x1.cf7d5de3009ebp+2, -0x1.ffffdd9c17531p-2, 0x1.d04a4b6c10073p+2, -0x1.ffffde7598337p-2,
    0x1.d11738f575698p+2, -0x1.ffffdf49b976dp-2, 0x1.d1e4267f2ea5ep+2, -0x1.ffffe0189d194p-2,
    0x1.d2b1140939aa0p+2, -0x1.ffffe0e264400p-2, 0x1.d37e01939470bp+2, -0x1.ffffe1a72f3eap-2,
    0x1.d44aef1e3d017p+2, -0x1.ffffe2671d9c4p-2, 0x1.d517dca931705p+2, -0x1.ffffe3224e189p-2,
    0x1.d5e4ca346fdd7p+2, -0x1.ffffe3d8deb0ep-2, 0x1.d6b1b7bff674dp+2, -0x1.ffffe48aeca4cp-2,
    0x1.d77ea54bc36e2p+2, -0x1.ffffe538947adp-2, 0x1.d84b92d7d50c2p+2, -0x1.ffffe5e1f2053p-2,
    0x1.d9188064299ccp+2, -0x1.ffffe68720662p-2, 0x1.d9e56df0bf78ap+2, -0x1.ffffe7283a145p-2,
    0x1.dab25b7d9502ap+2, -0x1.ffffe7c558deep-2, 0x1.db7f490aa8a83p+2, -0x1.ffffe85e95f20p-2,
    0x1.dc4c3697f8e07p+2, -0x1.ffffe8f409da6p-2, 0x1.dd192425842c3p+2, -0x1.ffffe985cc89ap-2,
    0x1.dde611b34915fp+2, -0x1.ffffea13f559dp-2, 0x1.deb2ff4146314p+2, -0x1.ffffea9e9b116p-2,
    0x1.df7feccf7a1abp+2, -0x1.ffffeb25d3e6cp-2, 0x1.e04cda5de377bp+2, -0x1.ffffeba9b583dp-2,
    0x1.e119c7ec80f62p+2, -0x1.ffffec2a55096p-2, 0x1.e1e6b57b514c5p+2, -0x1.ffffeca7c712dp-2,
    0x1.e2b3a30a5338cp+2, -0x1.ffffed221fb91p-2, 0x1.e38090998581cp+2, -0x1.ffffed997295ep-2,
    0x1.e44d7e28e6f58p+2, -0x1.ffffee0dd2c72p-2, 0x1.e51a6bb87669bp+2, -0x1.ffffee7f52f1cp-2,
    0x1.e5e7594832bb5p+2, -0x1.ffffeeee0544ep-2, 0x1.e6b446d81acebp+2, -0x1.ffffef59fb7c7p-2,
    0x1.e78134682d8f1p+2, -0x1.ffffefc346e46p-2, 0x1.e84e21f869ee8p+2, -0x1.fffff029f85b3p-2,
    0x1.e91b0f88cee5cp+2, -0x1.fffff08e20549p-2, 0x1.e9e7fd195b742p+2, -0x1.fffff0efcedc5p-2,
    0x1.eab4eaaa0e9f4p+2, -0x1.fffff14f1398bp-2, 0x1.eb81d83ae772dp+2, -0x1.fffff1abfdccfp-2,
    0x1.ec4ec5cbe500dp+2, -0x1.fffff2069c5bep-2, 0x1.ed1bb35d0660cp+2, -0x1.fffff25efdca0p-2,
    0x1.ede8a0ee4ab04p+2, -0x1.fffff2b530403p-2, 0x1.eeb58e7fb1125p+2, -0x1.fffff309418dap-2,
    0x1.ef827c1138af7p+2, -0x1.fffff35b3f2a3p-2, 0x1.f04f69a2e0b57p+2, -0x1.fffff3ab3638ap-2,
    0x1.f11c5734a8575p+2, -0x1.fffff3f933889p-2, 0x1.f1e944c68ecd3p+2, -0x1.fffff4454398ap-2,
    0x1.f2b6325893542p+2, -0x1.fffff48f72986p-2, 0x1.f3831feab52dfp+2, -0x1.fffff4d7cc6a5p-2,
    0x1.f4500d7cf3a12p+2, -0x1.fffff51e5ca5dp-2, 0x1.f51cfb0f4df8dp+2, -0x1.fffff5632e98fp-2,
    0x1.f5e9e8a1c384ap+2, -0x1.fffff5a64d4a3p-2, 0x1.f6b6d63453989p+2, -0x1.fffff5e7c37a7p-2,
    0x1.f783c3c6fd8cbp+2, -0x1.fffff6279ba66p-2, 0x1.f850b159c0bd8p+2, -0x1.fffff665e008ap-2,
    0x1.f91d9eec9c8b4p+2, -0x1.fffff6a29a9adp-2, 0x1.f9ea8c7f905a6p+2, -0x1.fffff6ddd517cp-2,
    0x1.fab77a129b930p+2, -0x1.fffff71798fc9p-2, 0x1.fb8467a5bda11p+2, -0x1.fffff74fef8a6p-2,
    0x1.fc515538f5f43p+2, -0x1.fffff786e1c7ep-2, 0x1.fd1e42cc43ff7p+2, -0x1.fffff7bc78827p-2,
    0x1.fdeb305fa7398p+2, -0x1.fffff7f0bc501p-2, 0x1.feb81df31f1c7p+2, -0x1.fffff823b5904p-2,
    0x1.ff850b86ab258p+2, -0x1.fffff8556c6dap-2, 0x1.0028fc8d256abp+3, -0x1.fffff885e8df1p-2,
    0x1.008f7356fed7dp+3, -0x1.fffff8b532a94p-2, 0x1.00f5ea20e19dap+3, -0x1.fffff8e3515f9p-2,
    0x1.015c60eacd80ep+3, -0x1.fffff9104c659p-2, 0x1.01c2d7b4c2480p+3, -0x1.fffff93c2af01p-2,
    0x1.02294e7ebfbadp+3, -0x1.fffff966f4064p-2, 0x1.028fc548c5a26p+3, -0x1.fffff990ae82fp-2,
    0x1.02f63c12d3c94p+3, -0x1.fffff9b961159p-2, 0x1.035cb2dce9fb5p+3, -0x1.fffff9e112434p-2,
    0x1.03c329a70805ap+3, -0x1.fffffa07c867ep-2, 0x1.0429a0712db6ap+3, -0x1.fffffa2d89b73p-2,
    0x1.0490173b5addep+3, -0x1.fffffa525c3d9p-2, 0x1.04f68e058f4c4p+3, -0x1.fffffa7645e15p-2,
    0x1.055d04cfcad3ap+3, -0x1.fffffa994c635p-2, 0x1.05c37b9a0d474p+3, -0x1.fffffabb75600p-2,
    0x1.0629f264567b3p+3, -0x1.fffffadcc6508p-2, 0x1.0690692ea644dp+3, -0x1.fffffafd448b2p-2,
    0x1.06f6dff8fc7a8p+3, -0x1.fffffb1cf5449p-2, 0x1.075d56c358f39p+3, -0x1.fffffb3bdd909p-2,
    0x1.07c3cd8dbb888p+3, -0x1.fffffb5a0262bp-2, 0x1.082a445824129p+3, -0x1.fffffb77688f5p-2,
    0x1.0890bb22926c2p+3, -0x1.fffffb9414cc3p-2, 0x1.08f731ed06707p+3, -0x1.fffffbb00bb13p-2,
    0x1.095da8b77ffbbp+3, -0x1.fffffbcb51b95p-2, 0x1.09c41f81feeaep+3, -0x1.fffffbe5eb432p-2,
    0x1.0a2a964c831bep+3, -0x1.fffffbffdc919p-2, 0x1.0a910d170c6d8p+3, -0x1.fffffc1929ccap-2,
    0x1.0af783e19abf5p+3, -0x1.fffffc31d7021p-2, 0x1.0b5dfaac2df1bp+3, -0x1.fffffc49e825dp-2,
    0x1.0bc47176c5e5cp+3, -0x1.fffffc6161132p-2, 0x1.0c2ae841627d6p+3, -0x1.fffffc78458c8p-2,
    0x1.0c915f0c039b6p+3, -0x1.fffffc8e993d0p-2, 0x1.0cf7d5d6a9230p+3, -0x1.fffffca45fb83p-2,
    0x1.0d5e4ca152f86p+3, -0x1.fffffcb99c7b4p-2, 0x1.0dc4c36c01005p+3, -0x1.fffffcce52ed2p-2,
    0x1.0e2b3a36b3203p+3, -0x1.fffffce2865f5p-2, 0x1.0e91b101693e3p+3, -0x1.fffffcf63a0e6p-2,
    0x1.0ef827cc23411p+3, -0x1.fffffd0971226p-2, 0x1.0f5e9e96e1102p+3, -0x1.fffffd1c2eaf4p-2,
    0x1.0fc51561a2936p+3, -0x1.fffffd2e75b5cp-2, 0x1.102b8c2c67b37p+3, -0x1.fffffd4049238p-2,
    0x1.109202f730597p+3, -0x1.fffffd51abd38p-2, 0x1.10f879c1fc6f1p+3, -0x1.fffffd62a08edp-2,
    0x1.115ef08ccbde9p+3, -0x1.fffffd732a0cep-2, 0x1.11c567579e92dp+3, -0x1.fffffd834af40p-2,
    0x1.122bde2274772p+3, -0x1.fffffd9305d99p-2, 0x1.129254ed4d775p+3, -0x1.fffffda25d42cp-2,
    0x1.12f8cbb8297fcp+3, -0x1.fffffdb153a4dp-2, 0x1.135f4283087d3p+3, -0x1.fffffdbfeb655p-2,
    0x1.13c5b94dea5d0p+3, -0x1.fffffdce26dadp-2, 0x1.142c3018cf0cep+3, -0x1.fffffddc084d1p-2,
    0x1.1492a6e3b67b2p+3, -0x1.fffffde991f54p-2, 0x1.14f91daea0965p+3, -0x1.fffffdf6c5febp-2,
    0x1.155f94798d4d8p+3, -0x1.fffffe03a686ep-2, 0x1.15c60b447c904p+3, -0x1.fffffe10359dep-2,
    0x1.162c820f6e4e8p+3, -0x1.fffffe1c7546ep-2, 0x1.1692f8da62787p+3, -0x1.fffffe2867783p-2,
    0x1.16f96fa558fecp+3, -0x1.fffffe340e1bcp-2, 0x1.175fe67051d2ap+3, -0x1.fffffe3f6b0f6p-2,
    0x1.17c65d3b4ce57p+3, -0x1.fffffe4a80253p-2, 0x1.182cd4064a28fp+3, -0x1.fffffe554f23bp-2,
    0x1.18934ad1498f6p+3, -0x1.fffffe5fd9c62p-2, 0x1.18f9c19c4b0b2p+3, -0x1.fffffe6a21bcep-2,
    0x1.196038674e8f1p+3, -0x1.fffffe7428ad9p-2, 0x1.19c6af32540e6p+3, -0x1.fffffe7df0338p-2,
    0x1.1a2d25fd5b7c7p+3, -0x1.fffffe8779dfcp-2, 0x1.1a939cc864cd2p+3, -0x1.fffffe90c7398p-2,
    0x1.1afa13936ff48p+3, -0x1.fffffe99d9be3p-2, 0x1.1b608a5e7ce6dp+3, -0x1.fffffea2b2e1fp-2,
    0x1.1bc701298b98ep+3, -0x1.fffffeab540fcp-2, 0x1.1c2d77f49bff9p+3, -0x1.fffffeb3bea96p-2,
    0x1.1c93eebfae101p+3, -0x1.fffffebbf4082p-2, 0x1.1cfa658ac1bfep+3, -0x1.fffffec3f57cap-2,
    0x1.1d60dc55d704dp+3, -0x1.fffffecbc44f4p-2, 0x1.1dc75320edd4cp+3, -0x1.fffffed361c02p-2,
    0x1.1e2dc9ec06260p+3, -0x1.fffffedacf07bp-2, 0x1.1e9440b71fef0p+3, -0x1.fffffee20d567p-2,
    0x1.1efab7823b268p+3, -0x1.fffffee91dd58p-2, 0x1.1f612e4d57c37p+3, -0x1.fffffef001a6ap-2,
    0x1.1fc7a51875bd0p+3, -0x1.fffffef6b9e46p-2, 0x1.202e1be3950a9p+3, -0x1.fffffefd47a25p-2,
    0x1.209492aeb5a3bp+3, -0x1.ffffff03abed5p-2, 0x1.20fb0979d7803p+3, -0x1.ffffff09e7cb7p-2,
    0x1.21618044fa982p+3, -0x1.ffffff0ffc3c7p-2, 0x1.21c7f7101ee3cp+3, -0x1.ffffff15ea399p-2,
    0x1.222e6ddb445b5p+3, -0x1.ffffff1bb2b61p-2, 0x1.2294e4a66af78p+3, -0x1.ffffff21569f3p-2,
    0x1.22fb5b7192b11p+3, -0x1.ffffff26d6dc2p-2, 0x1.2361d23cbb810p+3, -0x1.ffffff2c344eap-2,
    0x1.23c84907e5605p+3, -0x1.ffffff316fd2bp-2, 0x1.242ebfd310487p+3, -0x1.ffffff368a3eep-2,
    0x1.2495369e3c32cp+3, -0x1.ffffff3b84647p-2, 0x1.24fbad696918ep+3, -0x1.ffffff405f0fbp-2,
    0x1.2562243496f49p+3, -0x1.ffffff451b078p-2, 0x1.25c89affc5bfep+3, -0x1.ffffff49b90e3p-2,
    0x1.262f11caf574cp+3, -0x1.ffffff4e39e11p-2, 0x1.26958896260d8p+3, -0x1.ffffff529e38dp-2,
    0x1.26fbff6157847p+3, -0x1.ffffff56e6c9ap-2, 0x1.2762762c89d42p+3, -0x1.ffffff5b14432p-2,
    0x1.27c8ecf7bcf73p+3, -0x1.ffffff5f2750ap-2, 0x1.282f63c2f0e86p+3, -0x1.ffffff6320995p-2,
    0x1.2895da8e25a2ap+3, -0x1.ffffff6700c01p-2, 0x1.28fc51595b210p+3, -0x1.ffffff6ac863fp-2,
    0x1.2962c824915e9p+3, -0x1.ffffff6e781fep-2, 0x1.29c93eefc856bp+3, -0x1.ffffff72108b2p-2,
    0x1.2a2fb5bb0004cp+3, -0x1.ffffff7592392p-2, 0x1.2a962c8638643p+3, -0x1.ffffff78fdb9bp-2,
    0x1.2afca3517170bp+3, -0x1.ffffff7c53992p-2, 0x1.2b631a1cab25fp+3, -0x1.ffffff7f94602p-2,
    0x1.2bc990e7e57fdp+3, -0x1.ffffff82c0943p-2, 0x1.2c3007b3207a3p+3, -0x1.ffffff85d8b76p-2,
    0x1.2c967e7e5c112p+3, -0x1.ffffff88dd48bp-2, 0x1.2cfcf5499840cp+3, -0x1.ffffff8bcec3ep-2,
    0x1.2d636c14d5055p+3, -0x1.ffffff8eada19p-2, 0x1.2dc9e2e0125b2p+3, -0x1.ffffff917a579p-2,
    0x1.2e3059ab503e9p+3, -0x1.ffffff943558bp-2, 0x1.2e96d0768eac2p+3, -0x1.ffffff96df14ep-2,
    0x1.2efd4741cda08p+3, -0x1.ffffff9977f97p-2, 0x1.2f63be0d0d184p+3, -0x1.ffffff9c0070dp-2,
    0x1.2fca34d84d102p+3, -0x1.ffffff9e78e2ep-2, 0x1.3030aba38d851p+3, -0x1.ffffffa0e1b51p-2,
    0x1.3097226ece73ep+3, -0x1.ffffffa33b4a1p-2, 0x1.30fd993a0fd99p+3, -0x1.ffffffa586026p-2,
    0x1.3164100551b34p+3, -0x1.ffffffa7c23bfp-2, 0x1.31ca86d093fe1p+3, -0x1.ffffffa9f0526p-2,
    0x1.3230fd9bd6b72p+3, -0x1.ffffffac109f3p-2, 0x1.3297746719dbcp+3, -0x1.ffffffae23799p-2,
    0x1.32fdeb325d695p+3, -0x1.ffffffb029368p-2, 0x1.336461fda15d4p+3, -0x1.ffffffb22228fp-2,
    0x1.33cad8c8e5b4fp+3, -0x1.ffffffb40ea1dp-2, 0x1.34314f942a6e0p+3, -0x1.ffffffb5eef01p-2,
    0x1.3497c65f6f85fp+3, -0x1.ffffffb7c3609p-2, 0x1.34fe3d2ab4fa8p+3, -0x1.ffffffb98c3e6p-2,
    0x1.3564b3f5fac95p+3, -0x1.ffffffbb49d2bp-2, 0x1.35cb2ac140f04p+3, -0x1.ffffffbcfc64fp-2,
    0x1.3631a18c876d0p+3, -0x1.ffffffbea43abp-2, 0x1.36981857ce3d9p+3, -0x1.ffffffc04197ep-2,
    0x1.36fe8f23155fep+3, -0x1.ffffffc1d4becp-2, 0x1.376505ee5cd1dp+3, -0x1.ffffffc35defdp-2,
    0x1.37cb7cb9a4917p+3, -0x1.ffffffc4dd6a2p-2, 0x1.3831f384ec9cep+3, -0x1.ffffffc6536b2p-2,
    0x1.38986a5034f24p+3, -0x1.ffffffc7c02ebp-2, 0x1.38fee11b7d8fcp+3, -0x1.ffffffc923ef4p-2,
    0x1.396557e6c6738p+3, -0x1.ffffffca7ee5ep-2, 0x1.39cbceb20f9bdp+3, -0x1.ffffffcbd14a2p-2,
    0x1.3a32457d59071p+3, -0x1.ffffffcd1b523p-2, 0x1.3a98bc48a2b38p+3, -0x1.ffffffce5d32fp-2,
    0x1.3aff3313ec9f9p+3, -0x1.ffffffcf971ffp-2, 0x1.3b65a9df36c9bp+3, -0x1.ffffffd0c94b8p-2,
    0x1.3bcc20aa81305p+3, -0x1.ffffffd1f3e6ap-2, 0x1.3c329775cbd20p+3, -0x1.ffffffd317214p-2,
    0x1.3c990e4116ad3p+3, -0x1.ffffffd4332a0p-2, 0x1.3cff850c61c08p+3, -0x1.ffffffd5482e5p-2,
    0x1.3d65fbd7ad0aap+3, -0x1.ffffffd6565aap-2, 0x1.3dcc72a2f88a2p+3, -0x1.ffffffd75dda3p-2,
    0x1.3e32e96e443dbp+3, -0x1.ffffffd85ed74p-2, 0x1.3e99603990241p+3, -0x1.ffffffd9597b0p-2,
    0x1.3effd704dc3bfp+3, -0x1.ffffffda4ded9p-2, 0x1.3f664dd028842p+3, -0x1.ffffffdb3c561p-2,
    0x1.3fccc49b74fb8p+3, -0x1.ffffffdc24dacp-2, 0x1.40333b65a9dddp+3, -0x1.0000000000000p-1,
};
constexpr int kExpTabN = 256;                 // 2^(j/256)
constexpr int kFp64TabDoubles = kExpTabN + 514;

// Rounding to an integer by adding 1.5 * 2^52: one FMA rounds a x + magic (|a x| < 2^51) to
// the nearest integer n held in the low mantissa bits, so n as a double is (t - magic) and n
// as an int is the low 32 bits of t (two's complement) — no v_rndne / v_cvt.
constexpr double kRoundMagic = 0x1.8p52;
__device__ __forceinline__ int round_magic_lo(double t) {
    return (int)__builtin_bit_cast(long long, t);
}
__device__ __forceinline__ double exp_tab_nonpos(double y, const double* __restrict__ et) {
    y = y > -745.0 ? y : -745.0;
    const double tk = __builtin_fma(y, 369.32993046757462, kRoundMagic);   // 256 / ln2
    const double kd = tk - kRoundMagic;                                // exact
    double r = __builtin_fma(-kd, 6.93147180369123816490e-01 / 256, y);   // kd * hi exact
    r = __builtin_fma(-kd, 1.90821492927058770002e-10 / 256, r);
    double p = __builtin_fma(r, 1.0 / 24, 1.0 / 6);
    p = __builtin_fma(p, r, 0.5);
    p = __builtin_fma(p, r, 1.0);
    p = __builtin_fma(p, r, 1.0);
    const int k = round_magic_lo(tk);
    return __builtin_ldexp(et[k & (kExpTabN - 1)] * p, k >> 8);
}
__device__ __forceinline__ double log1p_tab_unit(double u, const double* __restrict__ lt) {
    const double m = 1.0 + u;
    const double c = u - (m - 1.0);                                    // exact
    const int j = round_magic_lo(__builtin_fma(m - 1.0, 256.0, kRoundMagic));   // rint: 0..256
    const double rj = lt[2 * j], lj = lt[2 * j + 1];
    const double t = __builtin_fma(c, rj, __builtin_fma(m, rj, -1.0));
    double q = __builtin_fma(t, 1.0 / 7, -1.0 / 6);
    q = __builtin_fma(q, t, 1.0 / 5);
    q = __builtin_fma(q, t, -1.0 / 4);
    q = __builtin_fma(q, t, 1.0 / 3);
    q = __builtin_fma(q, t, -0.5);
    return lj + __builtin_fma(q * t, t, t);
}
// torch.nn.Softplus (threshold 20) = x > 20 ? x : max(x, 0) + log1p(e^-|x|)
__device__ __forceinline__ double softplus_tab(double x, const double* __restrict__ tab) {
    const double r = log1p_tab_unit(exp_tab_nonpos(-__builtin_fabs(x), tab), tab + kExpTabN);
    const double y = __builtin_fmax(x, 0.0) + r;
    return x > 20.0 ? x : y;
}

// The fp64 decoder_v2_4 MLP form: the same tables at the accuracy the fp64 parity contract
// needs (outputs within rtol 1e-10 of the reference; every Softplus here within 1e-13
// ABSOLUTE of glibc over the decoders' range, tests/test_fastmath_cpu.py) instead of <= 3 ulp:
//   exp:   one-part ln2/256 reduction (kd * ulp(ln2/256) <= 2e-16 relative for |y| <= 40;
//          below that e^y < 5e-18 absolute), degree-3 Taylor (r^4/24 <= 1.4e-13 relative);
//   log1p: m = 1 + u rounded (the dropped rounding error c is <= 1.1e-16 absolute), degree-4
//          series of log1p(t), |t| <= 2^-9 (t^5/5 <= 6e-15 absolute).
// 29 VALU (21 of them fp64) + 2 LDS reads per unit instead of ~37 + 2 (the table pair r_j, l_j
// is one 16-byte read).
// a * s + v as ONE VOP3 v_fma_f64 with s in an SGPR pair and v in a (loop-invariant) VGPR pair:
// gfx9 VOP3 takes no literal and one scalar operand, so hipcc otherwise copies a non-inline
// constant addend into the accumulator of a v_fmac_f64 before every use (two v_mov_b32)
__device__ __forceinline__ double fma_vsv(double a, double s, double v) {
#if defined(__HIP_DEVICE_COMPILE__)
    double d;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(a), "s"(s), "v"(v));
    return d;
#else
    return __builtin_fma(a, s, v);       // host build of this header (tests/test_fastmath_cpu.py)
#endif
}
// e^-|x| for |x| < 2^51 / 369 (no clamp: below -745 the ldexp underflows to 0 exactly); the
// -|x| is a source modifier of both reduction FMAs
__device__ __forceinline__ double exp_tab_negabs_lite(double x, const double* __restrict__ et) {
#if defined(__HIP_DEVICE_COMPILE__)
    double tk;
    asm("v_fma_f64 %0, -|%1|, %2, %3" : "=v"(tk) : "v"(x), "s"(369.32993046757462), "v"(kRoundMagic));
#else
    const double tk = __builtin_fma(-__builtin_fabs(x), 369.32993046757462, kRoundMagic);
#endif
    const double kd = tk - kRoundMagic;                                // exact
    const double r = __builtin_fma(-kd, 6.93147180559945309417e-01 / 256, -__builtin_fabs(x));
    double p = fma_vsv(r, 1.0 / 6, 0.5);                              // degree 3: r^4/24 <= 1.4e-13
    p = __builtin_fma(p, r, 1.0);
    p = __builtin_fma(p, r, 1.0);
    const int k = round_magic_lo(tk);
    return __builtin_ldexp(et[k & (kExpTabN - 1)] * p, k >> 8);
}
__device__ __forceinline__ double log1p_tab_unit_lite(double u, const double* __restrict__ lt) {
    const double m = 1.0 + u;
    const int j = round_magic_lo(fma_vsv(u, 256.0, kRoundMagic));      // rint(256 u): 0..256
    const double rj = lt[2 * j], lj = lt[2 * j + 1];
    const double t = __builtin_fma(m, rj, -1.0);
    double q = fma_vsv(t, -0.25, 1.0 / 3);
    q = __builtin_fma(q, t, -0.5);
    return lj + __builtin_fma(q * t, t, t);
}
// max(x, 0) as one v_max_f64 (fmax would canonicalise x first: NaN quieting, one more op)
__device__ __forceinline__ double relu_f64(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    double d;
    asm("v_max_f64 %0, %1, 0" : "=v"(d) : "v"(x));
    return d;
#else
    return x > 0.0 ? x : 0.0;
#endif
}
__device__ __forceinline__ double softplus_tab_lite(double x, const double* __restrict__ tab) {
    const double r = log1p_tab_unit_lite(exp_tab_negabs_lite(x, tab), tab + kExpTabN);
    const double v = relu_f64(x) + r;
    return x > 20.0 ? x : v;
}

// softplus_tab_lite's values with one VALU op less per call (the fp64 decoder_v2_4 forward):
// torch's threshold (x > 20 -> x) moves into the exponent of e^-|x|: 2^-2048 flushes it to 0,
// log1p(0) = l_0 + 0 = 0 exactly, and relu(x) + 0 = x — the same bits as selecting x, one
// v_cndmask on the 32-bit exponent instead of two on the result halves.
__device__ __forceinline__ double softplus_fast(double x, const double* __restrict__ tab) {
#if defined(__HIP_DEVICE_COMPILE__)
    double tk;
    asm("v_fma_f64 %0, -|%1|, %2, %3" : "=v"(tk) : "v"(x), "s"(369.32993046757462), "v"(kRoundMagic));
#else
    const double tk = __builtin_fma(-__builtin_fabs(x), 369.32993046757462, kRoundMagic);
#endif
    const double kd = tk - kRoundMagic;                                // exact
    const double r = __builtin_fma(-kd, 6.93147180559945309417e-01 / 256, -__builtin_fabs(x));
    double p = fma_vsv(r, 1.0 / 6, 0.5);
    p = __builtin_fma(p, r, 1.0);
    p = __builtin_fma(p, r, 1.0);
    const int k = round_magic_lo(tk);
    const int e = x > 20.0 ? -2048 : (k >> 8);
    const double u = __builtin_ldexp(tab[k & (kExpTabN - 1)] * p, e);
    return relu_f64(x) + log1p_tab_unit_lite(u, tab + kExpTabN);
}

// e^-|x| with torch's Softplus threshold in the exponent: x > 20 -> exactly 0 (softplus_fast's
// first half; the fp64 reverse pass, gnnd_train.hip sp_and_grad)
__device__ __forceinline__ double exp_negabs_thr(double x, const double* __restrict__ tab) {
#if defined(__HIP_DEVICE_COMPILE__)
    double tk;
    asm("v_fma_f64 %0, -|%1|, %2, %3" : "=v"(tk) : "v"(x), "s"(369.32993046757462), "v"(kRoundMagic));
#else
    const double tk = __builtin_fma(-__builtin_fabs(x), 369.32993046757462, kRoundMagic);
#endif
    const double kd = tk - kRoundMagic;                                // exact
    const double r = __builtin_fma(-kd, 6.93147180559945309417e-01 / 256, -__builtin_fabs(x));
    double p = fma_vsv(r, 1.0 / 6, 0.5);
    p = __builtin_fma(p, r, 1.0);
    p = __builtin_fma(p, r, 1.0);
    const int k = round_magic_lo(tk);
    const int e = x > 20.0 ? -2048 : (k >> 8);
    return __builtin_ldexp(tab[k & (kExpTabN - 1)] * p, e);
}

// fp64 Softplus from ONE table read: a = |x| = a_j + r (a_j = j/64, |r| <= 1/128) and the
// degree-4 Taylor polynomial of f(a) = ln(1 + e^-a) about a_j, its coefficients from the
// tabulated f_j and s_j = 1/(1 + e^a_j) (derivatives: -s, t, -t(1 - 2s), t(1 - 6t) with
// t = s(1 - s)); remainder <= (1/128)^5/120 max|f^(5)| (|f^(5)| <= ~1/8): within 5e-14
// ABSOLUTE of glibc, measured 3.1e-14 near a = 0.85 (tests/test_fastmath_cpu.py; softplus_fast:
// 7e-14).  a >= 32 + 1/128 takes the zero entry (f < 1.3e-14), and
// so does x > 20 (torch's threshold: relu(x) + 0 = x exactly).  Valid for |x| < 2^51 / 64.
// 19 VALU and one 16-byte LDS read instead of softplus_fast's 25 and two reads.
constexpr int kSpTabN = 2050;
constexpr int kSpTabDoubles = 2 * kSpTabN;
struct SpIdx {
    double r;
    int j;
};
__device__ __forceinline__ SpIdx sp_index(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    double tk;
    asm("v_fma_f64 %0, |%1|, %2, %3" : "=v"(tk) : "v"(x), "s"(64.0), "v"(kRoundMagic));
#else
    const double tk = __builtin_fma(__builtin_fabs(x), 64.0, kRoundMagic);
#endif
    const double kd = tk - kRoundMagic;                                // exact
    SpIdx q;
    q.r = __builtin_fma(kd, -1.0 / 64, __builtin_fabs(x));             // exact
    const unsigned j = (unsigned)round_magic_lo(tk);
    q.j = x > 20.0 ? kSpTabN - 1 : (int)(j < (unsigned)(kSpTabN - 1) ? j : (unsigned)(kSpTabN - 1));
    return q;
}
// ln(1 + e^-a) from the entry {f0, s} at offset r (the Taylor polynomial above, Horner form
// f0 + r (-s + u (1/2 + r (B + r A))), u = t r, B = (2s - 1)/6, A = (1 - 6t)/24: 8 VALU, the
// r A term spread as r/24 - u/4 so no operand needs a register copy (A = 1/24 - t/4 as an
// accumulating FMA had the constant 1/24 copied into its destination first, one v_mov_b64)
__device__ __forceinline__ double sp_poly(double r, double f0, double s) {
    const double t = __builtin_fma(-s, s, s);
    const double u = t * r;
    const double b = __builtin_fma(s, 1.0 / 3, -1.0 / 6);
    double p = __builtin_fma(r, 1.0 / 24, b);
    p = __builtin_fma(u, -0.25, p);
    p = __builtin_fma(p, r, 0.5);
    return __builtin_fma(__builtin_fma(u, p, -s), r, f0);
}
// the table entry {f0, s} of index j as one 16-byte read (byte offset 16 j: one v_lshl_add)
struct SpEntry {
    double f0, s;
};
__device__ __forceinline__ SpEntry sp_entry(const double* __restrict__ st, int j) {
    return ((const SpEntry*)st)[j];
}
__device__ __forceinline__ double softplus_sp(double x, const double* __restrict__ st) {
    const SpIdx q = sp_index(x);
    const SpEntry e = sp_entry(st, q.j);
    return relu_f64(x) + sp_poly(q.r, e.f0, e.s);
}
// sigmoid(-a) = 1/(1 + e^a) about the same entry, degree 4 (the fp64 reverse pass's Softplus
// derivative, as accurate as the forward's softplus_sp: remainder r^5 s^(5) / 120 < 1e-13):
// with t = s (1 - s), s' = -t, s'' = t (1 - 2s), s''' = -t (1 - 6t), s'''' = t (1 - 2s)(1 - 12t),
// s - t r (1 + r (b2 + r (a2 + r c2))), b2 = s - 1/2, a2 = 1/6 - t, c2 = b2 (1/12 - t)
__device__ __forceinline__ double sig_poly(double r, double s) {
    const double t = __builtin_fma(-s, s, s);
    const double b2 = s - 0.5;
    const double c2 = b2 * (1.0 / 12 - t);
    const double p = __builtin_fma(__builtin_fma(__builtin_fma(c2, r, 1.0 / 6 - t), r, b2), r, 1.0);
    return __builtin_fma(-(t * r), p, s);
}
// the same polynomial centred: d = 1/2 - s(a_j + r) = (1/2 - s) + t r P, so that the sigmoid of
// the signed argument h is 1/2 + copysign(d, h) (one FMA, a sign copy and an add instead of
// 1 - s, a compare and a 64-bit select: the degree-4 term costs nothing)
__device__ __forceinline__ double sig_half_poly(double r, double s) {
    const double t = __builtin_fma(-s, s, s);
    const double b2 = s - 0.5;
    const double c2 = b2 * (1.0 / 12 - t);
    const double p = __builtin_fma(__builtin_fma(__builtin_fma(c2, r, 1.0 / 6 - t), r, b2), r, 1.0);
    return __builtin_fma(t * r, p, -b2);
}

// g(h) = softplus(h) - h/2 from ONE read of the signed table kSgTab: h = c_j + r, c_j = j kSgStep
// (j = round(h kSgScale) clamped to [kSgLo, kSgHi] by one v_med3_i32, r = h - c_j by one FMA
// after the int -> double conversion), and the degree-4 Taylor polynomial of g about c_j:
// g' = -sig, g'' = t = 1/4 - sig^2, g^(3) = 2 sig t, g^(4) = t (1 - 6t): sp_poly's Horner form
// with s - 1/2 -> sig.  No |h|, no threshold compare and select, and no separate |h|/2 term: the
// clamp entries are exactly linear (t = 0): j = kSgHi covers h > 20 (torch's threshold, Softplus =
// h: g = h/2; kSgScale puts 20 on the entry boundary, h = 20 itself takes entry 799), j = kSgLo
// h < -32.03 (g = -h/2, Softplus < 1.3e-14).  Step 1/39.975: remainder (step/2)^5/120 max|g^(5)|
// = 3.3e-13 ABSOLUTE (kSpTab's 1/64 step: 3.1e-14, but at 53 KB instead of 33 KB: one workgroup
// per CU fewer); tests/test_fastmath_cpu.py.  Valid for |h| < 2^31 / 40.  16 VALU per MLP unit
// in decode_kernel (layer 1, index, polynomial, layer 2) instead of 19 with kSpTab.
constexpr double kSgScale = 0x1.3fcccccccccccp+5;   // 39.974999999999994 (gen_fp64_tables.py)
constexpr double kSgStep = 1.0 / kSgScale;
constexpr int kSgLo = -1281, kSgHi = 800;
constexpr int kSgN = kSgHi - kSgLo + 1;
constexpr int kSgTabDoubles = 2 * kSgN;
__device__ __forceinline__ SpIdx sg_index(double x) {
    const double tk = __builtin_fma(x, kSgScale, kRoundMagic);
    int k = round_magic_lo(tk);
    k = k < kSgLo ? kSgLo : k;
    k = k > kSgHi ? kSgHi : k;
    SpIdx q;
    q.r = __builtin_fma((double)k, -kSgStep, x);
    q.j = k - kSgLo;
    return q;
}
// the same index for any finite h (sg_index's 32-bit index wraps for |h| >= 2^31 /
// 40): the index from h clamped to [-64, 64] (beyond it j is an end entry either way), r from
// h itself -- the end entries are exactly linear, so the value stays exact.  Identical to
// sg_index wherever that one is valid; the decoder takes it only for waves whose pre-activation
// bound reaches 2^25 (decode_kernel's MLP guard)
__device__ __forceinline__ SpIdx sg_index_safe(double x) {
    const double xi = __builtin_fmin(__builtin_fmax(x, -64.0), 64.0);
    const double tk = __builtin_fma(xi, kSgScale, kRoundMagic);
    int k = round_magic_lo(tk);
    k = k < kSgLo ? kSgLo : k;
    k = k > kSgHi ? kSgHi : k;
    SpIdx q;
    q.r = __builtin_fma((double)k, -kSgStep, x);
    q.j = k - kSgLo;
    return q;
}
// g(c + r) from the entry {f0 = g(c), sig = 1/2 - sigmoid(c)}: 8 VALU
__device__ __forceinline__ double sg_poly(double r, double f0, double sig) {
    const double t = __builtin_fma(-sig, sig, 0.25);
    const double u = t * r;
    const double b = sig * (1.0 / 3);
    double p = __builtin_fma(r, 1.0 / 24, b);
    p = __builtin_fma(u, -0.25, p);
    p = __builtin_fma(p, r, 0.5);
    return __builtin_fma(__builtin_fma(u, p, -sig), r, f0);
}
// g'(c + r) = sigmoid(c + r) - 1/2 about the same entry, degree 4 (the fp64 reverse pass's
// Softplus derivative): g^(5) = 2 sig t (1 - 12 t), so g' = -sig + t r (1 + r (sig + r ((1/6 - t)
// + r sig (1/12 - t)))) -- sig_half_poly with s - 1/2 -> sig; u = t r shared with sg_poly.  The
// clamp entries (t = 0) give exactly 1/2 (h > 20: torch's gradient 1) and -1/2 (h < -32.03)
__device__ __forceinline__ double sg_grad_poly(double r, double sig) {
    const double t = __builtin_fma(-sig, sig, 0.25);
    const double c2 = sig * (1.0 / 12 - t);
    const double p = __builtin_fma(__builtin_fma(__builtin_fma(c2, r, 1.0 / 6 - t), r, sig), r, 1.0);
    return __builtin_fma(t * r, p, -sig);
}
__device__ __forceinline__ double softplus_sg(double x, const double* __restrict__ tab) {
    const SpIdx q = sg_index(x);
    const SpEntry e = sp_entry(tab, q.j);
    return sg_poly(q.r, e.f0, e.s) + 0.5 * x;
}

// The fp64 decoder_v2_4 MLPs' Softplus table in LDS: GNND_F64_SPTAB 1 (default) a one-read
// table (GNND_F64_SGTAB 1, default: kSgTab, softplus_sg; 0: kSpTab, softplus_sp), 0 the exp +
// log1p tables (softplus_fast; A/B builds)
#ifndef GNND_F64_SPTAB
#define GNND_F64_SPTAB 1
#endif
#ifndef GNND_F64_SGTAB
#define GNND_F64_SGTAB GNND_F64_SPTAB
#endif
constexpr int kV24F64TabDoubles =
    GNND_F64_SGTAB ? kSgTabDoubles : GNND_F64_SPTAB ? kSpTabDoubles : kFp64TabDoubles;
__device__ __forceinline__ double v24_f64_tab_entry(int i) {
    if (GNND_F64_SGTAB) return kSgTab[i];
    if (GNND_F64_SPTAB) return kSpTab[i];
    return i < kExpTabN ? kExpTab[i] : kLogTab[i - kExpTabN];
}
__device__ __forceinline__ double softplus_v24(double x, const double* __restrict__ tab) {
    if (GNND_F64_SGTAB) return softplus_sg(x, tab);
    if (GNND_F64_SPTAB) return softplus_sp(x, tab);
    return softplus_fast(x, tab);
}
// softplus(x) - x/2 (the linear x/2 is summed per MLP: decode_kernel mlp_lin): kSgTab's g(x)
// directly, or |x|/2 + ln(1 + e^-|x|) from kSpTab (one FMA instead of relu's max + add); the
// exp + log1p form (GNND_F64_SPTAB 0) keeps the whole value
#ifndef GNND_F64_LINFOLD
#define GNND_F64_LINFOLD GNND_F64_SPTAB   // 0: whole Softplus per unit, no per-MLP linear part (A/B)
#endif
// the one-read forms in two steps (index, then the value from the read entry), so a caller can
// issue several units' table reads together (decode_kernel mlp128d_chains_cm)
template <bool SAFE = false>
__device__ __forceinline__ SpIdx v24_sp_index(double x) {
    if (GNND_F64_SGTAB) return SAFE ? sg_index_safe(x) : sg_index(x);
    return sp_index(x);
}
__device__ __forceinline__ double v24_sp_half(const SpIdx& q, const SpEntry& e, double x) {
    if (GNND_F64_SGTAB) return sg_poly(q.r, e.f0, e.s);
    return __builtin_fma(__builtin_fabs(x), 0.5, sp_poly(q.r, e.f0, e.s));
}
template <bool SAFE = false>
__device__ __forceinline__ double softplus_v24_half(double x, const double* __restrict__ tab) {
    if (!GNND_F64_LINFOLD) return softplus_v24(x, tab);
    if (GNND_F64_SPTAB) {
        const SpIdx q = v24_sp_index<SAFE>(x);
        return v24_sp_half(q, sp_entry(tab, q.j), x);
    }
    return softplus_fast(x, tab);
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
// the same butterfly as a product (the fp32 BP check step's magnitude products)
template <int G> __device__ __forceinline__ float group_prod_c(float v) {
    if constexpr (G > 1) v *= dpp_mov<0xB1>(v);
    if constexpr (G > 2) v *= dpp_mov<0x4E>(v);
    if constexpr (G > 4) v *= dpp_mov<0x141>(v);
    if constexpr (G > 8) v *= dpp_mov<0x140>(v);
    if constexpr (G > 16) v *= __shfl_xor(v, 16);
    if constexpr (G > 32) v *= __shfl_xor(v, 32);
    return v;
}
// fp64: the same butterfly, each step moving the two 32-bit halves with DPP
template <int CTRL> __device__ __forceinline__ double dpp_mov(double v) {
    const int2 h = __builtin_bit_cast(int2, v);
    const int2 r = {__builtin_amdgcn_update_dpp(0, h.x, CTRL, 0xf, 0xf, false),
                    __builtin_amdgcn_update_dpp(0, h.y, CTRL, 0xf, 0xf, false)};
    return __builtin_bit_cast(double, r);
}
template <int G> __device__ __forceinline__ double group_prod_c(double v) {
    if constexpr (G > 1) v *= dpp_mov<0xB1>(v);
    if constexpr (G > 2) v *= dpp_mov<0x4E>(v);
    if constexpr (G > 4) v *= dpp_mov<0x141>(v);
    if constexpr (G > 8) v *= dpp_mov<0x140>(v);
    if constexpr (G > 16) v *= __shfl_xor(v, 16);
    if constexpr (G > 32) v *= __shfl_xor(v, 32);
    return v;
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
