// gnnd_common.h — shared device/host helpers for libgnnd (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>
#include "../../include/gnnd.h"

#define GNND_BLOCK 256

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
// phase timing (timing experiments only, -DGNND_PHASE_PROF): one wave of workgroup 0 sums the
// shader-clock cycles (s_memtime) spent between consecutive marks and prints the per-phase
// totals at the end of the launch.  Release builds compile the marks away.
// ---------------------------------------------------------------------------------------
struct PhaseProf {
#ifdef GNND_PHASE_PROF
    uint64_t acc[16];
    uint64_t last;
    bool on;
    __device__ void start(bool enable) {
        on = enable;
        for (int i = 0; i < 16; ++i) acc[i] = 0;
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
            printf("PHASE %s iters %d | %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu\n",
                   tag, iters, (unsigned long long)acc[0], (unsigned long long)acc[1],
                   (unsigned long long)acc[2], (unsigned long long)acc[3], (unsigned long long)acc[4],
                   (unsigned long long)acc[5], (unsigned long long)acc[6], (unsigned long long)acc[7],
                   (unsigned long long)acc[8], (unsigned long long)acc[9], (unsigned long long)acc[10],
                   (unsigned long long)acc[11], (unsigned long long)acc[12], (unsigned long long)acc[13],
                   (unsigned long long)acc[14], (unsigned long long)acc[15]);
        (void)n;
    }
#endif
};
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
