// gnnd_propagate.hip — one MessagePassing.propagate() call on the device.
//
// Restates the per-script propagate bodies (paths relative to /root/reference/GNN-decode/):
//   V24   quantum/decoder_v2_4.py:132-144   QGNNI quantum/QGNNI.py:101-112
//   QBP   quantum/BP.py:101-119             CGNNI classical/CGNNI.py:99-108
//   CBP   classical/BP.py:99-119            NBP   quantum/neural_BP.py:108-131
//   V10   quantum/decoder_v1_0.py:109-131   V30   quantum/decoder_v3_0.py:106-118
// i.e.  out = post( scatter_(aggr, pre(msg), idx_j, dim_size)[idx_j] - pre(msg), extra[idx_j] )
// with idx_j = edge_index[0] for flow source_to_target and edge_index[1] for
// target_to_source (quantum/decoder_v2_4.py:89), PyG-1.x scatter_ fill rules
// (quantum/decoder_v2_4.py:34-51).
//
// Two device paths:
//  * tiled   — the batched edge_index is the single Tanner graph tiled over codewords (what
//              every reference model passes).  One workgroup owns a tile of codewords:
//              pre-op'd messages are staged in LDS, node aggregates are a deterministic
//              segmented reduce in edge order (no atomics, no int64 index reads), and the
//              per-edge output is written once, coalesced.  HBM-bound: per call it moves
//              E*B*s in + E*B*F*s out + N*B*s of extra.
//  * generic — any edge_index (and the reference's literal leave-one-out `mean`, whose
//              second gather indexes the per-edge array by node id): float atomics.
#include "gnnd_common.h"

namespace {

template <typename T> __device__ __forceinline__ T cst(double v) { return (T)v; }

constexpr int AG_ADD = GNND_AGGR_ADD, AG_MEAN = GNND_AGGR_MEAN, AG_MAX = GNND_AGGR_MAX;

__host__ __device__ constexpr bool is_bp(int var) {
    return var == GNND_QBP || var == GNND_CBP || var == GNND_NBP || var == GNND_V10;
}
// syndrome-aware quantum BP bodies (sign term (1 - s)/2, log(1+p) - log(1-p))
__host__ __device__ constexpr bool is_qbp(int var) {
    return var == GNND_QBP || var == GNND_NBP || var == GNND_V10;
}
// the weighted-BP scripts drop the +-10 pre-clamp and clamp p at 1 - 1e-15
__host__ __device__ constexpr bool is_nbp(int var) { return var == GNND_NBP || var == GNND_V10; }

__host__ __device__ constexpr int out_width(int var, int flow) {
    return (var == GNND_V24 || var == GNND_V30 || (var == GNND_QGNNI && flow == GNND_TARGET_TO_SOURCE) ||
            (var == GNND_NBP && flow == GNND_SOURCE_TO_TARGET)) ? 2 : 1;
}

template <int VAR, typename T> __device__ __forceinline__ T bp_lo() {
    return VAR == GNND_CBP ? cst<T>(1e-7) : cst<T>(1e-20);
}
template <int VAR, typename T> __device__ __forceinline__ T bp_hi() {
    return VAR == GNND_CBP ? cst<T>(1 - 1e-7) : is_nbp(VAR) ? cst<T>(1 - 1e-15) : cst<T>(1 - 1e-12);
}
// BP c->v input: tanh(x/2) after the +-10 clamp (QBP/CBP only)
template <int VAR, typename T> __device__ __forceinline__ T bp_tanh(T m) {
    if constexpr (is_nbp(VAR)) return g_tanh(m / T(2));
    else return g_tanh(g_clamp(m, T(-10), T(10)) / T(2));
}

// c->v pre-op on the per-edge message (the BP variants also produce the sign indicator;
// decoder_v3_0 aggregates the raw edge states on both sides, its tanh is commented out)
template <int VAR, int FLOW, typename T>
__device__ __forceinline__ T pre_op(T m, T* coeff) {
    if constexpr (FLOW == GNND_TARGET_TO_SOURCE && VAR != GNND_V30) {
        if constexpr (is_bp(VAR)) {
            T t = bp_tanh<VAR, T>(m);
            *coeff = t < T(0) ? T(1) : T(0);
            return g_log(g_clamp(g_abs(t), bp_lo<VAR, T>(), cst<T>(1e10)));
        } else {
            return g_tanh(m / T(2));
        }
    } else {
        return m;
    }
}

// post-op: val = aggregated-leave-one-out value, val2 = same for BP's sign indicator,
// ex = extra[idx_j] (or 0 if absent).  Writes F values.
template <int VAR, int FLOW, typename T>
__device__ __forceinline__ void post_op(T val, T val2, T ex, bool has_extra, T* o) {
    if constexpr (is_bp(VAR) && FLOW == GNND_TARGET_TO_SOURCE) {
        T n = val2;
        if constexpr (is_qbp(VAR)) n = n + (T(1) - ex) / T(2);
        const T hi = bp_hi<VAR, T>();
        T p = g_clamp(g_exp(val) * cos_pi(n), -hi, hi);
        if constexpr (is_qbp(VAR))
            o[0] = g_log(T(1) + p) - g_log(T(1) - p);
        else
            o[0] = g_log((T(1) + p) / (T(1) - p));
    } else if constexpr (out_width(VAR, FLOW) == 2) {
        o[0] = val;
        o[1] = ex;
    } else if constexpr (VAR == GNND_CGNNI) {
        o[0] = has_extra ? val + ex : val;
    } else {   // QGNNI / QBP / CBP / V10 source_to_target: + extra
        o[0] = val + ex;
    }
}

template <int AGGR, typename T> struct Agg {
    __device__ static T init() { return AGGR == AG_MAX ? cst<T>(-1e9) : T(0); }
    __device__ static T step(T a, T v) { return AGGR == AG_MAX ? (v > a ? v : a) : a + v; }
    __device__ static T fin(T a) { return (AGGR == AG_MAX && a == cst<T>(-1e9)) ? T(0) : a; }
};

// ---------------------------------------------------------------------------------------
// tiled path
// ---------------------------------------------------------------------------------------
template <int VAR, int FLOW, int AGGR, typename T>
__global__ void __launch_bounds__(GNND_BLOCK)
propagate_tiled_kernel(GraphView g, const T* __restrict__ msg, const T* __restrict__ extra,
                       T* __restrict__ out, int64_t B, int CW, FastDiv dNode, FastDiv dE) {
    constexpr bool BP = is_bp(VAR) && FLOW == GNND_TARGET_TO_SOURCE;
    constexpr bool VARSIDE = FLOW == GNND_SOURCE_TO_TARGET;
    constexpr int F = out_width(VAR, FLOW);
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int V = g.V, C = g.C, E = g.E, N = g.N;
    const int tid = threadIdx.x;
    int* s_tab = (int*)smem;
    const int nints = graph_table_ints(V, C, E);
    const uint32_t* s_evc = (const uint32_t*)s_tab;
    const int* s_vptr = s_tab + E;
    const int* s_cptr = s_vptr + V + 1;
    const int* s_cedge = s_cptr + C + 1;
    size_t off = ((size_t)nints * 4 + 15) & ~(size_t)15;
    const int NJ = VARSIDE ? V : C;                // nodes on the aggregation side
    T* s_src = (T*)(smem + off);                   // [CW][E]
    T* s_src2 = s_src + (size_t)CW * E;            // [CW][E]  BP sign indicator
    T* s_agg = s_src2 + (BP ? (size_t)CW * E : 0); // [CW][NJ]
    T* s_agg2 = s_agg + (size_t)CW * NJ;           // [CW][NJ] BP

    const int* gtab = (const int*)g.edge_vc;
    for (int i = tid; i < nints; i += GNND_BLOCK) s_tab[i] = gtab[i];
    const int64_t b0 = (int64_t)blockIdx.x * CW;
    const int nb = (int)((B - b0) < CW ? (B - b0) : CW);
    const int nE = nb * E;
    const T* mg = msg + b0 * E;
    for (int f = tid; f < nE; f += GNND_BLOCK) {
        T c2 = T(0);
        s_src[f] = pre_op<VAR, FLOW, T>(mg[f], &c2);
        if constexpr (BP) s_src2[f] = c2;
    }
    __syncthreads();
    for (int f = tid; f < nb * NJ; f += GNND_BLOCK) {
        int b = fdiv(f, dNode), j = f - b * NJ;
        const T* sb = s_src + b * E;
        T a = Agg<AGGR, T>::init(), a2 = Agg<AGGR, T>::init();
        if constexpr (VARSIDE) {
            for (int k = s_vptr[j], ke = s_vptr[j + 1]; k < ke; ++k) a = Agg<AGGR, T>::step(a, sb[k]);
        } else {
            for (int k = s_cptr[j], ke = s_cptr[j + 1]; k < ke; ++k) {
                int e = s_cedge[k];
                a = Agg<AGGR, T>::step(a, sb[e]);
                if constexpr (BP) a2 = Agg<AGGR, T>::step(a2, s_src2[b * E + e]);
            }
        }
        s_agg[f] = Agg<AGGR, T>::fin(a);
        if constexpr (BP) s_agg2[f] = Agg<AGGR, T>::fin(a2);
    }
    __syncthreads();
    T* og = out + b0 * E * F;
    const bool has_extra = extra != nullptr;
    for (int f = tid; f < nE; f += GNND_BLOCK) {
        int b = fdiv(f, dE), e = f - b * E;
        uint32_t vc = s_evc[e];
        int j = GNND_DIDX(VARSIDE ? (int)(vc & 0xffffu) : (int)(vc >> 16), NJ, GNND_DBG_NODE);
        T val = s_agg[b * NJ + j] - s_src[f];
        T val2 = T(0);
        if constexpr (BP) val2 = s_agg2[b * NJ + j] - s_src2[f];
        T ex = T(0);
        if (has_extra) ex = extra[(b0 + b) * N + (VARSIDE ? j : V + j)];
        T o[F];
        post_op<VAR, FLOW, T>(val, val2, ex, has_extra, o);
#pragma unroll
        for (int q = 0; q < F; ++q) og[(size_t)f * F + q] = o[q];
    }
}

constexpr size_t kLdsTarget = 32 * 1024;

template <int VAR, int FLOW, int AGGR, typename T>
int launch_tiled(const gnnd_graph* gr, const void* msg, const void* extra, void* out,
                 int64_t B, hipStream_t st) {
    const GraphView& g = gr->view;
    constexpr bool BP = is_bp(VAR) && FLOW == GNND_TARGET_TO_SOURCE;
    const int NJ = FLOW == GNND_SOURCE_TO_TARGET ? g.V : g.C;
    const size_t tab = ((size_t)graph_table_ints(g.V, g.C, g.E) * 4 + 15) & ~(size_t)15;
    const size_t per = sizeof(T) * ((size_t)g.E * (BP ? 2 : 1) + (size_t)NJ * (BP ? 2 : 1));
    if (tab + per > 160 * 1024) return GNND_ERR_UNSUPPORTED;
    size_t cw = tab + per >= kLdsTarget ? 1 : (kLdsTarget - tab) / per;
    if (cw > 64) cw = 64;
    size_t lds = tab + cw * per;
    auto kern = propagate_tiled_kernel<VAR, FLOW, AGGR, T>;
    if (lds > 64 * 1024)
        GNND_HIP_CHECK(hipFuncSetAttribute((const void*)kern,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    int64_t blocks = (B + (int64_t)cw - 1) / (int64_t)cw;
    if (blocks > 0x7fffffff) return GNND_ERR_UNSUPPORTED;
    kern<<<(unsigned)blocks, GNND_BLOCK, lds, st>>>(g, (const T*)msg, (const T*)extra, (T*)out, B,
                                                     (int)cw, make_fastdiv(NJ), make_fastdiv(g.E));
    GNND_LAUNCH_CHECK();
    return GNND_OK;
}

template <int VAR, int FLOW, typename T>
int tiled_aggr(const gnnd_graph* g, int aggr, const void* m, const void* ex, void* o, int64_t B,
               hipStream_t st) {
    if (aggr == AG_ADD) return launch_tiled<VAR, FLOW, AG_ADD, T>(g, m, ex, o, B, st);
    if (aggr == AG_MAX) return launch_tiled<VAR, FLOW, AG_MAX, T>(g, m, ex, o, B, st);
    return GNND_ERR_UNSUPPORTED;   // mean: literal semantics need the generic path
}

template <int VAR, typename T>
int tiled_flow(const gnnd_graph* g, int flow, int aggr, const void* m, const void* ex, void* o,
               int64_t B, hipStream_t st) {
    if (flow == GNND_SOURCE_TO_TARGET) return tiled_aggr<VAR, GNND_SOURCE_TO_TARGET, T>(g, aggr, m, ex, o, B, st);
    return tiled_aggr<VAR, GNND_TARGET_TO_SOURCE, T>(g, aggr, m, ex, o, B, st);
}

template <typename T>
int tiled_var(const gnnd_graph* g, int var, int flow, int aggr, const void* m, const void* ex,
              void* o, int64_t B, hipStream_t st) {
    switch (var) {
        case GNND_V24: return tiled_flow<GNND_V24, T>(g, flow, aggr, m, ex, o, B, st);
        case GNND_QGNNI: return tiled_flow<GNND_QGNNI, T>(g, flow, aggr, m, ex, o, B, st);
        case GNND_QBP: return tiled_flow<GNND_QBP, T>(g, flow, aggr, m, ex, o, B, st);
        case GNND_CGNNI: return tiled_flow<GNND_CGNNI, T>(g, flow, aggr, m, ex, o, B, st);
        case GNND_CBP: return tiled_flow<GNND_CBP, T>(g, flow, aggr, m, ex, o, B, st);
        case GNND_NBP: return tiled_flow<GNND_NBP, T>(g, flow, aggr, m, ex, o, B, st);
        case GNND_V10: return tiled_flow<GNND_V10, T>(g, flow, aggr, m, ex, o, B, st);
        case GNND_V30: return tiled_flow<GNND_V30, T>(g, flow, aggr, m, ex, o, B, st);
    }
    return GNND_ERR_INVALID_ARG;
}

// ---------------------------------------------------------------------------------------
// generic path (arbitrary edge_index), float atomics
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void atomic_max_t(float* a, float v) {
    unsigned int* p = (unsigned int*)a;
    unsigned int old = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (__uint_as_float(old) < v) {
        unsigned int prev = atomicCAS(p, old, __float_as_uint(v));
        if (prev == old) break;
        old = prev;
    }
}
__device__ __forceinline__ void atomic_max_t(double* a, double v) {
    unsigned long long* p = (unsigned long long*)a;
    unsigned long long old = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (__longlong_as_double((long long)old) < v) {
        unsigned long long prev = atomicCAS(p, old, (unsigned long long)__double_as_longlong(v));
        if (prev == old) break;
        old = prev;
    }
}

template <typename T>
__global__ void fill_kernel(T* p, int64_t n, T v) {
    int64_t i = (int64_t)blockIdx.x * GNND_BLOCK + threadIdx.x;
    if (i < n) p[i] = v;
}

template <int VAR, int FLOW, int AGGR, typename T>
__global__ void __launch_bounds__(GNND_BLOCK)
gen_scatter_kernel(const int64_t* __restrict__ idx, const T* __restrict__ msg, int64_t nE,
                   int64_t dim, T* src, T* src2, T* agg, T* agg2, T* cnt) {
    constexpr bool BP = is_bp(VAR) && FLOW == GNND_TARGET_TO_SOURCE;
    int64_t e = (int64_t)blockIdx.x * GNND_BLOCK + threadIdx.x;
    if (e >= nE) return;
    T c2 = T(0);
    T s = pre_op<VAR, FLOW, T>(msg[e], &c2);
    src[e] = s;
    if constexpr (BP) src2[e] = c2;
    int64_t j = idx[e];
    if (j < 0 || j >= dim) return;        // out-of-range index: output becomes NaN below
    if constexpr (AGGR == AG_MAX) {
        atomic_max_t(agg + j, s);
        if constexpr (BP) atomic_max_t(agg2 + j, c2);
    } else {
        atomicAdd(agg + j, s);
        if constexpr (BP) atomicAdd(agg2 + j, c2);
        if constexpr (AGGR == AG_MEAN) atomicAdd(cnt + j, T(1));
    }
}

// mean: lm[e] = (S[idx e] - src e) / max(cnt[idx e] - 1, 1)   (decoder_v2_4.py:27-31)
template <typename T>
__global__ void __launch_bounds__(GNND_BLOCK)
gen_mean_kernel(const int64_t* __restrict__ idx, int64_t nE, int64_t dim, const T* src,
                const T* agg, const T* cnt, T* lm) {
    int64_t e = (int64_t)blockIdx.x * GNND_BLOCK + threadIdx.x;
    if (e >= nE) return;
    int64_t j = idx[e];
    if (j < 0 || j >= dim) { lm[e] = T(NAN); return; }
    T c = cnt[j] - T(1);
    lm[e] = (agg[j] - src[e]) / (c < T(1) ? T(1) : c);
}

template <int VAR, int FLOW, int AGGR, typename T>
__global__ void __launch_bounds__(GNND_BLOCK)
gen_out_kernel(const int64_t* __restrict__ idx, int64_t nE, int64_t dim, const T* src,
               const T* src2, const T* agg, const T* agg2, const T* lm,
               const T* __restrict__ extra, T* __restrict__ out) {
    constexpr bool BP = is_bp(VAR) && FLOW == GNND_TARGET_TO_SOURCE;
    constexpr int F = out_width(VAR, FLOW);
    int64_t e = (int64_t)blockIdx.x * GNND_BLOCK + threadIdx.x;
    if (e >= nE) return;
    int64_t j = idx[e];
    if (j < 0 || j >= dim) {
#pragma unroll
        for (int q = 0; q < F; ++q) out[e * F + q] = T(NAN);
        return;
    }
    T val, val2 = T(0);
    if constexpr (AGGR == AG_MEAN) {
        // scatter_mean already returned the gathered per-edge array; propagate indexes it
        // again by node id (decoder_v2_4.py:136/138) — restated literally.
        val = (j < nE ? lm[j] : T(NAN)) - src[e];
        if constexpr (BP) val2 = (j < nE ? lm[nE + j] : T(NAN)) - src2[e];
    } else {
        val = Agg<AGGR, T>::fin(agg[j]) - src[e];
        if constexpr (BP) val2 = Agg<AGGR, T>::fin(agg2[j]) - src2[e];
    }
    const bool has_extra = extra != nullptr;
    T ex = has_extra ? extra[j] : T(0);
    T o[F];
    post_op<VAR, FLOW, T>(val, val2, ex, has_extra, o);
#pragma unroll
    for (int q = 0; q < F; ++q) out[e * F + q] = o[q];
}

struct GenLayout {   // element offsets inside the workspace
    int64_t src, src2, agg, agg2, cnt, lm, total;
};
GenLayout gen_layout(bool bp, int aggr, int64_t nE, int64_t dim) {
    GenLayout L;
    int64_t o = 0;
    L.src = o; o += nE;
    L.src2 = o; o += bp ? nE : 0;
    L.agg = o; o += dim;
    L.agg2 = o; o += bp ? dim : 0;
    L.cnt = o; o += aggr == AG_MEAN ? dim : 0;
    L.lm = o; o += aggr == AG_MEAN ? (bp ? 2 * nE : nE) : 0;
    L.total = o;
    return L;
}

template <int VAR, int FLOW, int AGGR, typename T>
int launch_generic(const int64_t* ei, int64_t stride, int64_t nE, const void* msg, const void* extra,
                   int64_t dim, void* out, void* ws, int64_t ws_bytes, hipStream_t st) {
    constexpr bool BP = is_bp(VAR) && FLOW == GNND_TARGET_TO_SOURCE;
    GenLayout L = gen_layout(BP, AGGR, nE, dim);
    if (ws_bytes < L.total * (int64_t)sizeof(T)) return GNND_ERR_INVALID_ARG;
    T* w = (T*)ws;
    const int64_t* idx = ei + (FLOW == GNND_SOURCE_TO_TARGET ? 0 : stride);
    const unsigned gE = (unsigned)((nE + GNND_BLOCK - 1) / GNND_BLOCK);
    const unsigned gD = (unsigned)((dim + GNND_BLOCK - 1) / GNND_BLOCK);
    const T init = AGGR == AG_MAX ? (T)-1e9 : T(0);
    if (dim > 0) {
        fill_kernel<T><<<gD, GNND_BLOCK, 0, st>>>(w + L.agg, dim, init);
        if (BP) fill_kernel<T><<<gD, GNND_BLOCK, 0, st>>>(w + L.agg2, dim, init);
        if (AGGR == AG_MEAN) fill_kernel<T><<<gD, GNND_BLOCK, 0, st>>>(w + L.cnt, dim, T(0));
        GNND_LAUNCH_CHECK();
    }
    if (nE == 0) return GNND_OK;
    gen_scatter_kernel<VAR, FLOW, AGGR, T><<<gE, GNND_BLOCK, 0, st>>>(
        idx, (const T*)msg, nE, dim, w + L.src, w + L.src2, w + L.agg, w + L.agg2, w + L.cnt);
    GNND_LAUNCH_CHECK();
    if (AGGR == AG_MEAN) {
        gen_mean_kernel<T><<<gE, GNND_BLOCK, 0, st>>>(idx, nE, dim, w + L.src, w + L.agg, w + L.cnt, w + L.lm);
        if (BP)
            gen_mean_kernel<T><<<gE, GNND_BLOCK, 0, st>>>(idx, nE, dim, w + L.src2, w + L.agg2, w + L.cnt,
                                                        w + L.lm + nE);
        GNND_LAUNCH_CHECK();
    }
    gen_out_kernel<VAR, FLOW, AGGR, T><<<gE, GNND_BLOCK, 0, st>>>(
        idx, nE, dim, w + L.src, w + L.src2, w + L.agg, w + L.agg2, w + L.lm, (const T*)extra,
        (T*)out);
    GNND_LAUNCH_CHECK();
    return GNND_OK;
}

template <int VAR, int FLOW, typename T>
int gen_aggr(int aggr, const int64_t* ei, int64_t s, int64_t nE, const void* m, const void* ex,
             int64_t dim, void* o, void* ws, int64_t wb, hipStream_t st) {
    if (aggr == AG_ADD) return launch_generic<VAR, FLOW, AG_ADD, T>(ei, s, nE, m, ex, dim, o, ws, wb, st);
    if (aggr == AG_MEAN) return launch_generic<VAR, FLOW, AG_MEAN, T>(ei, s, nE, m, ex, dim, o, ws, wb, st);
    if (aggr == AG_MAX) return launch_generic<VAR, FLOW, AG_MAX, T>(ei, s, nE, m, ex, dim, o, ws, wb, st);
    return GNND_ERR_INVALID_ARG;
}

template <int VAR, typename T>
int gen_flow(int flow, int aggr, const int64_t* ei, int64_t s, int64_t nE, const void* m,
             const void* ex, int64_t dim, void* o, void* ws, int64_t wb, hipStream_t st) {
    if (flow == GNND_SOURCE_TO_TARGET)
        return gen_aggr<VAR, GNND_SOURCE_TO_TARGET, T>(aggr, ei, s, nE, m, ex, dim, o, ws, wb, st);
    return gen_aggr<VAR, GNND_TARGET_TO_SOURCE, T>(aggr, ei, s, nE, m, ex, dim, o, ws, wb, st);
}

template <typename T>
int gen_var(int var, int flow, int aggr, const int64_t* ei, int64_t s, int64_t nE, const void* m,
            const void* ex, int64_t dim, void* o, void* ws, int64_t wb, hipStream_t st) {
    switch (var) {
        case GNND_V24: return gen_flow<GNND_V24, T>(flow, aggr, ei, s, nE, m, ex, dim, o, ws, wb, st);
        case GNND_QGNNI: return gen_flow<GNND_QGNNI, T>(flow, aggr, ei, s, nE, m, ex, dim, o, ws, wb, st);
        case GNND_QBP: return gen_flow<GNND_QBP, T>(flow, aggr, ei, s, nE, m, ex, dim, o, ws, wb, st);
        case GNND_CGNNI: return gen_flow<GNND_CGNNI, T>(flow, aggr, ei, s, nE, m, ex, dim, o, ws, wb, st);
        case GNND_CBP: return gen_flow<GNND_CBP, T>(flow, aggr, ei, s, nE, m, ex, dim, o, ws, wb, st);
        case GNND_NBP: return gen_flow<GNND_NBP, T>(flow, aggr, ei, s, nE, m, ex, dim, o, ws, wb, st);
        case GNND_V10: return gen_flow<GNND_V10, T>(flow, aggr, ei, s, nE, m, ex, dim, o, ws, wb, st);
        case GNND_V30: return gen_flow<GNND_V30, T>(flow, aggr, ei, s, nE, m, ex, dim, o, ws, wb, st);
    }
    return GNND_ERR_INVALID_ARG;
}

bool valid_common(int var, int flow, int aggr, int dtype) {
    return var >= GNND_V24 && var <= GNND_V30 &&
           (flow == GNND_SOURCE_TO_TARGET || flow == GNND_TARGET_TO_SOURCE) &&
           aggr >= AG_ADD && aggr <= AG_MAX && (dtype == GNND_F32 || dtype == GNND_F64);
}


// ---------------------------------------------------------------------------------------
// backward of one propagate call w.r.t. the per-edge message (aggr 'add', non-BP bodies).
// out_e[0] = S_j(pre(msg))_e - pre(msg_e) (+ extra or cat extra, which carry no msg
// gradient), so grad_pre_e = sum_{e' at node j(e)} g_e' - g_e (the same leave-one-out
// aggregation applied to the output gradient), times d pre / d msg:
//   c->v tanh(msg/2):  (grad * (1 - t*t)) / 2   (torch tanh_backward then div_backward)
// ---------------------------------------------------------------------------------------
template <int VAR, int FLOW, typename T>
__device__ __forceinline__ T pre_grad(T msg, T gpre) {
    if constexpr (FLOW == GNND_TARGET_TO_SOURCE && VAR != GNND_V30) {
        T t = g_tanh(msg / T(2));
        return (gpre * (T(1) - t * t)) / T(2);
    } else {
        return gpre;
    }
}

template <int VAR, int FLOW, typename T>
__global__ void __launch_bounds__(GNND_BLOCK)
propagate_tiled_bwd_kernel(GraphView g, const T* __restrict__ msg, const T* __restrict__ gout,
                           T* __restrict__ gmsg, int64_t B, int CW, FastDiv dNode, FastDiv dE) {
    constexpr bool VARSIDE = FLOW == GNND_SOURCE_TO_TARGET;
    constexpr int F = out_width(VAR, FLOW);
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int V = g.V, C = g.C, E = g.E;
    const int tid = threadIdx.x;
    int* s_tab = (int*)smem;
    const int nints = graph_table_ints(V, C, E);
    const uint32_t* s_evc = (const uint32_t*)s_tab;
    const int* s_vptr = s_tab + E;
    const int* s_cptr = s_vptr + V + 1;
    const int* s_cedge = s_cptr + C + 1;
    size_t off = ((size_t)nints * 4 + 15) & ~(size_t)15;
    const int NJ = VARSIDE ? V : C;
    T* s_g = (T*)(smem + off);                 // [CW][E]
    T* s_agg = s_g + (size_t)CW * E;           // [CW][NJ]
    const int* gtab = (const int*)g.edge_vc;
    for (int i = tid; i < nints; i += GNND_BLOCK) s_tab[i] = gtab[i];
    const int64_t b0 = (int64_t)blockIdx.x * CW;
    const int nb = (int)((B - b0) < CW ? (B - b0) : CW);
    const int nE = nb * E;
    const T* gg = gout + b0 * E * F;
    for (int f = tid; f < nE; f += GNND_BLOCK) s_g[f] = gg[(size_t)f * F];
    __syncthreads();
    for (int f = tid; f < nb * NJ; f += GNND_BLOCK) {
        int b = fdiv(f, dNode), j = f - b * NJ;
        const T* sb = s_g + b * E;
        T a = T(0);
        if constexpr (VARSIDE) {
            for (int k = s_vptr[j], ke = s_vptr[j + 1]; k < ke; ++k) a += sb[k];
        } else {
            for (int k = s_cptr[j], ke = s_cptr[j + 1]; k < ke; ++k) a += sb[s_cedge[k]];
        }
        s_agg[f] = a;
    }
    __syncthreads();
    const T* mg = msg + b0 * E;
    T* og = gmsg + b0 * E;
    for (int f = tid; f < nE; f += GNND_BLOCK) {
        int b = fdiv(f, dE), e = f - b * E;
        uint32_t vc = s_evc[e];
        int j = VARSIDE ? (int)(vc & 0xffffu) : (int)(vc >> 16);
        og[f] = pre_grad<VAR, FLOW, T>(mg[f], s_agg[b * NJ + j] - s_g[f]);
    }
}

// ---------------------------------------------------------------------------------------
// backward of the c->v BP bodies (QBP, CBP, NBP, V10; flow target_to_source, aggr 'add').
// The forward is recomputed per check:  t = tanh(x/2) (QBP/CBP: x clamped to +-10 first),
// L = log(clamp(|t|, lo, 1e10)), Lambda = S_c(L) - L, n = S_c([t<0]) - [t<0] (+ (1-s)/2),
// q = exp(Lambda), p = clamp(q cos(pi n), -hi, hi), out = log(1+p) - log(1-p) (CBP:
// log((1+p)/(1-p))).  torch's autograd rules, in its order:
//   g_p = g (1/(1+p) + 1/(1-p)) [p inside the clamp]   g_Lambda = (g_p cos) q
//   g_L = S_c(g_Lambda) - g_Lambda                     (leave-one-out, like the forward)
//   g_t = g_L / clamp(|t|) [|t| inside the clamp] sgn(t)
//   g_x = (g_t (1 - t^2)) / 2 [QBP/CBP: x inside +-10]
// ---------------------------------------------------------------------------------------
template <int VAR, typename T> struct BpFwd {
    T t, L, c;
    __device__ __forceinline__ void init(T m) {
        t = bp_tanh<VAR, T>(m);
        c = t < T(0) ? T(1) : T(0);
        L = g_log(g_clamp(g_abs(t), bp_lo<VAR, T>(), cst<T>(1e10)));
    }
    // gradient w.r.t. the input message given g_L
    __device__ __forceinline__ T input_grad(T m, T gL) const {
        const T u = g_abs(t);
        const T uc = g_clamp(u, bp_lo<VAR, T>(), cst<T>(1e10));
        T gu = (u >= bp_lo<VAR, T>() && u <= cst<T>(1e10)) ? gL / uc : T(0);
        T gt = gu * (t > T(0) ? T(1) : (t < T(0) ? T(-1) : T(0)));
        T gx = (gt * (T(1) - t * t)) / T(2);
        if constexpr (!is_nbp(VAR)) gx = (m >= T(-10) && m <= T(10)) ? gx : T(0);
        return gx;
    }
};
// g_Lambda of one edge from its leave-one-out sums (lam, n) and the output gradient
template <int VAR, typename T>
__device__ __forceinline__ T bp_lambda_grad(T lam, T n, T ex, T g) {
    if constexpr (is_qbp(VAR)) n = n + (T(1) - ex) / T(2);
    const T hi = bp_hi<VAR, T>();
    const T sgn = cos_pi(n), q = g_exp(lam);
    const T p = q * sgn;
    const T pc = g_clamp(p, -hi, hi);
    T gp;
    if constexpr (is_qbp(VAR)) gp = g / (T(1) + pc) + g / (T(1) - pc);
    else gp = T(2) * g / ((T(1) + pc) * (T(1) - pc));
    gp = (p >= -hi && p <= hi) ? gp : T(0);
    return (gp * sgn) * q;
}

template <int VAR, typename T>
__global__ void __launch_bounds__(GNND_BLOCK)
propagate_tiled_bp_bwd_kernel(GraphView g, const T* __restrict__ msg, const T* __restrict__ extra,
                              const T* __restrict__ gout, T* __restrict__ gmsg, int64_t B, int CW,
                              FastDiv dNode, FastDiv dE) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int V = g.V, C = g.C, E = g.E, N = g.N;
    const int tid = threadIdx.x;
    int* s_tab = (int*)smem;
    const int nints = graph_table_ints(V, C, E);
    const uint32_t* s_evc = (const uint32_t*)s_tab;
    const int* s_cptr = s_tab + E + V + 1;
    const int* s_cedge = s_cptr + C + 1;
    size_t off = ((size_t)nints * 4 + 15) & ~(size_t)15;
    T* s_L = (T*)(smem + off);                 // [CW][E]
    T* s_c = s_L + (size_t)CW * E;             // [CW][E]  sign indicator, then g_Lambda
    T* s_aL = s_c + (size_t)CW * E;            // [CW][C]  S_c(L), then S_c(g_Lambda)
    T* s_ac = s_aL + (size_t)CW * C;           // [CW][C]  S_c(sign)
    const int* gtab = (const int*)g.edge_vc;
    for (int i = tid; i < nints; i += GNND_BLOCK) s_tab[i] = gtab[i];
    const int64_t b0 = (int64_t)blockIdx.x * CW;
    const int nb = (int)((B - b0) < CW ? (B - b0) : CW);
    const int nE = nb * E;
    const T* mg = msg + b0 * E;
    for (int f = tid; f < nE; f += GNND_BLOCK) {
        BpFwd<VAR, T> fw;
        fw.init(mg[f]);
        s_L[f] = fw.L;
        s_c[f] = fw.c;
    }
    __syncthreads();
    for (int f = tid; f < nb * C; f += GNND_BLOCK) {
        int b = fdiv(f, dNode), j = f - b * C;
        T a = T(0), a2 = T(0);
        for (int k = s_cptr[j], ke = s_cptr[j + 1]; k < ke; ++k) {
            int e = s_cedge[k];
            a += s_L[b * E + e];
            a2 += s_c[b * E + e];
        }
        s_aL[f] = a;
        s_ac[f] = a2;
    }
    __syncthreads();
    const T* gg = gout + b0 * E;
    for (int f = tid; f < nE; f += GNND_BLOCK) {
        int b = fdiv(f, dE), e = f - b * E;
        int j = (int)(s_evc[e] >> 16);
        T ex = is_qbp(VAR) ? extra[(b0 + b) * N + V + j] : T(0);
        const T gl = bp_lambda_grad<VAR, T>(s_aL[b * C + j] - s_L[f], s_ac[b * C + j] - s_c[f], ex, gg[f]);
        s_c[f] = gl;            // same thread read s_c[f] above: in-place is safe                           // sign indicator no longer needed
    }
    __syncthreads();
    for (int f = tid; f < nb * C; f += GNND_BLOCK) {
        int b = fdiv(f, dNode), j = f - b * C;
        T a = T(0);
        for (int k = s_cptr[j], ke = s_cptr[j + 1]; k < ke; ++k) a += s_c[b * E + s_cedge[k]];
        s_aL[f] = a;
    }
    __syncthreads();
    T* og = gmsg + b0 * E;
    for (int f = tid; f < nE; f += GNND_BLOCK) {
        int b = fdiv(f, dE), e = f - b * E;
        int j = (int)(s_evc[e] >> 16);
        BpFwd<VAR, T> fw;
        fw.init(mg[f]);
        og[f] = fw.input_grad(mg[f], s_aL[b * C + j] - s_c[f]);
    }
}

template <int VAR, typename T>
int launch_tiled_bp_bwd(const gnnd_graph* gr, const void* msg, const void* extra, const void* gout,
                        void* gmsg, int64_t B, hipStream_t st) {
    const GraphView& g = gr->view;
    const size_t tab = ((size_t)graph_table_ints(g.V, g.C, g.E) * 4 + 15) & ~(size_t)15;
    const size_t per = sizeof(T) * (2 * (size_t)g.E + 2 * (size_t)g.C);
    if (tab + per > 160 * 1024) return GNND_ERR_UNSUPPORTED;
    size_t cw = tab + per >= kLdsTarget ? 1 : (kLdsTarget - tab) / per;
    if (cw > 64) cw = 64;
    size_t lds = tab + cw * per;
    auto kern = propagate_tiled_bp_bwd_kernel<VAR, T>;
    if (lds > 64 * 1024)
        GNND_HIP_CHECK(hipFuncSetAttribute((const void*)kern,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    int64_t blocks = (B + (int64_t)cw - 1) / (int64_t)cw;
    if (blocks > 0x7fffffff) return GNND_ERR_UNSUPPORTED;
    kern<<<(unsigned)blocks, GNND_BLOCK, lds, st>>>(g, (const T*)msg, (const T*)extra, (const T*)gout,
                                                     (T*)gmsg, B, (int)cw, make_fastdiv(g.C),
                                                     make_fastdiv(g.E));
    GNND_LAUNCH_CHECK();
    return GNND_OK;
}

// generic (any edge_index) BP backward: three edge passes with atomic node sums.
// workspace: L[nE], c/g_Lambda[nE], S(L)[dim], S(c)[dim], S(g_Lambda)[dim]
template <int VAR, typename T>
__global__ void __launch_bounds__(GNND_BLOCK)
gen_bp_bwd_a(const int64_t* __restrict__ idx, const T* __restrict__ msg, int64_t nE, int64_t dim,
             T* L, T* c, T* aL, T* ac) {
    int64_t e = (int64_t)blockIdx.x * GNND_BLOCK + threadIdx.x;
    if (e >= nE) return;
    BpFwd<VAR, T> fw;
    fw.init(msg[e]);
    L[e] = fw.L;
    c[e] = fw.c;
    int64_t j = idx[e];
    if (j < 0 || j >= dim) return;
    atomicAdd(aL + j, fw.L);
    atomicAdd(ac + j, fw.c);
}
template <int VAR, typename T>
__global__ void __launch_bounds__(GNND_BLOCK)
gen_bp_bwd_b(const int64_t* __restrict__ idx, const T* __restrict__ extra, const T* __restrict__ gout,
             int64_t nE, int64_t dim, const T* L, T* c, const T* aL, const T* ac, T* ag) {
    int64_t e = (int64_t)blockIdx.x * GNND_BLOCK + threadIdx.x;
    if (e >= nE) return;
    int64_t j = idx[e];
    if (j < 0 || j >= dim) { c[e] = T(NAN); return; }
    T ex = is_qbp(VAR) ? extra[j] : T(0);
    T gl = bp_lambda_grad<VAR, T>(aL[j] - L[e], ac[j] - c[e], ex, gout[e]);
    c[e] = gl;
    atomicAdd(ag + j, gl);
}
template <int VAR, typename T>
__global__ void __launch_bounds__(GNND_BLOCK)
gen_bp_bwd_c(const int64_t* __restrict__ idx, const T* __restrict__ msg, int64_t nE, int64_t dim,
             const T* gl, const T* ag, T* __restrict__ gmsg) {
    int64_t e = (int64_t)blockIdx.x * GNND_BLOCK + threadIdx.x;
    if (e >= nE) return;
    int64_t j = idx[e];
    if (j < 0 || j >= dim) { gmsg[e] = T(NAN); return; }
    BpFwd<VAR, T> fw;
    fw.init(msg[e]);
    gmsg[e] = fw.input_grad(msg[e], ag[j] - gl[e]);
}

int64_t gen_bwd_ws_elems(bool bp, int64_t nE, int64_t dim) {
    return bp ? 2 * nE + 3 * dim : dim;
}

template <int VAR, typename T>
int launch_generic_bp_bwd(const int64_t* ei, int64_t stride, int64_t nE, const void* msg,
                          const void* extra, const void* gout, int64_t dim, void* gmsg, void* ws,
                          int64_t ws_bytes, hipStream_t st) {
    if (ws_bytes < gen_bwd_ws_elems(true, nE, dim) * (int64_t)sizeof(T)) return GNND_ERR_INVALID_ARG;
    T* w = (T*)ws;
    T *L = w, *c = w + nE, *aL = w + 2 * nE, *ac = aL + dim, *ag = ac + dim;
    const int64_t* idx = ei + stride;                       // target_to_source: edge_index[1]
    if (dim > 0) {
        fill_kernel<T><<<(unsigned)((3 * dim + GNND_BLOCK - 1) / GNND_BLOCK), GNND_BLOCK, 0, st>>>(aL, 3 * dim, T(0));
        GNND_LAUNCH_CHECK();
    }
    if (nE == 0) return GNND_OK;
    const unsigned gE = (unsigned)((nE + GNND_BLOCK - 1) / GNND_BLOCK);
    gen_bp_bwd_a<VAR, T><<<gE, GNND_BLOCK, 0, st>>>(idx, (const T*)msg, nE, dim, L, c, aL, ac);
    gen_bp_bwd_b<VAR, T><<<gE, GNND_BLOCK, 0, st>>>(idx, (const T*)extra, (const T*)gout, nE, dim, L, c, aL, ac, ag);
    gen_bp_bwd_c<VAR, T><<<gE, GNND_BLOCK, 0, st>>>(idx, (const T*)msg, nE, dim, c, ag, (T*)gmsg);
    GNND_LAUNCH_CHECK();
    return GNND_OK;
}

template <int VAR, int FLOW, typename T>
int launch_tiled_bwd(const gnnd_graph* gr, const void* msg, const void* gout, void* gmsg,
                     int64_t B, hipStream_t st) {
    const GraphView& g = gr->view;
    const int NJ = FLOW == GNND_SOURCE_TO_TARGET ? g.V : g.C;
    const size_t tab = ((size_t)graph_table_ints(g.V, g.C, g.E) * 4 + 15) & ~(size_t)15;
    const size_t per = sizeof(T) * ((size_t)g.E + NJ);
    if (tab + per > 160 * 1024) return GNND_ERR_UNSUPPORTED;
    size_t cw = tab + per >= kLdsTarget ? 1 : (kLdsTarget - tab) / per;
    if (cw > 64) cw = 64;
    size_t lds = tab + cw * per;
    auto kern = propagate_tiled_bwd_kernel<VAR, FLOW, T>;
    if (lds > 64 * 1024)
        GNND_HIP_CHECK(hipFuncSetAttribute((const void*)kern,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    int64_t blocks = (B + (int64_t)cw - 1) / (int64_t)cw;
    if (blocks > 0x7fffffff) return GNND_ERR_UNSUPPORTED;
    kern<<<(unsigned)blocks, GNND_BLOCK, lds, st>>>(g, (const T*)msg, (const T*)gout, (T*)gmsg, B,
                                                     (int)cw, make_fastdiv(NJ), make_fastdiv(g.E));
    GNND_LAUNCH_CHECK();
    return GNND_OK;
}

template <int VAR, int FLOW, typename T>
__global__ void __launch_bounds__(GNND_BLOCK)
gen_bwd_scatter_kernel(const int64_t* __restrict__ idx, const T* __restrict__ gout, int64_t nE,
                       int64_t dim, T* acc) {
    constexpr int F = out_width(VAR, FLOW);
    int64_t e = (int64_t)blockIdx.x * GNND_BLOCK + threadIdx.x;
    if (e >= nE) return;
    int64_t j = idx[e];
    if (j < 0 || j >= dim) return;
    atomicAdd(acc + j, gout[e * F]);
}

template <int VAR, int FLOW, typename T>
__global__ void __launch_bounds__(GNND_BLOCK)
gen_bwd_out_kernel(const int64_t* __restrict__ idx, const T* __restrict__ msg,
                   const T* __restrict__ gout, int64_t nE, int64_t dim, const T* acc,
                   T* __restrict__ gmsg) {
    constexpr int F = out_width(VAR, FLOW);
    int64_t e = (int64_t)blockIdx.x * GNND_BLOCK + threadIdx.x;
    if (e >= nE) return;
    int64_t j = idx[e];
    gmsg[e] = (j < 0 || j >= dim) ? T(NAN) : pre_grad<VAR, FLOW, T>(msg[e], acc[j] - gout[e * F]);
}

template <int VAR, int FLOW, typename T>
int launch_generic_bwd(const int64_t* ei, int64_t stride, int64_t nE, const void* msg,
                       const void* gout, int64_t dim, void* gmsg, void* ws, int64_t ws_bytes,
                       hipStream_t st) {
    if (ws_bytes < dim * (int64_t)sizeof(T)) return GNND_ERR_INVALID_ARG;
    T* acc = (T*)ws;
    const int64_t* idx = ei + (FLOW == GNND_SOURCE_TO_TARGET ? 0 : stride);
    if (dim > 0) {
        fill_kernel<T><<<(unsigned)((dim + GNND_BLOCK - 1) / GNND_BLOCK), GNND_BLOCK, 0, st>>>(acc, dim, T(0));
        GNND_LAUNCH_CHECK();
    }
    if (nE == 0) return GNND_OK;
    const unsigned gE = (unsigned)((nE + GNND_BLOCK - 1) / GNND_BLOCK);
    gen_bwd_scatter_kernel<VAR, FLOW, T><<<gE, GNND_BLOCK, 0, st>>>(idx, (const T*)gout, nE, dim, acc);
    gen_bwd_out_kernel<VAR, FLOW, T><<<gE, GNND_BLOCK, 0, st>>>(idx, (const T*)msg, (const T*)gout,
                                                               nE, dim, acc, (T*)gmsg);
    GNND_LAUNCH_CHECK();
    return GNND_OK;
}

template <int VAR, typename T>
int bwd_flow(bool tiled, int flow, const gnnd_graph* g, const int64_t* ei, int64_t stride,
             int64_t nE, const void* msg, const void* extra, const void* gout, int64_t dim,
             void* gmsg, void* ws, int64_t wb, int64_t B, hipStream_t st) {
    if (flow == GNND_SOURCE_TO_TARGET)
        return tiled ? launch_tiled_bwd<VAR, GNND_SOURCE_TO_TARGET, T>(g, msg, gout, gmsg, B, st)
                     : launch_generic_bwd<VAR, GNND_SOURCE_TO_TARGET, T>(ei, stride, nE, msg, gout, dim, gmsg, ws, wb, st);
    if constexpr (is_bp(VAR))
        return tiled ? launch_tiled_bp_bwd<VAR, T>(g, msg, extra, gout, gmsg, B, st)
                     : launch_generic_bp_bwd<VAR, T>(ei, stride, nE, msg, extra, gout, dim, gmsg, ws, wb, st);
    return tiled ? launch_tiled_bwd<VAR, GNND_TARGET_TO_SOURCE, T>(g, msg, gout, gmsg, B, st)
                 : launch_generic_bwd<VAR, GNND_TARGET_TO_SOURCE, T>(ei, stride, nE, msg, gout, dim, gmsg, ws, wb, st);
}

template <typename T>
int bwd_var(bool tiled, int var, int flow, const gnnd_graph* g, const int64_t* ei, int64_t stride,
            int64_t nE, const void* msg, const void* extra, const void* gout, int64_t dim,
            void* gmsg, void* ws, int64_t wb, int64_t B, hipStream_t st) {
#define GNND_BWD_CASE(V) \
    case V: return bwd_flow<V, T>(tiled, flow, g, ei, stride, nE, msg, extra, gout, dim, gmsg, ws, wb, B, st);
    switch (var) {
        GNND_BWD_CASE(GNND_V24)
        GNND_BWD_CASE(GNND_QGNNI)
        GNND_BWD_CASE(GNND_QBP)
        GNND_BWD_CASE(GNND_CGNNI)
        GNND_BWD_CASE(GNND_CBP)
        GNND_BWD_CASE(GNND_NBP)
        GNND_BWD_CASE(GNND_V10)
        GNND_BWD_CASE(GNND_V30)
    }
#undef GNND_BWD_CASE
    return GNND_ERR_INVALID_ARG;
}

bool bwd_needs_extra(int variant, int flow) {
    return is_qbp(variant) && flow == GNND_TARGET_TO_SOURCE;
}

}  // namespace

GNND_DEBUG_TU(propagate)

extern "C" int gnnd_propagate_width(int variant, int flow) {
    if (variant < GNND_V24 || variant > GNND_V30) return -1;
    if (flow != GNND_SOURCE_TO_TARGET && flow != GNND_TARGET_TO_SOURCE) return -1;
    return out_width(variant, flow);
}

extern "C" int gnnd_propagate_tiled(const gnnd_graph* g, int variant, int flow, int aggr,
                                    int dtype, const void* d_msg, const void* d_extra,
                                    void* d_out, int64_t batch, void* stream) {
    if (!g || !valid_common(variant, flow, aggr, dtype) || batch < 0) return GNND_ERR_INVALID_ARG;
    if (batch == 0) return GNND_OK;
    if (!d_msg || !d_out) return GNND_ERR_INVALID_ARG;
    if (!d_extra && variant != GNND_CGNNI) return GNND_ERR_INVALID_ARG;
    hipStream_t st = (hipStream_t)stream;
    if (dtype == GNND_F32) return tiled_var<float>(g, variant, flow, aggr, d_msg, d_extra, d_out, batch, st);
    return tiled_var<double>(g, variant, flow, aggr, d_msg, d_extra, d_out, batch, st);
}

extern "C" int gnnd_propagate_generic_workspace(int variant, int flow, int aggr, int dtype,
                                                int64_t nE, int64_t dim, int64_t* h_bytes) {
    if (!valid_common(variant, flow, aggr, dtype) || nE < 0 || dim < 0 || !h_bytes)
        return GNND_ERR_INVALID_ARG;
    bool bp = is_bp(variant) && flow == GNND_TARGET_TO_SOURCE;
    *h_bytes = gen_layout(bp, aggr, nE, dim).total * (dtype == GNND_F64 ? 8 : 4);
    return GNND_OK;
}

extern "C" int gnnd_propagate_generic(int variant, int flow, int aggr, int dtype,
                                      const int64_t* d_ei, int64_t row_stride, int64_t nE,
                                      const void* d_msg, const void* d_extra, int64_t dim,
                                      void* d_out, void* d_ws, int64_t ws_bytes, void* stream) {
    if (!valid_common(variant, flow, aggr, dtype) || nE < 0 || dim < 0 || row_stride < nE)
        return GNND_ERR_INVALID_ARG;
    if (nE > 0 && (!d_ei || !d_msg || !d_out)) return GNND_ERR_INVALID_ARG;
    if (!d_extra && variant != GNND_CGNNI) return GNND_ERR_INVALID_ARG;
    if (!d_ws && ws_bytes > 0) return GNND_ERR_INVALID_ARG;
    hipStream_t st = (hipStream_t)stream;
    if (dtype == GNND_F32)
        return gen_var<float>(variant, flow, aggr, d_ei, row_stride, nE, d_msg, d_extra, dim, d_out, d_ws, ws_bytes, st);
    return gen_var<double>(variant, flow, aggr, d_ei, row_stride, nE, d_msg, d_extra, dim, d_out, d_ws, ws_bytes, st);
}

extern "C" int gnnd_propagate_tiled_bwd(const gnnd_graph* g, int variant, int flow, int aggr,
                                        int dtype, const void* d_msg, const void* d_extra,
                                        const void* d_grad_out, void* d_grad_msg, int64_t batch,
                                        void* stream) {
    if (!g || !valid_common(variant, flow, aggr, dtype) || batch < 0) return GNND_ERR_INVALID_ARG;
    if (aggr != AG_ADD) return GNND_ERR_UNSUPPORTED;
    if (batch == 0) return GNND_OK;
    if (!d_msg || !d_grad_out || !d_grad_msg) return GNND_ERR_INVALID_ARG;
    if (!d_extra && bwd_needs_extra(variant, flow)) return GNND_ERR_INVALID_ARG;
    hipStream_t st = (hipStream_t)stream;
    if (dtype == GNND_F32)
        return bwd_var<float>(true, variant, flow, g, nullptr, 0, 0, d_msg, d_extra, d_grad_out, 0, d_grad_msg, nullptr, 0, batch, st);
    return bwd_var<double>(true, variant, flow, g, nullptr, 0, 0, d_msg, d_extra, d_grad_out, 0, d_grad_msg, nullptr, 0, batch, st);
}

extern "C" int gnnd_propagate_generic_bwd_workspace(int variant, int flow, int aggr, int dtype,
                                                    int64_t nE, int64_t dim, int64_t* h_bytes) {
    if (!valid_common(variant, flow, aggr, dtype) || nE < 0 || dim < 0 || !h_bytes)
        return GNND_ERR_INVALID_ARG;
    if (aggr != AG_ADD) return GNND_ERR_UNSUPPORTED;
    const bool bp = is_bp(variant) && flow == GNND_TARGET_TO_SOURCE;
    *h_bytes = gen_bwd_ws_elems(bp, nE, dim) * (dtype == GNND_F64 ? 8 : 4);
    return GNND_OK;
}

extern "C" int gnnd_propagate_generic_bwd(int variant, int flow, int aggr, int dtype,
                                          const int64_t* d_ei, int64_t row_stride, int64_t nE,
                                          const void* d_msg, const void* d_extra,
                                          const void* d_grad_out, int64_t dim, void* d_grad_msg,
                                          void* d_ws, int64_t ws_bytes, void* stream) {
    if (!valid_common(variant, flow, aggr, dtype) || nE < 0 || dim < 0 || row_stride < nE)
        return GNND_ERR_INVALID_ARG;
    if (aggr != AG_ADD) return GNND_ERR_UNSUPPORTED;
    if (nE > 0 && (!d_ei || !d_msg || !d_grad_out || !d_grad_msg)) return GNND_ERR_INVALID_ARG;
    if (nE > 0 && !d_extra && bwd_needs_extra(variant, flow)) return GNND_ERR_INVALID_ARG;
    if (!d_ws && dim > 0) return GNND_ERR_INVALID_ARG;
    hipStream_t st = (hipStream_t)stream;
    if (dtype == GNND_F32)
        return bwd_var<float>(false, variant, flow, nullptr, d_ei, row_stride, nE, d_msg, d_extra, d_grad_out, dim, d_grad_msg, d_ws, ws_bytes, 0, st);
    return bwd_var<double>(false, variant, flow, nullptr, d_ei, row_stride, nE, d_msg, d_extra, d_grad_out, dim, d_grad_msg, d_ws, ws_bytes, 0, st);
}
