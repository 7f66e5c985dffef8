// gnnd_decode.hip — fused T-iteration GNN / BP decoder (one launch per batch).
//
// Restates GNNI.forward of the five reference decoders (paths relative to
// /root/reference/GNN-decode/):
//   CGNNI  classical/CGNNI.py:259-284   (fp32; c->v MLP 1->10->1 ReLU; residual; node MLP)
//   CBP    classical/BP.py:239-259      (fp32; log-domain sum-product, no weights)
//   QBP    quantum/BP.py:199-219        (fp64; syndrome-aware log-domain BP)
//   QGNNI  quantum/QGNNI.py:228-252     (fp64; c->v MLP 1->10->1 ReLU x syndrome; residual)
//   V24    quantum/decoder_v2_4.py:272-294 (fp64 reference; v->c MLP 2->128->1 Softplus,
//          c->v MLP 1->128->1 Softplus x syndrome, residual, per-edge readout MLP)
//
// MI355X mapping.  Every codeword has the same Tanner graph, so the graph tables are
// staged once per workgroup into LDS and each workgroup decodes a tile of CW codewords
// whose per-edge messages live in LDS for all T iterations: HBM is touched only to read
// x (N values per codeword) and write the V outputs.  One iteration is four phases
// separated by workgroup barriers:
//   A  variable sums   S_v = sum_{e in v} m_e          (thread per (cw, v), edge order)
//   B  v->c edge op    a_e = (S_v - m_e) + x_v ; t_e = pre(a_e)       (thread per (cw, e))
//   C  check sums      S_c = sum_{e in c} t_e          (thread per (cw, c), edge order)
//   D  c->v edge op    m_e = update(S_c - t_e, s_c) + m_prev          (thread per (cw, e))
// The node sums run in the reference's accumulation order (index_add in edge order from
// 0), so the leave-one-out values match torch_scatter's bit for bit; only the MLP dot
// products and transcendentals differ at the ulp level.
#include "gnnd_common.h"

namespace {

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

// ---------------------------------------------------------------------------------------
// per-edge MLPs (torch.nn.Linear y = x W^T + b), weights uniform across lanes -> SGPRs
// ---------------------------------------------------------------------------------------
// Linear(1,10) -> ReLU -> Linear(10,1); w = {W1[10], b1[10], W2[10], b2}
template <typename T>
__device__ __forceinline__ T mlp10_relu(const T* __restrict__ w, T u) {
    T acc = T(0);
#pragma unroll
    for (int k = 0; k < 10; ++k) {
        T h = g_fma(u, w[k], w[10 + k]);
        acc = g_fma(g_max(h, T(0)), w[20 + k], acc);
    }
    return acc + w[30];
}

// Linear(1,128) -> Softplus -> Linear(128,1); w = {W1[128], b1[128], W2[128], b2}
__device__ __forceinline__ double mlp128_sp(const double* __restrict__ w, double u) {
    double acc = 0.0;
#pragma unroll 8
    for (int k = 0; k < 128; ++k) {
        double h = fma(u, w[k], w[128 + k]);
        acc = fma(softplus_ref(h), w[256 + k], acc);
    }
    return acc + w[384];
}
// fp32 prepared weights: W1, b1 pre-scaled by log2(e), W2 by ln(2)
__device__ __forceinline__ float mlp128_sp(const float* __restrict__ w, float u) {
    float acc = 0.f;
#pragma unroll 16
    for (int k = 0; k < 128; ++k) {
        float hs = fmaf(u, w[k], w[128 + k]);
        acc = fmaf(softplus2_fast(hs), w[256 + k], acc);
    }
    return acc + w[384];
}

// Linear(2,128) -> Softplus -> Linear(128,1); w = {W1[:,0][128], W1[:,1][128], b1[128], W2[128], b2}
__device__ __forceinline__ double mlp128x2_sp(const double* __restrict__ w, double u0, double u1) {
    double acc = 0.0;
#pragma unroll 8
    for (int k = 0; k < 128; ++k) {
        double h = fma(u0, w[k], fma(u1, w[128 + k], w[256 + k]));
        acc = fma(softplus_ref(h), w[384 + k], acc);
    }
    return acc + w[512];
}
__device__ __forceinline__ float mlp128x2_sp(const float* __restrict__ w, float u0, float u1) {
    float acc = 0.f;
#pragma unroll 16
    for (int k = 0; k < 128; ++k) {
        float hs = fmaf(u0, w[k], fmaf(u1, w[128 + k], w[256 + k]));
        acc = fmaf(softplus2_fast(hs), w[384 + k], acc);
    }
    return acc + w[512];
}

// weight offsets in the packed layout (gnnd.h)
constexpr int kV24Ggc1 = 0, kV24Ggc2 = 513, kV24Mlp = 898;
constexpr int kMlp10Msg = 0, kMlp10Out = 31;

template <int MODEL> struct ModelTraits {
    static constexpr bool bp = (MODEL == GNND_QBP || MODEL == GNND_CBP);
};

// torch constants are Python doubles converted to the tensor dtype
template <typename T> __device__ __forceinline__ T cst(double v) { return (T)v; }

// ---------------------------------------------------------------------------------------
// the fused kernel
// ---------------------------------------------------------------------------------------
template <int MODEL, typename T>
__global__ void __launch_bounds__(GNND_BLOCK)
decode_kernel(GraphView g, const T* __restrict__ w, const T* __restrict__ x,
              T* __restrict__ out, int64_t B, int iters, int CW, FastDiv dV, FastDiv dC,
              FastDiv dE) {
    constexpr bool BP = ModelTraits<MODEL>::bp;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int V = g.V, C = g.C, E = g.E, N = g.N;
    const int tid = threadIdx.x;

    // ---- LDS carve: graph tables, then per-codeword state
    int* s_tab = (int*)smem;
    const int nints = graph_table_ints(V, C, E);
    const uint32_t* s_evc = (const uint32_t*)s_tab;
    const int* s_vptr = s_tab + E;
    const int* s_cptr = s_vptr + V + 1;
    const int* s_cedge = s_cptr + C + 1;
    size_t off = ((size_t)nints * 4 + 15) & ~(size_t)15;
    T* s_m = (T*)(smem + off);          // [CW][E] messages m (c->v, persistent)
    T* s_t = s_m + (size_t)CW * E;      // [CW][E] v->c quantity after pre-op
    T* s_t2 = s_t + (size_t)CW * E;     // [CW][E] BP only: sign indicator
    T* s_x = s_t2 + (BP ? (size_t)CW * E : 0);   // [CW][N] node features
    T* s_vs = s_x + (size_t)CW * N;     // [CW][V] variable sums
    T* s_cs = s_vs + (size_t)CW * V;    // [CW][C] check sums
    T* s_cs2 = s_cs + (size_t)CW * C;   // [CW][C] BP only: sign-count sums

    const int* gtab = (const int*)g.edge_vc;
    for (int i = tid; i < nints; i += GNND_BLOCK) s_tab[i] = gtab[i];

    const int64_t b0 = (int64_t)blockIdx.x * CW;
    const int nb = (int)((B - b0) < CW ? (B - b0) : CW);
    const T* xg = x + b0 * N;
    for (int i = tid; i < nb * N; i += GNND_BLOCK) s_x[i] = xg[i];
    for (int i = tid; i < nb * E; i += GNND_BLOCK) s_m[i] = T(0);
    __syncthreads();

    const int nV = nb * V, nC = nb * C, nE = nb * E;
    for (int it = 0; it < iters; ++it) {
        // A: variable sums (index_add order)
        for (int f = tid; f < nV; f += GNND_BLOCK) {
            int b = fdiv(f, dV), v = f - b * V;
            const T* mb = s_m + b * E;
            T s = T(0);
            for (int k = s_vptr[v], ke = s_vptr[v + 1]; k < ke; ++k) s += mb[k];
            s_vs[f] = s;
        }
        __syncthreads();
        // B: v->c edge op and c->v pre-op
        for (int f = tid; f < nE; f += GNND_BLOCK) {
            int b = fdiv(f, dE), e = f - b * E;
            int v = (int)(s_evc[e] & 0xffffu);
            T mv = s_m[f];
            T ext = s_vs[b * V + v] - mv;
            T xv = s_x[b * N + v];
            if constexpr (MODEL == GNND_V24) {
                T a = mlp128x2_sp(w + kV24Ggc1, ext, xv);
                s_t[f] = g_tanh(a / T(2));
            } else if constexpr (BP) {
                T a = ext + xv;
                T t = g_tanh(g_clamp(a, T(-10), T(10)) / T(2));
                s_t2[f] = t < T(0) ? T(1) : T(0);
                const T lo = MODEL == GNND_QBP ? cst<T>(1e-20) : cst<T>(1e-7);
                s_t[f] = g_log(g_clamp(g_abs(t), lo, cst<T>(1e10)));
            } else {   // CGNNI, QGNNI: a = ext + x ; tanh(a/2)
                T a = ext + xv;
                s_t[f] = g_tanh(a / T(2));
            }
        }
        __syncthreads();
        // C: check sums
        for (int f = tid; f < nC; f += GNND_BLOCK) {
            int b = fdiv(f, dC), c = f - b * C;
            const T* tb = s_t + b * E;
            T s = T(0), s2 = T(0);
            for (int k = s_cptr[c], ke = s_cptr[c + 1]; k < ke; ++k) {
                int e = s_cedge[k];
                s += tb[e];
                if constexpr (BP) s2 += s_t2[b * E + e];
            }
            s_cs[f] = s;
            if constexpr (BP) s_cs2[f] = s2;
        }
        __syncthreads();
        // D: c->v edge op (+ residual)
        for (int f = tid; f < nE; f += GNND_BLOCK) {
            int b = fdiv(f, dE), e = f - b * E;
            int c = (int)(s_evc[e] >> 16);
            T u = s_cs[b * C + c] - s_t[f];
            T sc = s_x[b * N + V + c];
            T mn;
            if constexpr (MODEL == GNND_V24) {
                mn = mlp128_sp(w + kV24Ggc2, u) * sc + s_m[f];
            } else if constexpr (MODEL == GNND_QGNNI) {
                mn = mlp10_relu(w + kMlp10Msg, u) * sc + s_m[f];
            } else if constexpr (MODEL == GNND_CGNNI) {
                mn = mlp10_relu(w + kMlp10Msg, u) + s_m[f];
            } else {   // BP: u = Lambda (sum of log|t| leave-one-out)
                T n = s_cs2[b * C + c] - s_t2[f];
                if constexpr (MODEL == GNND_QBP) n = n + (T(1) - sc) / T(2);
                const T hi = MODEL == GNND_QBP ? cst<T>(1 - 1e-12) : cst<T>(1 - 1e-7);
                T p = g_clamp(g_exp(u) * cos_pi(n), -hi, hi);
                if constexpr (MODEL == GNND_QBP)
                    mn = g_log(T(1) + p) - g_log(T(1) - p);
                else
                    mn = g_log((T(1) + p) / (T(1) - p));
            }
            s_m[f] = mn;
        }
        __syncthreads();
    }

    // ---- readout
    T* og = out + b0 * V;
    if constexpr (MODEL == GNND_V24) {
        // per-edge MLP_o(m_e) then variable sums (decoder_v2_4.py:291-292)
        for (int f = tid; f < nE; f += GNND_BLOCK) s_t[f] = mlp128_sp(w + kV24Mlp, s_m[f]);
        __syncthreads();
    }
    for (int f = tid; f < nV; f += GNND_BLOCK) {
        int b = fdiv(f, dV), v = f - b * V;
        const T* mb = (MODEL == GNND_V24 ? s_t : s_m) + b * E;
        T s = T(0);
        for (int k = s_vptr[v], ke = s_vptr[v + 1]; k < ke; ++k) s += mb[k];
        T r = s + s_x[b * N + v];
        T o;
        if constexpr (MODEL == GNND_CGNNI) {
            o = g_clamp(sigmoid_ref(-mlp10_relu(w + kMlp10Out, r)), cst<T>(1e-7), cst<T>(1 - 1e-7));
        } else if constexpr (MODEL == GNND_QGNNI) {
            o = sigmoid_ref(-mlp10_relu(w + kMlp10Out, r));
        } else if constexpr (MODEL == GNND_CBP) {
            o = g_clamp(sigmoid_ref(-r), cst<T>(1e-7), cst<T>(1 - 1e-7));
        } else {   // QBP, V24
            o = sigmoid_ref(-r);
        }
        og[f] = o;
    }
}

// ---------------------------------------------------------------------------------------
template <typename T>
__global__ void prepare_v24_f32_kernel(const T* __restrict__ in, T* __restrict__ outw) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= 1283) return;
    T v = in[i];
    // ggc1: [0,384) layer 1 (W1a, W1b, b1), [384,512) W2, 512 b2
    // ggc2 / mlp: [+0,+256) layer 1 (W1, b1), [+256,+384) W2, +384 b2
    int seg, loc;
    if (i < kV24Ggc2) { seg = 0; loc = i; }
    else if (i < kV24Mlp) { seg = 1; loc = i - kV24Ggc2; }
    else { seg = 2; loc = i - kV24Mlp; }
    int l1 = seg == 0 ? 384 : 256, l2 = seg == 0 ? 512 : 384;
    if (loc < l1) v = v * (T)kLog2e;
    else if (loc < l2) v = v * (T)kLn2;
    outw[i] = v;
}

int weights_count(int model) {
    switch (model) {
        case GNND_CGNNI: case GNND_QGNNI: return 62;
        case GNND_V24: return 1283;
        case GNND_CBP: case GNND_QBP: return 0;
        default: return -1;
    }
}

size_t state_elems_per_cw(int model, const GraphView& g) {
    const bool bp = model == GNND_CBP || model == GNND_QBP;
    return (size_t)g.E * (bp ? 3 : 2) + g.N + g.V + (size_t)g.C * (bp ? 2 : 1);
}

constexpr size_t kLdsTarget = 40 * 1024;     // ~4 workgroups (16 waves) per CU
constexpr size_t kLdsMax = 160 * 1024;

int choose_tile(int model, int dtype, const GraphView& g, int* cw, size_t* lds) {
    const size_t esz = dtype == GNND_F64 ? 8 : 4;
    const size_t tab = ((size_t)graph_table_ints(g.V, g.C, g.E) * 4 + 15) & ~(size_t)15;
    const size_t per = state_elems_per_cw(model, g) * esz;
    if (tab + per > kLdsMax) return GNND_ERR_UNSUPPORTED;
    size_t n = tab + per >= kLdsTarget ? 1 : (kLdsTarget - tab) / per;
    if (n > 64) n = 64;
    *cw = (int)n;
    *lds = tab + n * per;
    return GNND_OK;
}

template <int MODEL, typename T>
int launch_decode(const gnnd_graph* gr, const void* w, const void* x, void* out, int64_t B,
                  int iters, hipStream_t st) {
    const GraphView& g = gr->view;
    int cw;
    size_t lds;
    int rc = choose_tile(MODEL, sizeof(T) == 8 ? GNND_F64 : GNND_F32, g, &cw, &lds);
    if (rc != GNND_OK) return rc;
    auto kern = decode_kernel<MODEL, T>;
    if (lds > 64 * 1024)
        GNND_HIP_CHECK(hipFuncSetAttribute((const void*)kern,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    int64_t blocks = (B + cw - 1) / cw;
    if (blocks > 0x7fffffff) return GNND_ERR_UNSUPPORTED;
    kern<<<(unsigned)blocks, GNND_BLOCK, lds, st>>>(
        g, (const T*)w, (const T*)x, (T*)out, B, iters, cw, make_fastdiv(g.V), make_fastdiv(g.C),
        make_fastdiv(g.E));
    GNND_LAUNCH_CHECK();
    return GNND_OK;
}

template <typename T>
int dispatch_decode(const gnnd_graph* g, int model, const void* w, const void* x, void* out,
                    int64_t B, int iters, hipStream_t st) {
    switch (model) {
        case GNND_V24: return launch_decode<GNND_V24, T>(g, w, x, out, B, iters, st);
        case GNND_QGNNI: return launch_decode<GNND_QGNNI, T>(g, w, x, out, B, iters, st);
        case GNND_QBP: return launch_decode<GNND_QBP, T>(g, w, x, out, B, iters, st);
        case GNND_CGNNI: return launch_decode<GNND_CGNNI, T>(g, w, x, out, B, iters, st);
        case GNND_CBP: return launch_decode<GNND_CBP, T>(g, w, x, out, B, iters, st);
        default: return GNND_ERR_INVALID_ARG;
    }
}

}  // namespace

extern "C" int gnnd_weights_count(int model, int64_t* h_count) {
    int n = weights_count(model);
    if (n < 0 || !h_count) return GNND_ERR_INVALID_ARG;
    *h_count = n;
    return GNND_OK;
}

extern "C" int gnnd_prepare_weights(int model, int dtype, const void* d_w, void* d_prepared,
                                    void* stream) {
    int n = weights_count(model);
    if (n < 0 || (dtype != GNND_F32 && dtype != GNND_F64)) return GNND_ERR_INVALID_ARG;
    if (n == 0) return GNND_OK;
    if (!d_w || !d_prepared) return GNND_ERR_INVALID_ARG;
    hipStream_t st = (hipStream_t)stream;
    if (model == GNND_V24 && dtype == GNND_F32) {
        prepare_v24_f32_kernel<float><<<(1283 + 255) / 256, 256, 0, st>>>(
            (const float*)d_w, (float*)d_prepared);
        GNND_LAUNCH_CHECK();
        return GNND_OK;
    }
    size_t bytes = (size_t)n * (dtype == GNND_F64 ? 8 : 4);
    if (d_w != d_prepared)
        GNND_HIP_CHECK(hipMemcpyAsync(d_prepared, d_w, bytes, hipMemcpyDeviceToDevice, st));
    return GNND_OK;
}

extern "C" int gnnd_decode_tile(const gnnd_graph* g, int model, int dtype, int32_t* h_cw,
                                int32_t* h_lds) {
    if (!g || !h_cw || !h_lds || weights_count(model) < 0) return GNND_ERR_INVALID_ARG;
    if (dtype != GNND_F32 && dtype != GNND_F64) return GNND_ERR_INVALID_ARG;
    int cw;
    size_t lds;
    int rc = choose_tile(model, dtype, g->view, &cw, &lds);
    if (rc != GNND_OK) return rc;
    *h_cw = cw;
    *h_lds = (int32_t)lds;
    return GNND_OK;
}

extern "C" int gnnd_decode(const gnnd_graph* g, int model, int dtype, const void* d_w,
                           const void* d_x, void* d_out, int64_t batch, int32_t iters,
                           void* stream) {
    int nw = weights_count(model);
    if (!g || nw < 0 || batch < 0 || iters < 0 || !d_x || !d_out) return GNND_ERR_INVALID_ARG;
    if (nw > 0 && !d_w) return GNND_ERR_INVALID_ARG;
    if (batch == 0) return GNND_OK;
    if ((int64_t)batch * g->view.N > 0x7fffffffLL * 64) return GNND_ERR_UNSUPPORTED;
    hipStream_t st = (hipStream_t)stream;
    if (dtype == GNND_F32) return dispatch_decode<float>(g, model, d_w, d_x, d_out, batch, iters, st);
    if (dtype == GNND_F64) return dispatch_decode<double>(g, model, d_w, d_x, d_out, batch, iters, st);
    return GNND_ERR_INVALID_ARG;
}
