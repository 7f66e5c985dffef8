// gnnd_train_gnn.hip — fused training of the 10-hidden-unit GNN decoders (paths relative to
// /root/reference/GNN-decode/):
//   CGNNI  classical/CGNNI.py:212-284 (GatedGraphConv + GNNI), trained by :314-338
//          (Adam lr 3e-4, weight decay 5e-4) on LossFunc :287-309; fp32, the script's dtype
//   QGNNI  quantum/QGNNI.py:186-252 (GraphConv + GNNI), trained by :294-320 on the logical
//          |sin| LossFunc :255-290; fp64, the script's dtype
// Per iteration t, on the check-group slot plan (gnnd_graph::view), messages m per edge:
//   a_e = (S_v(m) - m_e) + x_v              ggc1 (source_to_target, + post/extra)
//   t_e = tanh(a_e / 2)
//   u_e = S_c(t) - t_e                      ggc2 (target_to_source)
//   m'_e = MLP(u_e) [* s_c, QGNNI] + m_e    update() + the GNNI residual m_p
// readout r_v = S_v(m^T) + x_v, p_v = sigmoid(-MLP_o(r_v)) [CGNNI: clamp(., 1e-7, 1 - 1e-7)].
// MLP = Linear(1, 10) -> ReLU -> Linear(10, 1); packed weights (gnnd.h): {W1[10], b1[10],
// W2[10], b2} of the message MLP (CGNNI ggc2.mlp2, QGNNI ggc2.mlp), then the readout's.
//
// Forward with tape (one codeword at a time per workgroup, grid-strided): tape[b] = t^t per
// slot for t = 0 .. T-1, then r_v [V].  Variable sums in edge (index_add) order through vslot,
// check sums by the G-lane butterfly.  Reverse pass: d loss / d p -> readout backward (lanes
// over variables) -> d loss / d m^T per slot -> t = T-1 .. 0: the message MLP's backward per
// slot (u recomputed from the tape by the same butterfly), d t = S_c(d u) - d u, d a = d t
// (1 - t^2) / 2, d m^t = d m^{t+1} + S_v(d a) - d a.  The 62 weight gradients accumulate in
// each lane's registers over all slots, iterations and codewords and are summed in a fixed
// order at the end (wave butterfly, then the waves in order) into the workgroup's gradient
// row: deterministic; gnnd_train_update reduces the rows and runs Adam.
#include "gnnd_decode_impl.h"

GNND_DEBUG_TU(train_gnn)

namespace {

constexpr int kGnnThreads = GNND_BLOCK;
constexpr int kGnnW = 62;                 // trainable weights (gnnd.h CGNNI / QGNNI layout)

__host__ __device__ constexpr size_t gnn_a16(size_t n) { return (n + 15) & ~(size_t)15; }
// LDS: slot table, var_ptr, vslot (ints), then per codeword nslot + nslot + 2V + C values
template <typename T> __host__ __device__ constexpr size_t gnn_lds(int V, int C, int E, int nslot) {
    return gnn_a16(((size_t)nslot + V + 1 + E) * 4) + sizeof(T) * (2 * (size_t)nslot + 2 * (size_t)V + C);
}

template <typename T> __device__ __forceinline__ T relu0(T x) { return x > T(0) ? x : T(0); }

// y = sum_k W2_k relu(W1_k u + b1_k) + b2, in unit order (the reference Linear's dot product
// order up to rounding)
template <typename T> __device__ __forceinline__ T mlp10(const T* __restrict__ w, T u) {
    T acc = T(0);
#pragma unroll
    for (int k = 0; k < 10; ++k) acc = g_fma(relu0(g_fma(u, w[k], w[10 + k])), w[20 + k], acc);
    return acc + w[30];
}

// backward of mlp10 at input u for upstream dy: accumulates the 31 weight gradients into g,
// returns d y / d u times dy
template <typename T> __device__ __forceinline__ T mlp10_bwd(const T* __restrict__ w, T u, T dy, T (&g)[31]) {
    T du = T(0);
#pragma unroll
    for (int k = 0; k < 10; ++k) {
        const T h = g_fma(u, w[k], w[10 + k]);
        const bool on = h > T(0);                    // torch relu backward: grad where h > 0
        g[20 + k] = g_fma(dy, on ? h : T(0), g[20 + k]);
        const T dh = on ? dy * w[20 + k] : T(0);
        g[k] = g_fma(dh, u, g[k]);
        g[10 + k] += dh;
        du = g_fma(dh, w[k], du);
    }
    g[30] += dy;
    return du;
}

template <int MODEL, typename T>
__device__ __forceinline__ T readout_p(const T* __restrict__ w, T r, T& s) {
    s = sigmoid_ref(-mlp10(w + 31, r));
    if constexpr (MODEL == GNND_CGNNI) return g_clamp(s, cst<T>(1e-7), cst<T>(1 - 1e-7));
    else return s;
}

template <int MODEL, typename T, int R>
__global__ void __launch_bounds__(kGnnThreads)
gnn_train_fwd_kernel(GraphView g, const T* __restrict__ w, const T* __restrict__ x,
                     T* __restrict__ out, T* __restrict__ tape, int64_t B, int iters) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int V = g.V, C = g.C, E = g.E, N = g.N, G = g.G, logG = g.logG;
    const int tid = threadIdx.x;
    const int nslot = C * G * R, IC = C * G;
    uint32_t* s_slot = (uint32_t*)smem;
    int* s_vptr = (int*)(s_slot + nslot);
    int* s_vslot = s_vptr + V + 1;
    T* s_m = (T*)(smem + gnn_a16(((size_t)nslot + V + 1 + E) * 4));   // [nslot] messages
    T* s_t = s_m + nslot;                // [nslot] (unused in the forward)
    T* s_sv = s_t + nslot;               // [V] S_v(m)
    T* s_xv = s_sv + V;
    T* s_xc = s_xv + V;
    for (int i = tid; i < nslot; i += kGnnThreads) s_slot[i] = g.slot_ve[i];
    for (int i = tid; i <= V; i += kGnnThreads) s_vptr[i] = g.var_ptr[i];
    for (int i = tid; i < E; i += kGnnThreads) s_vslot[i] = g.vslot[i];
    const size_t tpb = (size_t)iters * nslot + V;          // tape values per codeword

    for (int64_t b = blockIdx.x; b < B; b += gridDim.x) {
        T* tp = tape + (size_t)b * tpb;
        __syncthreads();
        for (int i = tid; i < N; i += kGnnThreads) {
            const T xv = x[b * N + i];
            if (i < V) s_xv[i] = xv; else s_xc[i - V] = xv;
        }
        for (int i = tid; i < nslot; i += kGnnThreads) s_m[i] = T(0);
        for (int i = tid; i < V; i += kGnnThreads) s_sv[i] = T(0);
        __syncthreads();
        for (int it = 0; it < iters; ++it) {
            T* tt = tp + (size_t)it * nslot;
            for (int f0 = 0; f0 < IC; f0 += kGnnThreads) {
                const int f = f0 + tid;
                const bool act = f < IC;
                const int rem = act ? f : IC - 1;
                const int c = rem >> logG, s0 = rem * R;
                T tv[R], mr[R], tsum = T(0);
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const uint32_t sv = s_slot[s0 + r];
                    const int v = (int)(sv & 0xffffu);
                    const bool valid = (int)(sv >> 16) != E;
                    mr[r] = s_m[s0 + r];
                    const T a = (s_sv[v] - mr[r]) + s_xv[v];
                    const T th = g_tanh(a / T(2));
                    tv[r] = valid ? th : T(0);
                    if (act) tt[s0 + r] = tv[r];
                    tsum = r == 0 ? tv[0] : tsum + tv[r];
                }
                const T Sc = group_sum(tsum, G);
                const T sc = s_xc[c];
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    T y = mlp10(w, Sc - tv[r]);
                    if constexpr (MODEL == GNND_QGNNI) y = y * sc;
                    if (act) s_m[s0 + r] = y + mr[r];
                }
            }
            __syncthreads();
            for (int v = tid; v < V; v += kGnnThreads) {       // S_v in edge order
                T s = T(0);
                for (int k = s_vptr[v]; k < s_vptr[v + 1]; ++k) s += s_m[s_vslot[k]];
                s_sv[v] = s;
            }
            __syncthreads();
        }
        for (int v = tid; v < V; v += kGnnThreads) {
            const T r = s_sv[v] + s_xv[v];
            T s;
            tp[(size_t)iters * nslot + v] = r;
            out[b * V + v] = readout_p<MODEL>(w, r, s);
        }
    }
}

// reverse pass: d loss / d out -> one gradient row [62] per workgroup
template <int MODEL, typename T, int R>
__global__ void __launch_bounds__(kGnnThreads)
gnn_train_bwd_kernel(GraphView g, const T* __restrict__ w, const T* __restrict__ x,
                     const T* __restrict__ dout, const T* __restrict__ tape,
                     T* __restrict__ rows, int64_t B, int iters) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int V = g.V, C = g.C, E = g.E, N = g.N, G = g.G, logG = g.logG;
    const int tid = threadIdx.x;
    const int nslot = C * G * R, IC = C * G;
    uint32_t* s_slot = (uint32_t*)smem;
    int* s_vptr = (int*)(s_slot + nslot);
    int* s_vslot = s_vptr + V + 1;
    T* s_G = (T*)(smem + gnn_a16(((size_t)nslot + V + 1 + E) * 4));   // [nslot] d / d m^{t+1}
    T* s_ga = s_G + nslot;               // [nslot] d / d a_e
    T* s_gv = s_ga + nslot;              // [V] d / d r_v, then sum of d a over v's edges
    T* s_xv = s_gv + V;                  // (unused: x_v enters additively)
    T* s_xc = s_xv + V;
    for (int i = tid; i < nslot; i += kGnnThreads) s_slot[i] = g.slot_ve[i];
    for (int i = tid; i <= V; i += kGnnThreads) s_vptr[i] = g.var_ptr[i];
    for (int i = tid; i < E; i += kGnnThreads) s_vslot[i] = g.vslot[i];
    const size_t tpb = (size_t)iters * nslot + V;
    T gm[31], go[31];                    // message / readout MLP gradients of this lane
#pragma unroll
    for (int k = 0; k < 31; ++k) gm[k] = go[k] = T(0);

    for (int64_t b = blockIdx.x; b < B; b += gridDim.x) {
        const T* tp = tape + (size_t)b * tpb;
        __syncthreads();                 // the previous codeword is done with LDS
        for (int i = tid; i < C; i += kGnnThreads) s_xc[i] = x[b * N + V + i];
        // readout: p = [clamp] sigmoid(-z), z = MLP_o(r)
        for (int v = tid; v < V; v += kGnnThreads) {
            const T r = tp[(size_t)iters * nslot + v];
            T s;
            (void)readout_p<MODEL>(w, r, s);
            T dp = dout[b * V + v];
            if constexpr (MODEL == GNND_CGNNI)          // clamp: gradient inside [min, max]
                if (!(s >= cst<T>(1e-7) && s <= cst<T>(1 - 1e-7))) dp = T(0);
            const T dz = -((dp * s) * (T(1) - s));      // d sigmoid(-z) / d z = -s (1 - s)
            s_gv[v] = mlp10_bwd(w + 31, r, dz, go);
        }
        __syncthreads();
        for (int i = tid; i < nslot; i += kGnnThreads) {   // d / d m^T = d / d r of its variable
            const uint32_t sv = s_slot[i];
            s_G[i] = (int)(sv >> 16) != E ? s_gv[sv & 0xffffu] : T(0);
        }
        for (int t = iters - 1; t >= 0; --t) {
            __syncthreads();
            const T* tt = tp + (size_t)t * nslot;
            for (int f0 = 0; f0 < IC; f0 += kGnnThreads) {
                const int f = f0 + tid;
                const bool act = f < IC;
                const int rem = act ? f : IC - 1;
                const int c = rem >> logG, s0 = rem * R;
                T tv[R], tsum = T(0);
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    tv[r] = tt[s0 + r];                      // padding slots hold 0
                    tsum = r == 0 ? tv[0] : tsum + tv[r];
                }
                const T Sc = group_sum(tsum, G);
                const T sc = s_xc[c];
                T du[R], dsum = T(0);
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const bool valid = (int)(s_slot[s0 + r] >> 16) != E;
                    T dy = valid && act ? s_G[s0 + r] : T(0);
                    if constexpr (MODEL == GNND_QGNNI) dy = dy * sc;
                    du[r] = valid && act ? mlp10_bwd(w, Sc - tv[r], dy, gm) : T(0);
                    dsum = r == 0 ? du[0] : dsum + du[r];
                }
                const T Sd = group_sum(dsum, G);
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const T dt = Sd - du[r];
                    if (act) s_ga[s0 + r] = (dt * (T(1) - tv[r] * tv[r])) / T(2);
                }
            }
            __syncthreads();
            for (int v = tid; v < V; v += kGnnThreads) {
                T s = T(0);
                for (int k = s_vptr[v]; k < s_vptr[v + 1]; ++k) s += s_ga[s_vslot[k]];
                s_gv[v] = s;
            }
            __syncthreads();
            // a_e = (S_v(m) - m_e) + x_v:  d / d m_e += S_v(d a) - d a_e (residual kept)
            for (int i = tid; i < nslot; i += kGnnThreads) {
                const uint32_t sv = s_slot[i];
                if ((int)(sv >> 16) == E) continue;
                s_G[i] += s_gv[sv & 0xffffu] - s_ga[i];
            }
        }
    }
    // the row: every weight's lane partials summed by a fixed butterfly per wave, then the
    // waves in order
    __shared__ T s_red[kGnnThreads / 64][kGnnW];
    const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
    for (int k = 0; k < kGnnW; ++k) {
        T v = k < 31 ? gm[k] : go[k - 31];
        for (int o = 1; o < 64; o <<= 1) v += __shfl_xor(v, o);
        if (lane == 0) s_red[wave][k] = v;
    }
    __syncthreads();
    for (int k = tid; k < kGnnW; k += kGnnThreads) {
        T s = T(0);
        for (int q = 0; q < kGnnThreads / 64; ++q) s += s_red[q][k];
        rows[(size_t)blockIdx.x * kGnnW + k] = s;
    }
}

template <int MODEL, typename T, int R>
int launch_gnn(const gnnd_graph* gr, const void* w, const void* x, void* out, const void* dout,
               const void* tape, void* rows, int64_t rows_bytes, int64_t B, int iters,
               hipStream_t st, bool fwd) {
    const GraphView& g = gr->view;
    const int nslot = g.C * g.G * g.R;
    const int64_t blocks = gnnd_gnn_train_rows(B);
    const size_t lds = gnn_lds<T>(g.V, g.C, g.E, nslot);
    // dynamic LDS up to the CU's 160 KB (fp64 LDPC-648 needs ~76 KB) together with the reverse
    // pass's static s_red rows; above the 64 KB default the kernel's limit is raised first
    constexpr size_t kStaticBwd = sizeof(T) * (kGnnThreads / 64) * kGnnW;
    if (lds + (fwd ? 0 : kStaticBwd) > 160 * 1024) return GNND_ERR_UNSUPPORTED;
    if (fwd) {
        auto k = gnn_train_fwd_kernel<MODEL, T, R>;
        if (lds > 64 * 1024)
            GNND_HIP_CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        k<<<(unsigned)blocks, kGnnThreads, lds, st>>>(g, (const T*)w, (const T*)x, (T*)out, (T*)tape, B, iters);
    } else {
        if (blocks * kGnnW * (int64_t)sizeof(T) > rows_bytes) return GNND_ERR_INVALID_ARG;
        auto k = gnn_train_bwd_kernel<MODEL, T, R>;
        if (lds > 64 * 1024)
            GNND_HIP_CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        k<<<(unsigned)blocks, kGnnThreads, lds, st>>>(g, (const T*)w, (const T*)x, (const T*)dout,
                                                      (const T*)tape, (T*)rows, B, iters);
    }
    GNND_LAUNCH_CHECK();
    return GNND_OK;
}

template <int MODEL, typename T>
int launch_gnn_r(const gnnd_graph* gr, const void* w, const void* x, void* out, const void* dout,
                 const void* tape, void* rows, int64_t rows_bytes, int64_t B, int iters,
                 hipStream_t st, bool fwd) {
    switch (gr->view.R) {
        case 1: return launch_gnn<MODEL, T, 1>(gr, w, x, out, dout, tape, rows, rows_bytes, B, iters, st, fwd);
        case 2: return launch_gnn<MODEL, T, 2>(gr, w, x, out, dout, tape, rows, rows_bytes, B, iters, st, fwd);
        case 3: return launch_gnn<MODEL, T, 3>(gr, w, x, out, dout, tape, rows, rows_bytes, B, iters, st, fwd);
        case 4: return launch_gnn<MODEL, T, 4>(gr, w, x, out, dout, tape, rows, rows_bytes, B, iters, st, fwd);
    }
    return GNND_ERR_UNSUPPORTED;
}

int launch_gnn_m(const gnnd_graph* gr, int model, int dtype, const void* w, const void* x,
                 void* out, const void* dout, const void* tape, void* rows, int64_t rows_bytes,
                 int64_t B, int iters, hipStream_t st, bool fwd) {
    if (model == GNND_CGNNI)
        return dtype == GNND_F32
                   ? launch_gnn_r<GNND_CGNNI, float>(gr, w, x, out, dout, tape, rows, rows_bytes, B, iters, st, fwd)
                   : launch_gnn_r<GNND_CGNNI, double>(gr, w, x, out, dout, tape, rows, rows_bytes, B, iters, st, fwd);
    if (model == GNND_QGNNI)
        return dtype == GNND_F32
                   ? launch_gnn_r<GNND_QGNNI, float>(gr, w, x, out, dout, tape, rows, rows_bytes, B, iters, st, fwd)
                   : launch_gnn_r<GNND_QGNNI, double>(gr, w, x, out, dout, tape, rows, rows_bytes, B, iters, st, fwd);
    return GNND_ERR_UNSUPPORTED;
}

}  // namespace

int64_t gnnd_gnn_tape_elems(const gnnd_graph* g, int64_t B, int iters) {
    return B * ((int64_t)iters * g->view.C * g->view.G * g->view.R + g->view.V);
}
int64_t gnnd_gnn_train_rows(int64_t B) { return B < 1024 ? B : 1024; }
int gnnd_launch_gnn_tape(const gnnd_graph* g, int model, int dtype, const void* w, const void* x,
                         void* out, int64_t B, int iters, void* tape, hipStream_t st) {
    if (!tape) return GNND_ERR_INVALID_ARG;
    return launch_gnn_m(g, model, dtype, w, x, out, nullptr, tape, nullptr, 0, B, iters, st, true);
}
int gnnd_launch_gnn_bwd(const gnnd_graph* g, int model, int dtype, const void* w, const void* x,
                        const void* dout, const void* tape, void* rows, int64_t rows_bytes,
                        int64_t B, int iters, hipStream_t st) {
    return launch_gnn_m(g, model, dtype, w, x, nullptr, dout, tape, rows, rows_bytes, B, iters, st, false);
}
