// gnnd_decode_v30.hip — fused decoder for the GRU edge-state GNN of quantum/decoder_v3_0.py
// (paths relative to /root/reference/GNN-decode/).
//
// GNNI.forward (:256-290) keeps one state m_e per edge and, for T iterations, updates it
// twice (GraphConv.forward :219-231 with the propagate body :106-118, no pre-op):
//   ggc1 (variable side):  mes = mlp1([S_v(m) - m_e, x_v]),  m_e <- GRU1(input m_e, hidden mes)
//   [last iteration: m_p = m]
//   ggc2 (check side):     mes = mlp2([S_c(m) - m_e, x_c]),  m_e <- GRU2(input m_e, hidden mes)
// mlp1/mlp2 = Linear(2,10) -> ReLU -> Linear(10,1), GRUk = torch.nn.GRUCell(1, 1) (gates
// r, z, n; h' = (h - n) z + n), all fp64 in the reference.  Readout (:274-288), two outputs
// over every node of the batch:
//   out0 = sigmoid(-(mlp(S_v(m)) + x))   (check rows: mlp(0) + x_c)
//   out1 = sigmoid(-mlp(S_c(m_p)))       (variable rows: mlp(0))
//
// MI355X mapping: the streaming layout of decode_kernel (gnnd_decode_impl.h) — a workgroup
// decodes a tile of codewords whose edge states live in LDS for all T iterations (slot
// order: G lanes x R slots per check).  Both half-steps of an iteration run in ONE pass
// over the check groups: the variable-side update needs S_v (from the previous variable-sum
// pass) and the edge's own state, so each lane updates its R edges on the variable side,
// sums the new states over the check with the G-lane butterfly (group_sum) and applies the
// check-side update in registers; one barrier-separated variable-sum pass then refreshes
// S_v.  The check sum of the last iteration's variable-side states IS S_c(m_p), so out1 is
// written from the same registers.  HBM traffic per codeword: N values in, 2N out.
#include "gnnd_decode_impl.h"

namespace {

constexpr int kV30Mlp1 = 0, kV30Rnn1 = 41, kV30Mlp2 = 53, kV30Rnn2 = 94, kV30Out = 106;

// Linear(2,10) -> ReLU -> Linear(10,1); w = {W1[10][2], b1[10], W2[10], b2} (torch.nn.Linear:
// y = x W^T + b)
template <typename T>
__device__ __forceinline__ T v30_mlp(const T* w, T a, T c) {
    T acc = T(0);
#pragma unroll
    for (int k = 0; k < 10; ++k) {
        const T h = g_fma(c, w[2 * k + 1], g_fma(a, w[2 * k], w[20 + k]));
        acc = g_fma(fmax(h, T(0)), w[30 + k], acc);
    }
    return acc + w[40];
}

// torch.nn.GRUCell(1, 1)(input xin, hidden h); w = {w_ih[3], w_hh[3], b_ih[3], b_hh[3]}
// (ATen gru_cell: r = sig(h_r + i_r), z = sig(h_z + i_z), n = tanh(i_n + r h_n),
// h' = (h - n) z + n)
template <typename T>
__device__ __forceinline__ T v30_gru(const T* w, T xin, T h) {
    const T ir = g_fma(xin, w[0], w[6]), iz = g_fma(xin, w[1], w[7]), in = g_fma(xin, w[2], w[8]);
    const T hr = g_fma(h, w[3], w[9]), hz = g_fma(h, w[4], w[10]), hn = g_fma(h, w[5], w[11]);
    const T r = sigmoid_ref(hr + ir);
    const T z = sigmoid_ref(hz + iz);
    const T n = g_tanh(in + r * hn);
    return (h - n) * z + n;
}

template <typename T, int R>
__global__ void __launch_bounds__(GNND_BLOCK)
decode_v30_kernel(GraphView g, const T* __restrict__ w, const T* __restrict__ x,
                  T* __restrict__ out, int64_t B, int iters, int CW, FastDiv dItem, FastDiv dV,
                  FastDiv dN) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int V = g.V, C = g.C, E = g.E, N = g.N, G = g.G, logG = g.logG;
    const int tid = threadIdx.x;

    T* s_w = (T*)smem;
    size_t off = ((size_t)kV30Count * sizeof(T) + 15) & ~(size_t)15;
    const int nslot = C * G * R;
    uint32_t* s_slot = (uint32_t*)(smem + off);
    int* s_vptr = (int*)(s_slot + nslot);
    int* s_vslot = s_vptr + V + 1;
    off += (((size_t)nslot + V + 1 + E) * 4 + 15) & ~(size_t)15;
    T* s_m = (T*)(smem + off);                             // [CW][nslot] edge states
    SumX<T>* s_sx = (SumX<T>*)(s_m + (size_t)CW * nslot);  // [CW][V]  {S_v, x_v}
    T* s_xc = (T*)(s_sx + (size_t)CW * V);                 // [CW][C]  check-row features

    for (int i = tid; i < kV30Count; i += GNND_BLOCK) s_w[i] = w[i];
    for (int i = tid; i < nslot; i += GNND_BLOCK) s_slot[i] = g.slot_ve[i];   // v | e << 16
    for (int i = tid; i <= V; i += GNND_BLOCK) s_vptr[i] = g.var_ptr[i];
    for (int i = tid; i < E; i += GNND_BLOCK) s_vslot[i] = g.vslot[i];
    const int64_t b0 = (int64_t)blockIdx.x * CW;
    const int nb = (int)((B - b0) < CW ? (B - b0) : CW);
    const T* xg = x + b0 * N;
    for (int i = tid; i < nb * N; i += GNND_BLOCK) {
        const int b = fdiv(i, dN), n = i - b * N;
        const T xv = xg[i];
        if (n < V) s_sx[b * V + n] = SumX<T>{T(0), xv};
        else s_xc[b * C + n - V] = xv;
    }
    for (int i = tid; i < nb * nslot; i += GNND_BLOCK) s_m[i] = T(0);
    __syncthreads();

    const T* w_mlp1 = s_w + kV30Mlp1;
    const T* w_rnn1 = s_w + kV30Rnn1;
    const T* w_mlp2 = s_w + kV30Mlp2;
    const T* w_rnn2 = s_w + kV30Rnn2;
    const T* w_out = s_w + kV30Out;
    T* out0 = out + b0 * N;                 // [B*N] sigmoid(-(mlp(S_v) + x))
    T* out1 = out + B * N + b0 * N;         // [B*N] sigmoid(-mlp(S_c(m_p)))

    const int IC = C * G;
    const int nItem = nb * IC;
    const int nV = nb * V;
    for (int it = 0; it < iters; ++it) {
        const bool last = it + 1 == iters;
        for (int f0 = 0; f0 < nItem; f0 += GNND_BLOCK) {
            const int f = f0 + tid;
            const bool act = f < nItem;
            const int fc = act ? f : nItem - 1;          // idle lanes compute on a copy
            const int b = fdiv(fc, dItem);
            const int rem = fc - b * IC;
            const int c = rem >> logG;
            const uint32_t* sl = s_slot + rem * R;
            T* mb = s_m + b * nslot + rem * R;
            const SumX<T>* sxb = s_sx + b * V;
            T m1[R];
            T tsum = T(0);
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const uint32_t sv = sl[r];
                const bool valid = (int)(sv >> 16) != E;
                const SumX<T> p = sxb[GNND_DIDX((int)(sv & 0xffffu), V, GNND_DBG_VAR)];   // padding: variable 0
                const T me = mb[r];
                m1[r] = v30_gru(w_rnn1, me, v30_mlp(w_mlp1, p.s - me, p.x));
                tsum += valid ? m1[r] : T(0);
            }
            const T Sc = group_sum(tsum, G);             // S_c of the variable-side states
            if (last && act && (rem & (G - 1)) == 0)
                out1[b * N + V + c] = sigmoid_ref(-mlp10_relu(w_out, Sc));
            const T xc = s_xc[b * C + c];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const T mn = v30_gru(w_rnn2, m1[r], v30_mlp(w_mlp2, Sc - m1[r], xc));
                if (act) mb[r] = mn;                     // padding slots are never summed
            }
        }
        __syncthreads();
        if (last) break;
        for (int f = tid; f < nV; f += GNND_BLOCK) {
            const int b = fdiv(f, dV), v = f - b * V;
            s_sx[f].s = var_sum(s_m + b * nslot, s_vslot, s_vptr[v], s_vptr[v + 1], nslot);
        }
        __syncthreads();
    }

    // readout over every node of the tile
    const T y0 = mlp10_relu(w_out, T(0));
    for (int f = tid; f < nb * N; f += GNND_BLOCK) {
        const int b = fdiv(f, dN), n = f - b * N;
        if (n < V) {
            const T s = iters > 0 ? var_sum(s_m + b * nslot, s_vslot, s_vptr[n], s_vptr[n + 1]) : T(0);
            out0[f] = sigmoid_ref(-(mlp10_relu(w_out, s) + s_sx[b * V + n].x));
            out1[f] = sigmoid_ref(-y0);
        } else {
            out0[f] = sigmoid_ref(-(y0 + s_xc[b * C + n - V]));
            if (iters == 0) out1[f] = sigmoid_ref(-y0);   // m_p = 0 (T = 0)
        }
    }
}

template <typename T, int R>
int launch_v30(const Plan& p, const void* w, const void* x, void* out, int64_t B, int iters,
               hipStream_t st) {
    const GraphView& g = *p.view;
    const int64_t blocks = (B + p.cw - 1) / p.cw;
    if (blocks > 0x7fffffff) return GNND_ERR_UNSUPPORTED;
    auto kern = decode_v30_kernel<T, R>;
    if (p.lds > 64 * 1024)
        GNND_HIP_CHECK(hipFuncSetAttribute((const void*)kern,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)p.lds));
    kern<<<(unsigned)blocks, GNND_BLOCK, p.lds, st>>>(g, (const T*)w, (const T*)x, (T*)out, B, iters,
                                                      p.cw, make_fastdiv(g.C * g.G),
                                                      make_fastdiv(g.V), make_fastdiv(g.N));
    GNND_LAUNCH_CHECK();
    return GNND_OK;
}

template <typename T>
int launch_v30_r(const gnnd_graph* gr, const void* w, const void* x, void* out, int64_t B,
                 int iters, hipStream_t st) {
    Plan p;
    const int rc = make_plan(GNND_V30, sizeof(T) == 8 ? GNND_F64 : GNND_F32, gr, &p, B);
    if (rc != GNND_OK) return rc;
    if (p.resident) return GNND_ERR_UNSUPPORTED;
    switch (p.view->R) {
        case 1: return launch_v30<T, 1>(p, w, x, out, B, iters, st);
        case 2: return launch_v30<T, 2>(p, w, x, out, B, iters, st);
        case 3: return launch_v30<T, 3>(p, w, x, out, B, iters, st);
        case 4: return launch_v30<T, 4>(p, w, x, out, B, iters, st);
    }
    return GNND_ERR_UNSUPPORTED;
}

}  // namespace

GNND_DEBUG_TU(decode_v30)

int gnnd_launch_v30(const gnnd_graph* g, int dtype, const void* w, const void* x, void* out,
                    int64_t B, int iters, hipStream_t st) {
    if (dtype == GNND_F32) return launch_v30_r<float>(g, w, x, out, B, iters, st);
    return launch_v30_r<double>(g, w, x, out, B, iters, st);
}
