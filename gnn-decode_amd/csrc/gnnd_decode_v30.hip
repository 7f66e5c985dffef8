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

// TAPE (training, gnnd_train_fwd): per codeword, iteration t < T and slot (slot order of the
// plan's view), tape[b][t][0][slot] = m (the state entering ggc1) and tape[b][t][1][slot] = m1
// (after ggc1); tape[b][T][0][slot] = the final states.  Padding slots are recorded too.
template <typename T, int R, bool TAPE = false>
__global__ void __launch_bounds__(GNND_BLOCK)
decode_v30_kernel(GraphView g, const T* __restrict__ w, const T* __restrict__ x,
                  T* __restrict__ out, int64_t B, int iters, int CW, FastDiv dItem, FastDiv dV,
                  FastDiv dN, T* __restrict__ tape = nullptr) {
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
            T* tp = nullptr;
            if constexpr (TAPE) tp = tape + ((b0 + b) * (iters + 1) + it) * 2 * nslot + rem * R;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const uint32_t sv = sl[r];
                const bool valid = (int)(sv >> 16) != E;
                const SumX<T> p = sxb[GNND_DIDX((int)(sv & 0xffffu), V, GNND_DBG_VAR)];   // padding: variable 0
                const T me = mb[r];
                m1[r] = v30_gru(w_rnn1, me, v30_mlp(w_mlp1, p.s - me, p.x));
                tsum += valid ? m1[r] : T(0);
                if constexpr (TAPE) if (act) { tp[r] = me; tp[nslot + r] = m1[r]; }
            }
            const T Sc = group_sum(tsum, G);             // S_c of the variable-side states
            if (last && act && (rem & (G - 1)) == 0)
                out1[b * N + V + c] = sigmoid_ref(-mlp10_relu(w_out, Sc));
            const T xc = s_xc[b * C + c];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const T mn = v30_gru(w_rnn2, m1[r], v30_mlp(w_mlp2, Sc - m1[r], xc));
                if (act) mb[r] = mn;                     // padding slots are never summed
                if constexpr (TAPE) if (act && last) tp[2 * nslot + r] = mn;   // tape[b][T][0]
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


// ---------------------------------------------------------------------------------------
// reverse pass of the training step (gnnd_train_bwd*, model V30): d loss / d (the 137 packed
// weights) from d loss / d out [2][B*N] and the forward's tape.  Reverse mode of the forward
// above, iteration t = T-1 .. 0, with G = d loss / d (the states leaving iteration t):
//   ggc2  mn = GRU2(m1, mes2), mes2 = mlp2(a2, x_c), a2 = S_c(m1) - m1
//         -> g_m1 = g_in(GRU2) - g_a2 + sum_{check} g_a2 (+ the out1 readout at t = T-1)
//   ggc1  m1 = GRU1(m, mes1), mes1 = mlp1(a1, x_v), a1 = S_v(m) - m
//         -> G' = g_in(GRU1) - g_a1 + sum_{variable} g_a1
// The readout (out0 = sigmoid(-(mlp(S_v(m^T)) + x)), out1 = sigmoid(-mlp(S_c(m_p)))) seeds G
// and the check sums' adjoint; torch's rules throughout (sigmoid' = y (1 - y), tanh' =
// 1 - y^2, ReLU' = [h > 0]).  One codeword at a time per workgroup (grid-strided): the
// edge phases run on the forward's check-group slot layout (check sums by the same lane
// butterfly, so S_c is recomputed bit-identically), the variable sums gather through vslot
// in edge order; the weight gradients are PARAMETER-parallel: each edge phase leaves per-slot
// records in LDS and wave w accumulates one parameter group over all slots in its lanes'
// registers (w0 ggc1.mlp1, w1 ggc2.mlp2, w2 both GRUs, w3 the readout mlp), summed over the
// wave's lanes at the end in a fixed butterfly -> one gradient row per workgroup.
// ---------------------------------------------------------------------------------------
constexpr int kV30Rec = 18;   // per-slot records: mlp1 {a1, x_v, g}, mlp2 {a2, x_c, g},
                              // GRU1 {m, mes1, g_r, g_z, g_n, g_hn}, GRU2 {m1, mes2, ...}

template <typename T> struct GruGrad { T gx, gh, gr, gz, gn, ghn; };
// torch.nn.GRUCell(1, 1) backward at (input xin, hidden h) for d loss / d h' = g: gates
// recomputed as v30_gru does; gr / gz / gn = d loss / d (the r, z, n gate pre-activations),
// ghn = d loss / d (h w_hh_n + b_hh_n)
template <typename T>
__device__ __forceinline__ GruGrad<T> v30_gru_bwd(const T* w, T xin, T h, T g) {
    const T ir = g_fma(xin, w[0], w[6]), iz = g_fma(xin, w[1], w[7]), in = g_fma(xin, w[2], w[8]);
    const T hr = g_fma(h, w[3], w[9]), hz = g_fma(h, w[4], w[10]), hn = g_fma(h, w[5], w[11]);
    const T r = sigmoid_ref(hr + ir);
    const T z = sigmoid_ref(hz + iz);
    const T n = g_tanh(in + r * hn);
    GruGrad<T> o;
    o.gn = (g * (T(1) - z)) * (T(1) - n * n);
    o.ghn = o.gn * r;
    o.gr = (o.gn * hn) * ((T(1) - r) * r);
    o.gz = (g * (h - n)) * ((T(1) - z) * z);
    o.gx = o.gr * w[0] + o.gz * w[1] + o.gn * w[2];
    o.gh = g * z + o.gr * w[3] + o.gz * w[4] + o.ghn * w[5];
    return o;
}
// {w_ih[3], w_hh[3], b_ih[3], b_hh[3]} gradients of one GRU application
template <typename T>
__device__ __forceinline__ void v30_gru_acc(T xin, T h, T gr, T gz, T gn, T ghn, T* acc) {
    acc[0] = g_fma(gr, xin, acc[0]); acc[1] = g_fma(gz, xin, acc[1]); acc[2] = g_fma(gn, xin, acc[2]);
    acc[3] = g_fma(gr, h, acc[3]);   acc[4] = g_fma(gz, h, acc[4]);   acc[5] = g_fma(ghn, h, acc[5]);
    acc[6] += gr; acc[7] += gz; acc[8] += gn;
    acc[9] += gr; acc[10] += gz; acc[11] += ghn;
}
// d mlp(a, c) / d a times g (the same pre-activations as v30_mlp)
template <typename T>
__device__ __forceinline__ T v30_mlp_gin(const T* w, T a, T c, T g) {
    T ga = T(0);
#pragma unroll
    for (int k = 0; k < 10; ++k) {
        const T h = g_fma(c, w[2 * k + 1], g_fma(a, w[2 * k], w[20 + k]));
        ga = g_fma(h > T(0) ? g * w[30 + k] : T(0), w[2 * k], ga);
    }
    return ga;
}
// {W1[10][2], b1[10], W2[10], b2} gradients of one mlp application with output gradient g
template <typename T>
__device__ __forceinline__ void v30_mlp_acc(const T* w, T a, T c, T g, T* acc) {
#pragma unroll
    for (int k = 0; k < 10; ++k) {
        const T h = g_fma(c, w[2 * k + 1], g_fma(a, w[2 * k], w[20 + k]));
        const T gp = h > T(0) ? g * w[30 + k] : T(0);
        acc[2 * k] = g_fma(gp, a, acc[2 * k]);
        acc[2 * k + 1] = g_fma(gp, c, acc[2 * k + 1]);
        acc[20 + k] += gp;
        acc[30 + k] = g_fma(g, fmax(h, T(0)), acc[30 + k]);
    }
    acc[40] += g;
}
// readout Linear(1,10) -> ReLU -> Linear(10,1), w = {W1[10], b1[10], W2[10], b2}
template <typename T>
__device__ __forceinline__ T mlp10_gin(const T* w, T s, T g) {
    T gs = T(0);
#pragma unroll
    for (int k = 0; k < 10; ++k) {
        const T h = g_fma(s, w[k], w[10 + k]);
        gs = g_fma(h > T(0) ? g * w[20 + k] : T(0), w[k], gs);
    }
    return gs;
}
template <typename T>
__device__ __forceinline__ void mlp10_acc(const T* w, T s, T g, T* acc) {
#pragma unroll
    for (int k = 0; k < 10; ++k) {
        const T h = g_fma(s, w[k], w[10 + k]);
        const T gp = h > T(0) ? g * w[20 + k] : T(0);
        acc[k] = g_fma(gp, s, acc[k]);
        acc[10 + k] += gp;
        acc[20 + k] = g_fma(g, fmax(h, T(0)), acc[20 + k]);
    }
    acc[30] += g;
}
// d loss / d (the readout mlp's output) of one output row: o = sigmoid(-z), dz = -(d o) o (1 - o)
template <typename T> __device__ __forceinline__ T sig_neg_bwd(T o, T d) { return -((d * (T(1) - o)) * o); }

__host__ __device__ constexpr size_t v30_a16(size_t n) { return (n + 15) & ~(size_t)15; }
// reverse-pass LDS: weights, graph tables, [3][nslot] states / adjoints / g_a1, [3][V] S_v,
// sum g_a1, x_v, [C] x_c, [2N][2] readout rows, [kV30Rec][nslot] records
__host__ __device__ constexpr size_t v30_bwd_lds(int V, int C, int E, int N, int nslot, size_t esz) {
    return v30_a16((size_t)kV30Count * esz) + v30_a16(((size_t)nslot + V + 1 + E) * 4) +
           esz * (3 * (size_t)nslot + 3 * (size_t)V + C + 4 * (size_t)N + (size_t)kV30Rec * nslot);
}

template <typename T, int R>
__global__ void __launch_bounds__(GNND_BLOCK)
v30_bwd_kernel(GraphView g, const T* __restrict__ w, const T* __restrict__ x,
               const T* __restrict__ out, const T* __restrict__ dout, const T* __restrict__ tape,
               T* __restrict__ rows, int64_t B, int iters) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int V = g.V, C = g.C, E = g.E, N = g.N, G = g.G, logG = g.logG;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int nslot = C * G * R, IC = C * G;
    T* s_w = (T*)smem;
    size_t off = v30_a16((size_t)kV30Count * sizeof(T));
    uint32_t* s_slot = (uint32_t*)(smem + off);
    int* s_vptr = (int*)(s_slot + nslot);
    int* s_vslot = s_vptr + V + 1;
    off += v30_a16(((size_t)nslot + V + 1 + E) * 4);
    T* s_m = (T*)(smem + off);      // [nslot] tape states m_t (final states first)
    T* s_G = s_m + nslot;           // [nslot] adjoint of the states leaving the iteration
    T* s_gx = s_G + nslot;          // [nslot] g_a1 (variable-summed)
    T* s_sv = s_gx + nslot;         // [V] S_v(m_t)
    T* s_gs = s_sv + V;             // [V] sum of g_a1 over the variable's edges
    T* s_xv = s_gs + V;             // [V]
    T* s_xc = s_xv + V;             // [C]
    T* s_ro = s_xc + C;             // [2N][2] readout rows {mlp input, d/d mlp output}
    T* s_rec = s_ro + 4 * (size_t)N;   // [kV30Rec][nslot]

    for (int i = tid; i < kV30Count; i += GNND_BLOCK) s_w[i] = w[i];
    for (int i = tid; i < nslot; i += GNND_BLOCK) s_slot[i] = g.slot_ve[i];
    for (int i = tid; i <= V; i += GNND_BLOCK) s_vptr[i] = g.var_ptr[i];
    for (int i = tid; i < E; i += GNND_BLOCK) s_vslot[i] = g.vslot[i];
    const T* w_mlp1 = s_w + kV30Mlp1;
    const T* w_rnn1 = s_w + kV30Rnn1;
    const T* w_mlp2 = s_w + kV30Mlp2;
    const T* w_rnn2 = s_w + kV30Rnn2;
    const T* w_out = s_w + kV30Out;

    constexpr int kAcc = 41;
    T acc[kAcc];                    // this lane's partials of its wave's parameter group
#pragma unroll
    for (int k = 0; k < kAcc; ++k) acc[k] = T(0);
    const T* out0 = out;
    const T* out1 = out + B * N;
    const T* d0 = dout;
    const T* d1 = dout + B * N;
    const size_t tstride = 2 * (size_t)nslot;

    for (int64_t b = blockIdx.x; b < B; b += gridDim.x) {
        const T* tp = tape + (size_t)b * (iters + 1) * tstride;
        const int64_t rb = b * N;
        __syncthreads();            // the previous codeword's phases are done with LDS
        for (int i = tid; i < N; i += GNND_BLOCK) {
            const T xv = x[rb + i];
            if (i < V) s_xv[i] = xv; else s_xc[i - V] = xv;
        }
        for (int i = tid; i < nslot; i += GNND_BLOCK) s_m[i] = tp[(size_t)iters * tstride + i];
        __syncthreads();
        // readout rows: out0 variable rows (mlp(S_v(m^T)) + x_v) seed the final states'
        // adjoint; out0 check rows and out1 variable rows read mlp(0); out1 check rows
        // (mlp(S_c(m_p))) are recorded by the t = T-1 edge phase
        for (int i = tid; i < 2 * N; i += GNND_BLOCK) {
            const int n = i < N ? i : i - N;
            const T o = i < N ? out0[rb + n] : out1[rb + n];
            const T d = i < N ? d0[rb + n] : d1[rb + n];
            const T gz = sig_neg_bwd(o, d);
            T s = T(0);
            if (i < V && iters > 0) {
                s = var_sum(s_m, s_vslot, s_vptr[i], s_vptr[i + 1]);
                s_gs[i] = mlp10_gin(w_out, s, gz);
            } else if (i < V) {
                s_gs[i] = T(0);
            }
            s_ro[2 * i] = s;
            s_ro[2 * i + 1] = gz;
        }
        __syncthreads();
        for (int i = tid; i < nslot; i += GNND_BLOCK) {
            const uint32_t sv = s_slot[i];
            s_G[i] = (int)(sv >> 16) != E ? s_gs[sv & 0xffffu] : T(0);
        }
        if (iters == 0 && wv == 3)
            for (int i = lane; i < 2 * N; i += 64) mlp10_acc(w_out, s_ro[2 * i], s_ro[2 * i + 1], acc);
        for (int t = iters - 1; t >= 0; --t) {
            const T* tm = tp + (size_t)t * tstride;      // m_t, then m1_t
            __syncthreads();                            // s_G of the previous step
            for (int i = tid; i < nslot; i += GNND_BLOCK) s_m[i] = tm[i];
            __syncthreads();
            for (int v = tid; v < V; v += GNND_BLOCK)
                s_sv[v] = var_sum(s_m, s_vslot, s_vptr[v], s_vptr[v + 1], nslot);
            __syncthreads();
            // edge phase on the forward's check-group layout (whole waves per round: the
            // check butterflies need every lane of the group)
            for (int f0 = 0; f0 < IC; f0 += GNND_BLOCK) {
                const int f = f0 + tid;
                const bool act = f < IC;
                const int rem = act ? f : IC - 1;
                const int c = rem >> logG;
                const int s0 = rem * R;
                T m1[R];
                bool valid[R];
                T tsum = T(0);
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    valid[r] = (int)(s_slot[s0 + r] >> 16) != E;
                    m1[r] = tm[nslot + s0 + r];
                    tsum += valid[r] ? m1[r] : T(0);
                }
                const T Sc = group_sum(tsum, G);         // the forward's S_c, same order
                const T xc = s_xc[c];
                T dSc = T(0);
                if (t == iters - 1) {                    // out1 check row: mlp(S_c(m_p))
                    const T gz = s_ro[2 * (N + V + c) + 1];
                    dSc = mlp10_gin(w_out, Sc, gz);
                    if (act && (rem & (G - 1)) == 0) s_ro[2 * (N + V + c)] = Sc;
                }
                T a2[R], ga2[R], gsum = T(0);
                GruGrad<T> g2[R];
                T mes2[R], Gv[R];
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    Gv[r] = s_G[s0 + r];
                    a2[r] = Sc - m1[r];
                    mes2[r] = v30_mlp(w_mlp2, a2[r], xc);
                    g2[r] = v30_gru_bwd(w_rnn2, m1[r], mes2[r], Gv[r]);
                    ga2[r] = v30_mlp_gin(w_mlp2, a2[r], xc, g2[r].gh);
                    gsum += valid[r] ? ga2[r] : T(0);
                }
                const T Sga = group_sum(gsum, G);
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int sl = s0 + r;
                    const uint32_t sv = s_slot[sl];
                    const int v = (int)(sv & 0xffffu);
                    const T gm1 = valid[r] ? (g2[r].gx - ga2[r]) + Sga + dSc : T(0);
                    const T m = s_m[sl];
                    const T a1 = s_sv[v] - m, xv = s_xv[v];
                    const T mes1 = v30_mlp(w_mlp1, a1, xv);
                    const GruGrad<T> g1 = v30_gru_bwd(w_rnn1, m, mes1, gm1);
                    const T ga1 = v30_mlp_gin(w_mlp1, a1, xv, g1.gh);
                    if (act) {
                        const bool ok = valid[r];
                        T* rc = s_rec + sl;
                        rc[0 * nslot] = a1; rc[1 * nslot] = xv; rc[2 * nslot] = ok ? g1.gh : T(0);
                        rc[3 * nslot] = a2[r]; rc[4 * nslot] = xc; rc[5 * nslot] = ok ? g2[r].gh : T(0);
                        rc[6 * nslot] = m; rc[7 * nslot] = mes1;
                        rc[8 * nslot] = ok ? g1.gr : T(0); rc[9 * nslot] = ok ? g1.gz : T(0);
                        rc[10 * nslot] = ok ? g1.gn : T(0); rc[11 * nslot] = ok ? g1.ghn : T(0);
                        rc[12 * nslot] = m1[r]; rc[13 * nslot] = mes2[r];
                        rc[14 * nslot] = ok ? g2[r].gr : T(0); rc[15 * nslot] = ok ? g2[r].gz : T(0);
                        rc[16 * nslot] = ok ? g2[r].gn : T(0); rc[17 * nslot] = ok ? g2[r].ghn : T(0);
                        s_gx[sl] = ok ? ga1 : T(0);
                        s_G[sl] = ok ? g1.gx - ga1 : T(0);
                    }
                }
            }
            __syncthreads();
            // variable sums of g_a1; the weight gradients of this iteration (parameter-parallel)
            for (int v = tid; v < V; v += GNND_BLOCK)
                s_gs[v] = var_sum(s_gx, s_vslot, s_vptr[v], s_vptr[v + 1], nslot);
            for (int i = lane; i < nslot; i += 64) {
                if ((int)(s_slot[i] >> 16) == E) continue;
                const T* rc = s_rec + i;
                if (wv == 0) {
                    v30_mlp_acc(w_mlp1, rc[0], rc[nslot], rc[2 * nslot], acc);
                } else if (wv == 1) {
                    v30_mlp_acc(w_mlp2, rc[3 * nslot], rc[4 * nslot], rc[5 * nslot], acc);
                } else if (wv == 2) {
                    v30_gru_acc(rc[6 * nslot], rc[7 * nslot], rc[8 * nslot], rc[9 * nslot],
                                rc[10 * nslot], rc[11 * nslot], acc);
                    v30_gru_acc(rc[12 * nslot], rc[13 * nslot], rc[14 * nslot], rc[15 * nslot],
                                rc[16 * nslot], rc[17 * nslot], acc + 12);
                }
            }
            if (t == iters - 1 && wv == 3)
                for (int i = lane; i < 2 * N; i += 64) mlp10_acc(w_out, s_ro[2 * i], s_ro[2 * i + 1], acc);
            __syncthreads();
            for (int i = tid; i < nslot; i += GNND_BLOCK) {
                const uint32_t sv = s_slot[i];
                if ((int)(sv >> 16) != E) s_G[i] += s_gs[sv & 0xffffu];
            }
        }
    }
    // one gradient row per workgroup: each wave's parameter group summed over its lanes
    // (fixed xor butterfly), written in the packed layout
    const int n = wv == 0 ? 41 : wv == 1 ? 41 : wv == 2 ? 24 : 31;
    T* row = rows + (size_t)blockIdx.x * kV30Count;
#pragma unroll
    for (int k = 0; k < kAcc; ++k) {
        T v = acc[k];
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) v += __shfl_xor(v, o);
        if (lane == 0 && k < n) {
            const int dst = wv == 0 ? kV30Mlp1 + k : wv == 1 ? kV30Mlp2 + k
                            : wv == 2 ? (k < 12 ? kV30Rnn1 + k : kV30Rnn2 + k - 12) : kV30Out + k;
            row[dst] = v;
        }
    }
}

template <typename T, int R>
int launch_v30(const Plan& p, const void* w, const void* x, void* out, int64_t B, int iters,
               hipStream_t st, void* tape = nullptr) {
    const GraphView& g = *p.view;
    const int64_t blocks = (B + p.cw - 1) / p.cw;
    if (blocks > 0x7fffffff) return GNND_ERR_UNSUPPORTED;
    auto kern = tape ? decode_v30_kernel<T, R, true> : decode_v30_kernel<T, R, false>;
    if (p.lds > 64 * 1024)
        GNND_HIP_CHECK(hipFuncSetAttribute((const void*)kern,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)p.lds));
    kern<<<(unsigned)blocks, GNND_BLOCK, p.lds, st>>>(g, (const T*)w, (const T*)x, (T*)out, B, iters,
                                                      p.cw, make_fastdiv(g.C * g.G),
                                                      make_fastdiv(g.V), make_fastdiv(g.N), (T*)tape);
    GNND_LAUNCH_CHECK();
    return GNND_OK;
}

template <typename T>
int launch_v30_r(const gnnd_graph* gr, const void* w, const void* x, void* out, int64_t B,
                 int iters, hipStream_t st, void* tape = nullptr) {
    Plan p;
    const int rc = make_plan(GNND_V30, sizeof(T) == 8 ? GNND_F64 : GNND_F32, gr, &p, B);
    if (rc != GNND_OK) return rc;
    if (p.resident || (tape && p.view != &gr->view)) return GNND_ERR_UNSUPPORTED;
    switch (p.view->R) {
        case 1: return launch_v30<T, 1>(p, w, x, out, B, iters, st, tape);
        case 2: return launch_v30<T, 2>(p, w, x, out, B, iters, st, tape);
        case 3: return launch_v30<T, 3>(p, w, x, out, B, iters, st, tape);
        case 4: return launch_v30<T, 4>(p, w, x, out, B, iters, st, tape);
    }
    return GNND_ERR_UNSUPPORTED;
}

template <typename T, int R>
int launch_v30_bwd(const gnnd_graph* gr, const void* w, const void* x, const void* out,
                   const void* dout, const void* tape, void* rows, int64_t rows_bytes, int64_t B,
                   int iters, hipStream_t st) {
    const GraphView& g = gr->view;            // the tape's slot layout (launch_v30_r)
    const int nslot = g.C * g.G * g.R;
    const int64_t blocks = gnnd_v30_train_rows(B);
    if (blocks * kV30Count * (int64_t)sizeof(T) > rows_bytes) return GNND_ERR_INVALID_ARG;
    const size_t lds = v30_bwd_lds(g.V, g.C, g.E, g.N, nslot, sizeof(T));
    if (lds > 160 * 1024) return GNND_ERR_UNSUPPORTED;
    auto kern = v30_bwd_kernel<T, R>;
    if (lds > 64 * 1024)
        GNND_HIP_CHECK(hipFuncSetAttribute((const void*)kern,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    kern<<<(unsigned)blocks, GNND_BLOCK, lds, st>>>(g, (const T*)w, (const T*)x, (const T*)out,
                                                    (const T*)dout, (const T*)tape, (T*)rows, B, iters);
    GNND_LAUNCH_CHECK();
    return GNND_OK;
}

template <typename T>
int launch_v30_bwd_r(const gnnd_graph* gr, const void* w, const void* x, const void* out,
                     const void* dout, const void* tape, void* rows, int64_t rows_bytes, int64_t B,
                     int iters, hipStream_t st) {
    switch (gr->view.R) {
        case 1: return launch_v30_bwd<T, 1>(gr, w, x, out, dout, tape, rows, rows_bytes, B, iters, st);
        case 2: return launch_v30_bwd<T, 2>(gr, w, x, out, dout, tape, rows, rows_bytes, B, iters, st);
        case 3: return launch_v30_bwd<T, 3>(gr, w, x, out, dout, tape, rows, rows_bytes, B, iters, st);
        case 4: return launch_v30_bwd<T, 4>(gr, w, x, out, dout, tape, rows, rows_bytes, B, iters, st);
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

// training (gnnd_train.hip dispatches model V30 here)
int64_t gnnd_v30_tape_elems(const gnnd_graph* g, int64_t B, int iters) {
    return B * (int64_t)(iters + 1) * 2 * ((int64_t)g->view.C * g->view.G * g->view.R);
}
int64_t gnnd_v30_train_rows(int64_t B) { return B < 1024 ? B : 1024; }
int gnnd_launch_v30_tape(const gnnd_graph* g, int dtype, const void* w, const void* x, void* out,
                         int64_t B, int iters, void* tape, hipStream_t st) {
    if (!tape) return GNND_ERR_INVALID_ARG;
    if (dtype == GNND_F32) return launch_v30_r<float>(g, w, x, out, B, iters, st, tape);
    return launch_v30_r<double>(g, w, x, out, B, iters, st, tape);
}
int gnnd_launch_v30_bwd(const gnnd_graph* g, int dtype, const void* w, const void* x,
                        const void* out, const void* dout, const void* tape, void* rows,
                        int64_t rows_bytes, int64_t B, int iters, hipStream_t st) {
    if (dtype == GNND_F32)
        return launch_v30_bwd_r<float>(g, w, x, out, dout, tape, rows, rows_bytes, B, iters, st);
    return launch_v30_bwd_r<double>(g, w, x, out, dout, tape, rows, rows_bytes, B, iters, st);
}
