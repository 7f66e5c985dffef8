// gnnd_train_wbp.hip — fused training of the weighted ("neural") BP decoders with per-edge
// weight tables (paths relative to /root/reference/GNN-decode/):
//   NBP  quantum/neural_BP.py:95-160, 263-314 (readout after the last layer)
//   V22  quantum/decoder_v2_2.py:120-160, 272-347 (a readout after EVERY layer; the script's
//        8 edge-type weights arrive expanded per edge, gnnd.h V22 layout)
//   V10  quantum/decoder_v1_0.py:97-133, 236-313 (the check-side layer's W scales the whole
//        v->c argument; plain readout): a_e = ((S_v(m) - m_e) + x_v) W_t[e], W_t = w[tE + e],
//        alpha = w[TE]; readout r_v = S_v(m) + x_v.  The tape keeps the unweighted argument
//        z_e = (S_v(m) - m_e) + x_v; the reverse pass takes d W_t[e] = g_a z_e and carries
//        g_z = g_a W_t[e] into the variable leave-one-out (unit message weight).
// fp64 only (both scripts train in double).  Per layer t (packed weights w: W_t = w[2tE + e],
// Wp_t = w[(2t+1)E + e], W_out = w[2TE + e], W_pr = w[2TE + E + e], alpha = w[2TE + 2E]):
//   a_e  = (S_v(m W_t) - m_e W_t[e]) + x_v Wp_t[e]                          (v -> c)
//   t_e  = tanh(a_e / 2), L_e = log(clamp(|t_e|, 1e-20, 1e10)), c_e = [t_e < 0]
//   p_e  = clamp(exp(S_c(L) - L_e) cos(pi (S_c(c) - c_e + (1 - s_c)/2)), +-(1 - 1e-15))
//   m'_e = (log(1 + p_e) - log(1 - p_e)) + m_e alpha                         (c -> v, residual)
//   readout r_v = S_v(m' W_out) + S_v(x_v W_pr), out = sigmoid(-r_v)
// The forward (training tape: every layer's entering states and v->c arguments) follows the
// fused decoder's operation order (gnnd_decode_impl.h decode_resident_kernel, scalar fp64
// path): same sums in the same order, so it reproduces the reference goldens.
// The reverse pass walks t = T-1 .. 0 with torch's autograd rules (clamp passes the gradient
// inside [min, max] inclusive, abs -> sign, log -> 1/x, tanh -> 1 - y^2; the sign/cos factor
// is piecewise constant).  Every per-edge weight has ONE owner lane in a workgroup (the lane
// of the edge's slot), so its gradient accumulates into the workgroup's gradient row in
// global memory with plain read-modify-writes (no atomics); alpha's gradient is summed over
// the lanes at the end.  One codeword at a time per workgroup (grid-strided): deterministic.
#include "gnnd_decode_impl.h"

GNND_DEBUG_TU(train_wbp)

namespace {

struct WbpLayout {          // packed per-edge weight tables (gnnd.h NBP / V22)
    int E, T;
    __device__ __forceinline__ int msg(int t, int e) const { return 2 * t * E + e; }
    __device__ __forceinline__ int prior(int t, int e) const { return (2 * t + 1) * E + e; }
    __device__ __forceinline__ int out_w(int e) const { return 2 * T * E + e; }
    __device__ __forceinline__ int out_p(int e) const { return 2 * T * E + E + e; }
    __device__ __forceinline__ int alpha() const { return 2 * T * E + 2 * E; }
};
struct V10Layout {          // gnnd.h V10: the check-side layers' W, then alpha
    int E, T;
    __device__ __forceinline__ int chk(int t, int e) const { return t * E + e; }
    __device__ __forceinline__ int alpha() const { return T * E; }
};
// kernel kinds: the readout and weight placement of each script
enum WbpKind { kWbpNbp = 0, kWbpV22 = 1, kWbpV10 = 2 };

constexpr int kWbpThreads = GNND_BLOCK;

// graph tables staged per workgroup: slot table, var_ptr, vslot, then per-codeword arrays
__host__ __device__ constexpr size_t wbp_a16(size_t n) { return (n + 15) & ~(size_t)15; }
__host__ __device__ constexpr size_t wbp_lds(int V, int C, int E, int nslot) {
    return wbp_a16(((size_t)nslot + V + 1 + E) * 4) + 8 * (2 * (size_t)nslot + 3 * (size_t)V + C);
}

// forward with tape: tape[b][t][0][slot] = m entering layer t, tape[b][t][1][slot] = a_e of
// layer t (V10: the unweighted z_e); tape[b][T][0][slot] = the final states.  out: PER_LAYER
// [T][B][V], else [B][V].
template <int R, int KIND>
__global__ void __launch_bounds__(kWbpThreads)
wbp_train_fwd_kernel(GraphView g, const double* __restrict__ w, const double* __restrict__ x,
                     double* __restrict__ out, double* __restrict__ tape, int64_t B, int iters) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr bool PER_LAYER = KIND == kWbpV22, V10 = KIND == kWbpV10;
    const int V = g.V, C = g.C, E = g.E, N = g.N, G = g.G, logG = g.logG;
    const int tid = threadIdx.x;
    const int nslot = C * G * R, IC = C * G;
    uint32_t* s_slot = (uint32_t*)smem;
    int* s_vptr = (int*)(s_slot + nslot);
    int* s_vslot = s_vptr + V + 1;
    double* s_m = (double*)(smem + wbp_a16(((size_t)nslot + V + 1 + E) * 4));   // [nslot] states
    double* s_sv = s_m + nslot;          // [V] S_v(m W_t) (V10: S_v(m))
    double* s_xv = s_sv + V;
    double* s_xc = s_xv + V;
    for (int i = tid; i < nslot; i += kWbpThreads) s_slot[i] = g.slot_ve[i];
    for (int i = tid; i <= V; i += kWbpThreads) s_vptr[i] = g.var_ptr[i];
    for (int i = tid; i < E; i += kWbpThreads) s_vslot[i] = g.vslot[i];
    const WbpLayout L{E, iters};
    const V10Layout L10{E, iters};
    const double alpha = w[V10 ? L10.alpha() : L.alpha()];
    const size_t tstride = 2 * (size_t)nslot;

    for (int64_t b = blockIdx.x; b < B; b += gridDim.x) {
        double* tp = tape + (size_t)b * (iters + 1) * tstride;
        __syncthreads();
        for (int i = tid; i < N; i += kWbpThreads) {
            const double xv = x[b * N + i];
            if (i < V) s_xv[i] = xv; else s_xc[i - V] = xv;
        }
        for (int i = tid; i < nslot; i += kWbpThreads) s_m[i] = 0.0;
        for (int i = tid; i < V; i += kWbpThreads) s_sv[i] = 0.0;    // S_v(0 W_0)
        __syncthreads();
        for (int it = 0; it < iters; ++it) {
            const bool last = it + 1 == iters;
            double* tt = tp + (size_t)it * tstride;
            for (int f0 = 0; f0 < IC; f0 += kWbpThreads) {
                const int f = f0 + tid;
                const bool act = f < IC;
                const int rem = act ? f : IC - 1;
                const int c = rem >> logG, s0 = rem * R;
                double tv[R], cf[R], mr[R], tsum = 0.0, csum = 0.0;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const uint32_t sv = s_slot[s0 + r];
                    const int v = (int)(sv & 0xffffu), e = (int)(sv >> 16);
                    const bool valid = e != E;
                    const int ec = valid ? e : 0;
                    mr[r] = s_m[s0 + r];
                    double a;
                    if constexpr (V10) {     // decode_resident_kernel's V10 order
                        const double z = (s_sv[v] - mr[r]) + s_xv[v];
                        a = z * w[L10.chk(it, ec)];
                        if (act) { tt[s0 + r] = mr[r]; tt[nslot + s0 + r] = z; }
                    } else {
                        a = (s_sv[v] - mr[r] * w[L.msg(it, ec)]) + s_xv[v] * w[L.prior(it, ec)];
                        if (act) { tt[s0 + r] = mr[r]; tt[nslot + s0 + r] = a; }
                    }
                    double cc;
                    const double l = wbp_L(a, cc);
                    tv[r] = valid ? l : 0.0;
                    cf[r] = valid ? cc : 0.0;
                    tsum = r == 0 ? tv[0] : tsum + tv[r];
                    csum = r == 0 ? cf[0] : csum + cf[r];
                }
                const double Sc = group_sum(tsum, G), Sc2 = group_sum(csum, G);
                const double sc = s_xc[c];
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const double mn = wbp_out(Sc - tv[r], Sc2 - cf[r], sc) + mr[r] * alpha;
                    if (act) {
                        s_m[s0 + r] = mn;
                        if (last) tt[tstride + s0 + r] = mn;     // tape[b][T][0]
                    }
                }
            }
            __syncthreads();
            // readout of this layer and the next layer's weighted variable sums, edge order
            for (int v = tid; v < V; v += kWbpThreads) {
                const int k0 = s_vptr[v], k1 = s_vptr[v + 1];
                const double xv = s_xv[v];
                if constexpr (V10) {         // S_v(m), then the readout sigmoid(-(S_v + x_v))
                    double sn = 0.0;
                    for (int k = k0; k < k1; ++k) sn += s_m[s_vslot[k]];
                    if (last) out[b * V + v] = sigmoid_ref(-(sn + xv));
                    s_sv[v] = sn;
                    continue;
                }
                double so = 0.0, s2 = 0.0, sn = 0.0;
                for (int k = k0; k < k1; ++k) {
                    const double mk = s_m[s_vslot[k]];
                    so += mk * w[L.out_w(k)];
                    s2 += xv * w[L.out_p(k)];
                    if (!last) sn += mk * w[L.msg(it + 1, k)];
                }
                if (PER_LAYER) out[(size_t)it * B * V + b * V + v] = sigmoid_ref(-(so + s2));
                else if (last) out[b * V + v] = sigmoid_ref(-(so + s2));
                s_sv[v] = sn;
            }
            __syncthreads();
        }
        if (iters == 0 && !PER_LAYER)
            for (int v = tid; v < V; v += kWbpThreads) {
                double s2 = 0.0;
                if constexpr (V10) s2 = s_xv[v];
                else
                    for (int k = s_vptr[v]; k < s_vptr[v + 1]; ++k) s2 += s_xv[v] * w[L.out_p(k)];
                out[b * V + v] = sigmoid_ref(-s2);
            }
    }
}

// reverse pass: d loss / d out -> one gradient row [2TE + 2E + 1] (V10: [TE + 1]) per workgroup
template <int R, int KIND>
__global__ void __launch_bounds__(kWbpThreads)
wbp_train_bwd_kernel(GraphView g, const double* __restrict__ w, const double* __restrict__ x,
                     const double* __restrict__ out, const double* __restrict__ dout,
                     const double* __restrict__ tape, double* __restrict__ rows, int64_t B,
                     int iters) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr bool PER_LAYER = KIND == kWbpV22, V10 = KIND == kWbpV10;
    const int V = g.V, C = g.C, E = g.E, N = g.N, G = g.G, logG = g.logG;
    const int tid = threadIdx.x;
    const int nslot = C * G * R, IC = C * G;
    uint32_t* s_slot = (uint32_t*)smem;
    int* s_vptr = (int*)(s_slot + nslot);
    int* s_vslot = s_vptr + V + 1;
    double* s_G = (double*)(smem + wbp_a16(((size_t)nslot + V + 1 + E) * 4));   // d / d m leaving t
    double* s_ga = s_G + nslot;          // [nslot] d / d a_e
    double* s_gr = s_ga + nslot;         // [V] d / d r_v of layer t's readout
    double* s_gs = s_gr + V;             // [V] sum of d / d a over the variable's edges
    double* s_xv = s_gs + V;
    double* s_xc = s_xv + V;
    for (int i = tid; i < nslot; i += kWbpThreads) s_slot[i] = g.slot_ve[i];
    for (int i = tid; i <= V; i += kWbpThreads) s_vptr[i] = g.var_ptr[i];
    for (int i = tid; i < E; i += kWbpThreads) s_vslot[i] = g.vslot[i];
    const WbpLayout L{E, iters};
    const V10Layout L10{E, iters};
    const int ialpha = V10 ? L10.alpha() : L.alpha();
    const int P = ialpha + 1;
    const double alpha = w[ialpha];
    const double hi = 1 - 1e-15;
    const size_t tstride = 2 * (size_t)nslot;
    double* row = rows + (size_t)blockIdx.x * P;
    for (int i = tid; i < P; i += kWbpThreads) row[i] = 0.0;
    double galpha = 0.0;                 // this lane's share of d loss / d alpha

    for (int64_t b = blockIdx.x; b < B; b += gridDim.x) {
        const double* tp = tape + (size_t)b * (iters + 1) * tstride;
        __syncthreads();                 // row zeroed / previous codeword done with LDS
        for (int i = tid; i < N; i += kWbpThreads) {
            const double xv = x[b * N + i];
            if (i < V) s_xv[i] = xv; else s_xc[i - V] = xv;
        }
        for (int i = tid; i < nslot; i += kWbpThreads) s_G[i] = 0.0;
        for (int t = iters - 1; t >= 0; --t) {
            const bool ro = PER_LAYER || t == iters - 1;     // layer t has a readout
            __syncthreads();
            if (ro)
                for (int v = tid; v < V; v += kWbpThreads) {
                    const size_t o = (PER_LAYER ? (size_t)t * B * V : 0) + (size_t)b * V + v;
                    const double p = out[o];
                    s_gr[v] = -((dout[o] * (1.0 - p)) * p);     // sigmoid(-r) backward
                }
            __syncthreads();
            const double* tt = tp + (size_t)t * tstride;      // m^t, a^t
            const double* tn = tt + tstride;                   // m^{t+1}
            for (int f0 = 0; f0 < IC; f0 += kWbpThreads) {
                const int f = f0 + tid;
                const bool act = f < IC;
                const int rem = act ? f : IC - 1;
                const int c = rem >> logG, s0 = rem * R;
                int vv[R], ee[R];
                bool ok[R];
                double a[R], th[R], cl[R], Lr[R], cf[R], Gm[R], tsum = 0.0, csum = 0.0;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const uint32_t sv = s_slot[s0 + r];
                    vv[r] = (int)(sv & 0xffffu);
                    ee[r] = (int)(sv >> 16);
                    ok[r] = ee[r] != E;
                    const int ec = ok[r] ? ee[r] : 0;
                    // readout of layer t: d / d m^{t+1} and the readout weights
                    double Gv = s_G[s0 + r];
                    if (ro && ok[r]) {
                        const double gr = s_gr[vv[r]];
                        if constexpr (V10) {
                            Gv += gr;                  // r_v = S_v(m) + x_v: unit weights
                        } else {
                            Gv += w[L.out_w(ec)] * gr;
                            if (act) {
                                row[L.out_w(ec)] += tn[s0 + r] * gr;
                                row[L.out_p(ec)] += s_xv[vv[r]] * gr;
                            }
                        }
                    }
                    Gm[r] = ok[r] ? Gv : 0.0;
                    // (V10: the forward's a = z W_t[e], the same product)
                    a[r] = V10 ? tt[nslot + s0 + r] * w[L10.chk(t, ec)] : tt[nslot + s0 + r];
                    th[r] = g_tanh(a[r] / 2.0);
                    cf[r] = th[r] < 0.0 ? 1.0 : 0.0;
                    cl[r] = g_clamp(fabs(th[r]), 1e-20, 1e10);
                    Lr[r] = g_log(cl[r]);
                    const double tv = ok[r] ? Lr[r] : 0.0, cv = ok[r] ? cf[r] : 0.0;
                    tsum = r == 0 ? tv : tsum + tv;
                    csum = r == 0 ? cv : csum + cv;
                }
                const double Sc = group_sum(tsum, G), Sc2 = group_sum(csum, G);
                const double sc = s_xc[c];
                double glam[R], gsum = 0.0;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const double m = tt[s0 + r];
                    if (act && ok[r]) galpha = __builtin_fma(m, Gm[r], galpha);
                    // c -> v message backward: msg = log(1 + p) - log(1 - p)
                    const double lam = Sc - (ok[r] ? Lr[r] : 0.0);
                    const double n = (Sc2 - (ok[r] ? cf[r] : 0.0)) + (1.0 - sc) / 2.0;
                    const double cs = cos_pi(n), ex = g_exp(lam);
                    const double praw = ex * cs;
                    const double p = g_clamp(praw, -hi, hi);
                    const double gp = Gm[r] / (1.0 + p) + Gm[r] / (1.0 - p);
                    const double gpr = (praw >= -hi && praw <= hi) ? gp : 0.0;
                    glam[r] = ok[r] ? (gpr * cs) * ex : 0.0;
                    gsum = r == 0 ? glam[0] : gsum + glam[r];
                }
                const double Sg = group_sum(gsum, G);
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int sl = s0 + r;
                    const double gL = Sg - glam[r];
                    const double at = fabs(th[r]);
                    const double gabs = (at >= 1e-20 && at <= 1e10) ? gL / cl[r] : 0.0;
                    const double gt = th[r] > 0.0 ? gabs : th[r] < 0.0 ? -gabs : 0.0;
                    const double ga = ok[r] ? (gt * (1.0 - th[r] * th[r])) / 2.0 : 0.0;
                    if (act) {
                        s_G[sl] = Gm[r] * alpha;                     // residual m^t alpha
                        if constexpr (V10) {
                            // a = z W_t[e]: d W_t[e] = g_a z, d z = g_a W_t[e]
                            const int ec = ok[r] ? ee[r] : 0;
                            s_ga[sl] = ga * w[L10.chk(t, ec)];
                            if (ok[r]) row[L10.chk(t, ee[r])] += tt[nslot + sl] * ga;
                        } else {
                            s_ga[sl] = ga;
                            if (ok[r]) row[L.prior(t, ee[r])] += s_xv[vv[r]] * ga;
                        }
                    }
                }
            }
            __syncthreads();
            for (int v = tid; v < V; v += kWbpThreads) {
                double s = 0.0;
                for (int k = s_vptr[v]; k < s_vptr[v + 1]; ++k) s += s_ga[s_vslot[k]];
                s_gs[v] = s;
            }
            __syncthreads();
            // a_e = (S_v(m W_t) - m_e W_t[e]) + ...:  d / d (m W_t)[e] = S_v(g_a) - g_a[e]
            // (V10: z_e = (S_v(m) - m_e) + x_v:  d / d m_e = S_v(g_z) - g_z[e])
            for (int i = tid; i < nslot; i += kWbpThreads) {
                const uint32_t sv = s_slot[i];
                const int e = (int)(sv >> 16);
                if (e == E) continue;
                const double gmw = s_gs[sv & 0xffffu] - s_ga[i];
                if constexpr (V10) {
                    s_G[i] += gmw;
                } else {
                    row[L.msg(t, e)] += tt[i] * gmw;
                    s_G[i] += w[L.msg(t, e)] * gmw;
                }
            }
        }
    }
    // alpha: sum over the workgroup's lanes (fixed butterfly per wave, then the waves in order)
    __shared__ double s_al[kWbpThreads / 64];
    for (int o = 1; o < 64; o <<= 1) galpha += __shfl_xor(galpha, o);
    __syncthreads();
    if ((tid & 63) == 0) s_al[tid >> 6] = galpha;
    __syncthreads();
    if (tid == 0) {
        double s = 0.0;
        for (int k = 0; k < kWbpThreads / 64; ++k) s += s_al[k];
        row[ialpha] = s;
    }
}

template <int R>
int launch_wbp(const gnnd_graph* gr, int model, const void* w, const void* x, void* out,
               const void* dout, const void* tape, void* rows, int64_t rows_bytes, int64_t B,
               int iters, hipStream_t st, bool fwd) {
    const GraphView& g = gr->view;
    const int nslot = g.C * g.G * g.R;
    const int64_t blocks = gnnd_wbp_train_rows(B);
    const size_t lds = wbp_lds(g.V, g.C, g.E, nslot);
    if (lds > 64 * 1024) return GNND_ERR_UNSUPPORTED;
    const int kind = model == GNND_V22 ? kWbpV22 : model == GNND_V10 ? kWbpV10 : kWbpNbp;
    if (fwd) {
        auto k = kind == kWbpV22 ? wbp_train_fwd_kernel<R, kWbpV22>
               : kind == kWbpV10 ? wbp_train_fwd_kernel<R, kWbpV10> : wbp_train_fwd_kernel<R, kWbpNbp>;
        k<<<(unsigned)blocks, kWbpThreads, lds, st>>>(g, (const double*)w, (const double*)x,
                                                       (double*)out, (double*)tape, B, iters);
    } else {
        const int64_t P = gnnd_wbp_weights(gr, model, iters);
        if (blocks * P * 8 > rows_bytes) return GNND_ERR_INVALID_ARG;
        auto k = kind == kWbpV22 ? wbp_train_bwd_kernel<R, kWbpV22>
               : kind == kWbpV10 ? wbp_train_bwd_kernel<R, kWbpV10> : wbp_train_bwd_kernel<R, kWbpNbp>;
        k<<<(unsigned)blocks, kWbpThreads, lds, st>>>(g, (const double*)w, (const double*)x,
                                                       (const double*)out, (const double*)dout,
                                                       (const double*)tape, (double*)rows, B, iters);
    }
    GNND_LAUNCH_CHECK();
    return GNND_OK;
}

int launch_wbp_r(const gnnd_graph* gr, int model, const void* w, const void* x, void* out,
                 const void* dout, const void* tape, void* rows, int64_t rows_bytes, int64_t B,
                 int iters, hipStream_t st, bool fwd) {
    switch (gr->view.R) {
        case 1: return launch_wbp<1>(gr, model, w, x, out, dout, tape, rows, rows_bytes, B, iters, st, fwd);
        case 2: return launch_wbp<2>(gr, model, w, x, out, dout, tape, rows, rows_bytes, B, iters, st, fwd);
        case 3: return launch_wbp<3>(gr, model, w, x, out, dout, tape, rows, rows_bytes, B, iters, st, fwd);
        case 4: return launch_wbp<4>(gr, model, w, x, out, dout, tape, rows, rows_bytes, B, iters, st, fwd);
    }
    return GNND_ERR_UNSUPPORTED;
}

}  // namespace

int64_t gnnd_wbp_tape_elems(const gnnd_graph* g, int64_t B, int iters) {
    return B * (int64_t)(iters + 1) * 2 * ((int64_t)g->view.C * g->view.G * g->view.R);
}
int64_t gnnd_wbp_train_rows(int64_t B) { return B < 1024 ? B : 1024; }
// trainable values of a weighted-BP model's packed tables (gnnd.h NBP / V22 / V10 layouts)
int64_t gnnd_wbp_weights(const gnnd_graph* g, int model, int iters) {
    const int64_t E = g->view.E;
    return model == GNND_V10 ? (int64_t)iters * E + 1 : 2 * (int64_t)iters * E + 2 * E + 1;
}
int gnnd_launch_wbp_tape(const gnnd_graph* g, int model, const void* w, const void* x, void* out,
                         int64_t B, int iters, void* tape, hipStream_t st) {
    if (!tape) return GNND_ERR_INVALID_ARG;
    return launch_wbp_r(g, model, w, x, out, nullptr, tape, nullptr, 0, B, iters, st, true);
}
int gnnd_launch_wbp_bwd(const gnnd_graph* g, int model, const void* w, const void* x,
                        const void* out, const void* dout, const void* tape, void* rows,
                        int64_t rows_bytes, int64_t B, int iters, hipStream_t st) {
    return launch_wbp_r(g, model, w, x, (void*)out, dout, tape, rows, rows_bytes, B, iters, st, false);
}
