// gnnd_train.hip — fused training step of decoder_v2_4, its
// syndrome loss, Adam, and the hard-decision metrics.
//
// Forward: the streaming decode kernel with its TAPE instantiation (gnnd_decode_impl.h) runs
// GNNI.forward (quantum/decoder_v2_4.py:272-294) and records, per iteration and edge, the
// v->c MLP input ext = S_v - m, the tanh output t and the c->v MLP input u = S_c - t, plus
// the final messages m^T.  The loss (quantum/decoder_v2_4.py:297-317) and its gradient are
// one launch (syndrome_loss_kernel).
// Backward (this file): reverse-mode through the whole T-iteration loop in ONE launch, each
// workgroup looping over a strided set of codewords, replacing the reference's autograd
// graph of ~60 small ops per iteration:
//   readout  dr_v = -(g_v (1 - p_v)) p_v,  MLP_o backward at m^T  -> dm
//   t = T-1 .. 0:
//     A  MLP_c backward at u with dy = dm s_c                      -> du, grads ggc2.mlp
//     B  dt = LOO_c(du), da = (dt (1 - t^2)) / 2                   (check leave-one-out)
//     C  MLP_v backward at (ext, x_v) with dy = da                  -> dext, grads ggc1.mlp
//     D  dm += LOO_v(dext)                                         (residual keeps dm)
// The MLP phases are UNIT-parallel: a wave walks its share of the codeword's edges two at a
// time while each lane owns two of the 128 hidden units (weights in VGPRs), so every weight
// gradient accumulates in the lane's registers over all edges, iterations and codewords with
// no cross-lane traffic; only d(input) of an edge needs a wave reduction (fp32: one
// permlane-swap + DPP chain for both edges).  The edge phases B/D are edge-parallel
// leave-one-out sums in LDS.  Per-workgroup gradient partials are summed over the
// workgroups in a fixed order by a second kernel (deterministic, run-to-run identical).
// torch's autograd rules are followed: Softplus(beta 1, threshold 20) backward
// g z / (z + 1), z = e^h (g above the threshold), tanh backward g (1 - t^2), division by 2.
#include "gnnd_decode_impl.h"

GNND_DEBUG_TU(train)
#include <type_traits>
#include <stdlib.h>

namespace {

// threads per workgroup: 16 waves (4 per SIMD) in fp32 (128 VGPRs), 8 in fp64 (<= 256 VGPRs)
template <typename T> constexpr int train_threads() { return sizeof(T) == 4 ? 1024 : 512; }
// fp64 Softplus table of the reverse pass: GNND_BWD_SGTAB 1 (default) the signed one-read table
// (kSgTab, sg_index / sg_poly / sg_grad_poly), 0 the |h|-indexed kSpTab (A/B builds)
#ifndef GNND_BWD_SGTAB
#define GNND_BWD_SGTAB 1
#endif
constexpr int kBwdTabDoubles = GNND_BWD_SGTAB ? kSgTabDoubles : kSpTabDoubles;
__device__ __forceinline__ double bwd_tab_entry(int i) { return GNND_BWD_SGTAB ? kSgTab[i] : kSpTab[i]; }
// LDS bytes of the Softplus tables the fp64 reverse pass stages ahead of its graph tables
template <typename T> constexpr size_t bwd_tab_bytes() { return sizeof(T) == 8 ? (size_t)kBwdTabDoubles * 8 : 0; }
constexpr int kV24W = 1283;                 // packed plain weights (gnnd.h)

// fp64 Softplus and its derivative at N arguments h from one table entry each, all N 16-byte
// reads issued before the first use (hipcc otherwise schedules the chains one after another,
// lgkmcnt(0) after each read):
//   sph = softplus(h) - h/2  (the linear h/2 part is summed once per wave, Units::sx*, instead
//         of a max + add per unit),
//   sg  = sigmoid(h).
// kSgTab: sph = g(h) and sg = 1/2 + g'(h) from the signed entry (no |h|, no threshold select, no
// sign copy); the linear clamp entries give sph = h/2, sg = 1 above torch's threshold (h > 20).
// kSpTab: sph = |h|/2 + ln(1 + e^-|h|), sg = 1/2 + copysign(1/2 - s(|h|), h), the zero entry
// above the threshold.
template <int N>
__device__ __forceinline__ void sph_and_grad_n(const double (&h)[N], double (&sph)[N],
                                               double (&sg)[N], const double* tab) {
    SpIdx q[N];
    SpEntry e[N];
#pragma unroll
    for (int i = 0; i < N; ++i) q[i] = GNND_BWD_SGTAB ? sg_index(h[i]) : sp_index(h[i]);
#pragma unroll
    for (int i = 0; i < N; ++i) e[i] = sp_entry(tab, q[i].j);
#pragma unroll
    for (int i = 0; i < N; ++i) {
        if (GNND_BWD_SGTAB) {
            sph[i] = sg_poly(q[i].r, e[i].f0, e[i].s);
            sg[i] = 0.5 + sg_grad_poly(q[i].r, e[i].s);
        } else {
            sph[i] = __builtin_fma(__builtin_fabs(h[i]), 0.5, sp_poly(q[i].r, e[i].f0, e[i].s));
            // sigmoid(h) = 1/2 + copysign(1/2 - s(|h|), h)
            sg[i] = 0.5 + __builtin_copysign(sig_half_poly(q[i].r, e[i].s), h[i]);
        }
    }
}
__device__ __forceinline__ void sp_and_grad(float h, float& sp, float& sg, const float*) {
    if (h > 20.f) { sp = h; sg = 1.f; return; }
    const float z = __builtin_amdgcn_exp2f(h * kLog2e);
    const float z1 = 1.f + z;
    sp = kLn2 * __builtin_amdgcn_logf(z1);
    sg = z * __builtin_amdgcn_rcpf(z1);
}

// total of a wave64 value, uniform (SGPR) result: DPP row reduction (quad_perm x2, half /
// full row mirror), then row_bcast:15 / row_bcast:31 carry the row sums into lane 63 —
// all on the VALU, no LDS round trip (the __shfl_xor form costs two ds_bpermute
// latencies on every edge's critical path).
template <int CTRL, int ROWS> __device__ __forceinline__ int dpp_i(int v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, ROWS, 0xf, false);
}
__device__ __forceinline__ float wave_sum(float v) {
    v += __int_as_float(dpp_i<0xB1, 0xf>(__float_as_int(v)));
    v += __int_as_float(dpp_i<0x4E, 0xf>(__float_as_int(v)));
    v += __int_as_float(dpp_i<0x141, 0xf>(__float_as_int(v)));
    v += __int_as_float(dpp_i<0x140, 0xf>(__float_as_int(v)));
    v += __int_as_float(dpp_i<0x142, 0xa>(__float_as_int(v)));   // row_bcast:15 -> rows 1, 3
    v += __int_as_float(dpp_i<0x143, 0xc>(__float_as_int(v)));   // row_bcast:31 -> rows 2, 3
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
// totals of two wave64 values at once (gfx950 lane swaps): v_permlane32_swap folds the upper
// half of a onto its lower half and the lower half of b onto its upper half, so lanes 0-31
// carry a and lanes 32-63 carry b; v_permlane16_swap folds row pairs, four row DPP steps
// finish each row.  One chain for both (vs two six-step DPP chains with their wait states).
__device__ __forceinline__ void wave_sum2(float a, float b, float& ra, float& rb) {
    const auto s32 = __builtin_amdgcn_permlane32_swap(__float_as_int(a), __float_as_int(b), false, false);
    float v = __int_as_float(s32[0]) + __int_as_float(s32[1]);
    const auto s16 = __builtin_amdgcn_permlane16_swap(__float_as_int(v), __float_as_int(v), false, false);
    v = __int_as_float(s16[0]) + __int_as_float(s16[1]);
    v += __int_as_float(dpp_i<0xB1, 0xf>(__float_as_int(v)));
    v += __int_as_float(dpp_i<0x4E, 0xf>(__float_as_int(v)));
    v += __int_as_float(dpp_i<0x141, 0xf>(__float_as_int(v)));
    v += __int_as_float(dpp_i<0x140, 0xf>(__float_as_int(v)));
    ra = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
    rb = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
}
// totals of FOUR wave64 values (two pairs): the two permlane32 folds as above, then ONE
// v_permlane16_swap between the two folded vectors leaves one edge per 16-lane row, and one
// four-step row DPP chain finishes all four (wave_sum2 twice: two swaps16 and two chains).
// Row order of the swap: GNND_PL16_MAP 0 -> rows {a, c, b, d}, 1 -> {c, a, d, b}.
#ifndef GNND_PL16_MAP
#define GNND_PL16_MAP 0
#endif
__device__ __forceinline__ void wave_sum4(f32x2 ab, f32x2 cd, float& ra, float& rb, float& rc,
                                          float& rd) {
    const auto s1 = __builtin_amdgcn_permlane32_swap(__float_as_int(ab.x), __float_as_int(ab.y), false, false);
    const float v1 = __int_as_float(s1[0]) + __int_as_float(s1[1]);      // lanes 0-31 a, 32-63 b
    const auto s2 = __builtin_amdgcn_permlane32_swap(__float_as_int(cd.x), __float_as_int(cd.y), false, false);
    const float v2 = __int_as_float(s2[0]) + __int_as_float(s2[1]);      // c | d
    const auto s3 = __builtin_amdgcn_permlane16_swap(__float_as_int(v1), __float_as_int(v2), false, false);
    float v = __int_as_float(s3[0]) + __int_as_float(s3[1]);
    v += __int_as_float(dpp_i<0xB1, 0xf>(__float_as_int(v)));
    v += __int_as_float(dpp_i<0x4E, 0xf>(__float_as_int(v)));
    v += __int_as_float(dpp_i<0x141, 0xf>(__float_as_int(v)));
    v += __int_as_float(dpp_i<0x140, 0xf>(__float_as_int(v)));
    const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
    const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
    const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
    const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
    if (GNND_PL16_MAP == 0) { ra = r0; rc = r1; rb = r2; rd = r3; }
    else { rc = r0; ra = r1; rd = r2; rb = r3; }
}
// wave_sum4 without the lane reads: every lane of 16-lane row r ends with the total of the
// edge kRowEdge[r] (rows {a, c, b, d} under GNND_PL16_MAP 0), for a store by the rows' lanes
__device__ __forceinline__ float wave_rows4(f32x2 ab, f32x2 cd) {
    const auto s1 = __builtin_amdgcn_permlane32_swap(__float_as_int(ab.x), __float_as_int(ab.y), false, false);
    const float v1 = __int_as_float(s1[0]) + __int_as_float(s1[1]);
    const auto s2 = __builtin_amdgcn_permlane32_swap(__float_as_int(cd.x), __float_as_int(cd.y), false, false);
    const float v2 = __int_as_float(s2[0]) + __int_as_float(s2[1]);
    const auto s3 = __builtin_amdgcn_permlane16_swap(__float_as_int(v1), __float_as_int(v2), false, false);
    float v = __int_as_float(s3[0]) + __int_as_float(s3[1]);
    v += __int_as_float(dpp_i<0xB1, 0xf>(__float_as_int(v)));
    v += __int_as_float(dpp_i<0x4E, 0xf>(__float_as_int(v)));
    v += __int_as_float(dpp_i<0x141, 0xf>(__float_as_int(v)));
    v += __int_as_float(dpp_i<0x140, 0xf>(__float_as_int(v)));
    return v;
}
// edge (0..3 of the step's four) whose total row r of wave_rows4 holds
__device__ __forceinline__ int row_edge(int row) {
    return GNND_PL16_MAP == 0 ? (row == 1 ? 2 : row == 2 ? 1 : row) : (row == 0 ? 2 : row == 1 ? 0 : row == 2 ? 3 : 1);
}
template <int CTRL, int ROWS> __device__ __forceinline__ double dpp_d(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = dpp_i<CTRL, ROWS>((int)b), hi = dpp_i<CTRL, ROWS>((int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double wave_sum(double v) {
    v += dpp_d<0xB1, 0xf>(v);
    v += dpp_d<0x4E, 0xf>(v);
    v += dpp_d<0x141, 0xf>(v);
    v += dpp_d<0x140, 0xf>(v);
    v += dpp_d<0x142, 0xa>(v);
    v += dpp_d<0x143, 0xc>(v);
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, 63), hi = __builtin_amdgcn_readlane((int)(b >> 32), 63);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// fp64 wave_rows4: the same lane folds on both 32-bit halves of every value, then the row
// DPP chain in fp64 (21 VALU for four edges' totals; two six-step wave_sum chains per edge pair
// were ~40 dependent ops per pair)
__device__ __forceinline__ double pl32_fold(double a, double b) {
    const long long ia = __double_as_longlong(a), ib = __double_as_longlong(b);
    const auto lo = __builtin_amdgcn_permlane32_swap((int)ia, (int)ib, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((int)(ia >> 32), (int)(ib >> 32), false, false);
    return __longlong_as_double(((long long)hi[0] << 32) | (unsigned)lo[0]) +
           __longlong_as_double(((long long)hi[1] << 32) | (unsigned)lo[1]);
}
__device__ __forceinline__ double wave_rows4(double a, double b, double c, double d) {
    const double v1 = pl32_fold(a, b), v2 = pl32_fold(c, d);
    const long long i1 = __double_as_longlong(v1), i2 = __double_as_longlong(v2);
    const auto lo = __builtin_amdgcn_permlane16_swap((int)i1, (int)i2, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((int)(i1 >> 32), (int)(i2 >> 32), false, false);
    double v = __longlong_as_double(((long long)hi[0] << 32) | (unsigned)lo[0]) +
               __longlong_as_double(((long long)hi[1] << 32) | (unsigned)lo[1]);
    v += dpp_d<0xB1, 0xf>(v);
    v += dpp_d<0x4E, 0xf>(v);
    v += dpp_d<0x141, 0xf>(v);
    v += dpp_d<0x140, 0xf>(v);
    return v;
}

// v with lane k replaced by the uniform value x (compare + select)
template <typename T> __device__ __forceinline__ T put_lane(T v, T x, int k, int lane) {
    return lane == k ? x : v;
}

// two hidden units of one MLP owned by this lane: k0 = lane, k1 = lane + 64
template <typename T> struct Units {
    T w1a[2], w1b[2], b1[2], w2[2];         // w1b only for the 2-input MLP
    T gw1a[2], gw1b[2], gb1[2], gw2[2], gb2;
    // fp64: layer-1 gradients accumulate WITHOUT the W2 factor (applied at flush), d input
    // through w2w1a = W2 W1a, and the linear half of relu(h) in dW2 as the per-wave sums
    // sx0 = sum dy u0, sx1 = sum dy u1 (with gb2 = sum dy): dW2 += (W1a sx0 + W1b sx1 + b1 gb2)/2
    T w2w1a[2], sx0, sx1;
    f32x2 pgw1a[2], pgw1b[2], pgb1[2], pgw2[2];  // fp32 packed path: per-edge-half partials
    float s1a[2], s1b[2], sb1[2];                // fp32: layer 1 in log2 units (x log2 e)
    float ws1a[2];                               // fp32: W2 W1a (d input with W2 factored out)
    __device__ void zero_packed() {
        zero_pg();
        for (int j = 0; j < 2; ++j) {
            s1a[j] = (float)w1a[j] * kLog2e;
            s1b[j] = (float)w1b[j] * kLog2e;
            sb1[j] = (float)b1[j] * kLog2e;
            ws1a[j] = (float)w2[j] * (float)w1a[j];
        }
    }
    // fp32: the per-edge-half partials live for one pass over the edges only (zero_pg at its
    // start, fold at its end): between passes only the scalar gradients stay in registers
    __device__ __forceinline__ void zero_pg() {
        for (int j = 0; j < 2; ++j) pgw1a[j] = pgw1b[j] = pgb1[j] = pgw2[j] = f32x2{0.f, 0.f};
    }
    __device__ __forceinline__ void fold() {       // (layer-1 partials carry no W2 factor)
        for (int j = 0; j < 2; ++j) {
            gw1a[j] += (pgw1a[j].x + pgw1a[j].y) * (float)w2[j];
            gw1b[j] += (pgw1b[j].x + pgw1b[j].y) * (float)w2[j];
            gb1[j] += (pgb1[j].x + pgb1[j].y) * (float)w2[j];
            gw2[j] += (pgw2[j].x + pgw2[j].y) * kLn2;
        }
    }
    // fp32: the per-lane constants a unit pass reads (s1a, s1b, sb1, ws1a, W2) parked in LDS
    // between passes ([10][64] floats per MLP, identical in every wave: wave 0 writes them), so
    // only the active MLP's stay in registers (the 16-wave reverse pass holds 128 VGPRs)
    __device__ void park(float* sp, int lane) const {
        for (int j = 0; j < 2; ++j) {
            sp[(0 + j) * 64 + lane] = s1a[j];
            sp[(2 + j) * 64 + lane] = s1b[j];
            sp[(4 + j) * 64 + lane] = sb1[j];
            sp[(6 + j) * 64 + lane] = ws1a[j];
            sp[(8 + j) * 64 + lane] = (float)w2[j];
        }
    }
    __device__ __forceinline__ void unpark(const float* sp, int lane) {
        for (int j = 0; j < 2; ++j) {
            s1a[j] = sp[(0 + j) * 64 + lane];
            s1b[j] = sp[(2 + j) * 64 + lane];
            sb1[j] = sp[(4 + j) * 64 + lane];
            ws1a[j] = sp[(6 + j) * 64 + lane];
            w2[j] = (T)sp[(8 + j) * 64 + lane];
        }
    }
    __device__ void load1(const T* __restrict__ w, int lane) {    // {W1, b1, W2, b2}
        for (int j = 0; j < 2; ++j) {
            const int k = lane + 64 * j;
            w1a[j] = w[k]; w1b[j] = T(0); b1[j] = w[128 + k]; w2[j] = w[256 + k];
            gw1a[j] = gw1b[j] = gb1[j] = gw2[j] = T(0);
        }
        gb2 = sx0 = sx1 = T(0);
        for (int j = 0; j < 2; ++j) w2w1a[j] = w2[j] * w1a[j];
        zero_packed();
    }
    __device__ void load2(const T* __restrict__ w, int lane) {    // {W1a, W1b, b1, W2, b2}
        for (int j = 0; j < 2; ++j) {
            const int k = lane + 64 * j;
            w1a[j] = w[k]; w1b[j] = w[128 + k]; b1[j] = w[256 + k]; w2[j] = w[384 + k];
            gw1a[j] = gw1b[j] = gb1[j] = gw2[j] = T(0);
        }
        gb2 = sx0 = sx1 = T(0);
        for (int j = 0; j < 2; ++j) w2w1a[j] = w2[j] * w1a[j];
        zero_packed();
    }
    // fp64: four CONSECUTIVE edges per wave step (the fp32 unit pass's shape): eight independent
    // Softplus/sigmoid evaluations per lane, weight gradients summed over the four edges as a
    // tree, the four d inputs row-reduced by one wave_rows4 (every lane of row r ends with the
    // total of edge row_edge(r))
    template <bool TWO>
    __device__ __forceinline__ double bwd4_rows_f64(const double (&x0)[4], const double (&x1)[4],
                                                    const double (&dy)[4], const double* tab) {
        double p[4] = {0.0, 0.0, 0.0, 0.0};
        double h8[8], sph8[8], sg8[8];
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                double h = x0[i] * w1a[j];
                if constexpr (TWO) h = h + x1[i] * w1b[j];
                h8[4 * j + i] = h + b1[j];
            }
        sph_and_grad_n<8>(h8, sph8, sg8, tab);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const double* sp = sph8 + 4 * j;
            double dh[4];                         // d y / d h without the W2 factor
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                dh[i] = dy[i] * sg8[4 * j + i];
                p[i] += dh[i] * w2w1a[j];
            }
            gw2[j] += (dy[0] * sp[0] + dy[1] * sp[1]) + (dy[2] * sp[2] + dy[3] * sp[3]);
            gw1a[j] += (dh[0] * x0[0] + dh[1] * x0[1]) + (dh[2] * x0[2] + dh[3] * x0[3]);
            if constexpr (TWO)
                gw1b[j] += (dh[0] * x1[0] + dh[1] * x1[1]) + (dh[2] * x1[2] + dh[3] * x1[3]);
            gb1[j] += (dh[0] + dh[1]) + (dh[2] + dh[3]);
        }
        gb2 += (dy[0] + dy[1]) + (dy[2] + dy[3]);
        sx0 += (dy[0] * x0[0] + dy[1] * x0[1]) + (dy[2] * x0[2] + dy[3] * x0[3]);
        if constexpr (TWO) sx1 += (dy[0] * x1[0] + dy[1] * x1[1]) + (dy[2] * x1[2] + dy[3] * x1[3]);
        return wave_rows4(p[0], p[1], p[2], p[3]);
    }
    // fp32: edges a and b ride the two halves of every packed op (v_pk_fma/mul/add_f32 with
    // the lane's weights broadcast); the weight gradients accumulate per half (pg*) and are
    // folded at flush.  Layer 1 runs on log2(e)-scaled weights, so hs = h log2 e feeds exp2
    // directly and sp log2 e = max(hs, log2(1 + 2^min(hs, 20 log2 e))) accumulates into gW2
    // (times ln 2 at flush).  Softplus(beta 1, threshold 20): the capped exp argument cannot
    // overflow, e^20 / (1 + e^20) rounds to 1 (the threshold branch's derivative) and the
    // value is h above the threshold.
    template <bool TWO>
    __device__ __forceinline__ void bwd2_f32(float xa0, float xa1, float dya, float xb0, float xb1,
                                             float dyb, float& ra, float& rb) {
        const f32x2 p = bwd2_f32_part<TWO>(xa0, xa1, dya, xb0, xb1, dyb);
        wave_sum2(p.x, p.y, ra, rb);
    }
    // four edges: two pairs' unit work, one shared wave reduction (wave_sum4)
    template <bool TWO>
    __device__ __forceinline__ void bwd4_f32(const float (&x0)[4], const float (&x1)[4],
                                             const float (&dy)[4], float (&r)[4]) {
        const f32x2 pab = bwd2_f32_part<TWO>(x0[0], x1[0], dy[0], x0[1], x1[1], dy[1]);
        const f32x2 pcd = bwd2_f32_part<TWO>(x0[2], x1[2], dy[2], x0[3], x1[3], dy[3]);
        wave_sum4(pab, pcd, r[0], r[1], r[2], r[3]);
    }
    // four CONSECUTIVE edges as two packed pairs {0,1}, {2,3} (the ds_read_b128 inputs of the
    // unit pass): returns the row-reduced vector of wave_rows4 (every lane of row r holds the
    // d input total of edge kRowEdge[r])
    template <bool TWO>
    __device__ __forceinline__ float bwd4_rows(f32x4 x0, f32x4 x1, f32x4 dy) {
        const f32x2 pab = bwd2_f32_part2<TWO>(f32x2{x0.x, x0.y}, f32x2{x1.x, x1.y}, f32x2{dy.x, dy.y});
        const f32x2 pcd = bwd2_f32_part2<TWO>(f32x2{x0.z, x0.w}, f32x2{x1.z, x1.w}, f32x2{dy.z, dy.w});
        return wave_rows4(pab, pcd);
    }
    // the per-lane unit work of two edges: weight-gradient partials accumulated, returns the
    // lane's d input partials (log2 units) of both edges, to be wave-reduced
    template <bool TWO>
    __device__ __forceinline__ f32x2 bwd2_f32_part(float xa0, float xa1, float dya, float xb0,
                                                   float xb1, float dyb) {
        return bwd2_f32_part2<TWO>(f32x2{xa0, xb0}, f32x2{xa1, xb1}, f32x2{dya, dyb});
    }
    template <bool TWO>
    __device__ __forceinline__ f32x2 bwd2_f32_part2(f32x2 x0, f32x2 x1, f32x2 dy) {
        f32x2 p = {0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            f32x2 h = x0 * s1a[j] + sb1[j];
            if constexpr (TWO) h = x1 * s1b[j] + h;
            constexpr float kCap = 20.f * kLog2e;
            const f32x2 hc = {__builtin_fminf(h.x, kCap), __builtin_fminf(h.y, kCap)};
            const f32x2 z = {__builtin_amdgcn_exp2f(hc.x), __builtin_amdgcn_exp2f(hc.y)};
            const f32x2 z1 = z + 1.f;
            const f32x2 l = {__builtin_amdgcn_logf(z1.x), __builtin_amdgcn_logf(z1.y)};
            // sp log2 e = max(h, l): l > h below the cap, h above it (l of the capped
            // argument); two plain v_max_f32 (fmaxf would add NaN-quieting canonicalisations)
            f32x2 sp;
            asm("v_max_f32 %0, %1, %2" : "=v"(sp.x) : "v"(h.x), "v"(l.x));
            asm("v_max_f32 %0, %1, %2" : "=v"(sp.y) : "v"(h.y), "v"(l.y));
            const f32x2 sg = z * f32x2{__builtin_amdgcn_rcpf(z1.x), __builtin_amdgcn_rcpf(z1.y)};
            pgw2[j] = dy * sp + pgw2[j];
            // dh = dy W2 sg: the lane's constant W2 is factored out of the layer-1 partials
            // (applied in fold) and into ws1a = W2 s1a for d input: one packed multiply less
            const f32x2 dh = dy * sg;
            pgw1a[j] = dh * x0 + pgw1a[j];
            if constexpr (TWO) pgw1b[j] = dh * x1 + pgw1b[j];
            pgb1[j] = pgb1[j] + dh;
            p = dh * ws1a[j] + p;            // d input (natural units)
        }
        gb2 += dy.x;
        gb2 += dy.y;
        return p;
    }
    // store this wave's gradients into its row of the workgroup's per-wave buffer (packed
    // plain layout; every index of the MLP written by exactly one lane)
    template <bool TWO>
    __device__ void flush(T* acc, int lane, bool folded) {
        if constexpr (sizeof(T) == 4) {
            if (!folded) fold();
        } else {
            for (int j = 0; j < 2; ++j) {             // the factored-out W2 and relu's linear half
                gw1a[j] *= w2[j];
                gw1b[j] *= w2[j];
                gb1[j] *= w2[j];
                gw2[j] += (w1a[j] * sx0 + w1b[j] * sx1 + b1[j] * gb2) * 0.5;
            }
        }
        for (int j = 0; j < 2; ++j) {
            const int k = lane + 64 * j;
            if constexpr (TWO) {
                acc[k] = gw1a[j]; acc[128 + k] = gw1b[j]; acc[256 + k] = gb1[j]; acc[384 + k] = gw2[j];
            } else {
                acc[k] = gw1a[j]; acc[128 + k] = gb1[j]; acc[256 + k] = gw2[j];
            }
        }
        if (lane == 0) acc[TWO ? 512 : 384] = gb2;
    }
};

// The syndrome loss fused into the reverse pass (y non-null): instead of reading d loss /
// d p from gnnd_syndrome_loss, each workgroup computes the loss terms of its codeword's
// component (check rows of the component graph; logical rows = per-variable bit masks, every
// row's support inside one component) and their gradient itself, and writes the component's
// loss to loss_b[b * ncomp + k].  Same per-row and per-variable summation orders as
// syndrome_loss_kernel except the logical rows (summed in variable order here).
template <typename T> struct BwdLoss {
    const T* y;                  // [B*V] labels (nullptr: gp holds d loss / d p)
    const uint32_t* lmask;       // [V] logical-row bit masks of the WHOLE graph's variables
    int nl, logical_only, ncomp;
    T* loss_b;                   // [B * ncomp]
};
// Split graphs (views non-null): blocks [k*cblk, (k+1)*cblk) run component k (graph views[k],
// rows addressed through its GraphView addressing fields) of codewords j, j + cblk, ...
template <typename T, int kTrainThreads = train_threads<T>(), int kMinWaves = 1, bool kSibs = true>
__global__ void __launch_bounds__(kTrainThreads, kMinWaves)   // kMinWaves: per SIMD
v24_bwd_kernel(GraphView g0, const T* __restrict__ w, const T* __restrict__ x,
               const T* __restrict__ p, const T* __restrict__ gp, TapeView<T> tape,
               T* __restrict__ gpart, int64_t B, int iters, const GraphView* __restrict__ views,
               int cblk, BwdLoss<T> lossp, int) {
    // kSibs: the sibling tables (checks and variables of degree <= 4) and the leave-one-out
    // phases folded into per-wave prologues; a compile-time switch so each instantiation keeps
    // one iteration loop (two loops in one kernel spilled the 16-wave shape's registers)
    constexpr bool sibs = kSibs;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    GNND_PPROF(pf);
    GNND_PSTART(pf, blockIdx.x == 0 && (GNND_PPROF_ALLWAVES || threadIdx.x < 64));
    GraphView g = g0;
    int blk = blockIdx.x, nblk = gridDim.x, comp = 0;
    if (views) {                       // uniform: component k
        comp = blk / cblk;
        g = views[comp];
        blk -= comp * cblk;
        nblk = cblk;
    }
    const int V = g.V, C = g.C, E = g.E;
    constexpr int kTrainWaves = kTrainThreads / 64;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // uniform: edge loops on SALU
#ifndef GNND_BWD_PARK
#define GNND_BWD_PARK 1
#endif
    constexpr bool kParkF32 = sizeof(T) == 4 && GNND_BWD_PARK;
    // fp64: the Softplus table (kSgTab; kSpTab in GNND_BWD_SGTAB=0 builds) at LDS byte 0 (sph_and_grad_n)
    constexpr size_t kTabB = bwd_tab_bytes<T>();
    T* s_ftab = (T*)smem;
    int* s_tab = (int*)(smem + kTabB);
    const int nints = graph_table_ints(V, C, E);
    const uint32_t* s_evc = (const uint32_t*)s_tab;
    const int* s_vptr = s_tab + E;
    const int* s_cptr = s_vptr + V + 1;
    const int* s_cedge = s_cptr + C + 1;
    size_t off = kTabB + (((size_t)nints * 4 + 15) & ~(size_t)15);
    // per-edge arrays at a 4-aligned stride Ep (the fp32 unit passes read four consecutive
    // edges with one ds_read_b128; entries E..Ep-1 stay zero: finite inputs, dy = 0)
    const int Ep = (E + 3) & ~3;
    T* s_dm = (T*)(smem + off);              // [E] d loss / d m (current iteration)
    T* s_g = s_dm + Ep;                      // [E] du, then dext
    T* s_da = s_g + Ep;                      // [E] d a
    T* s_u = s_da + Ep;                      // [E] tape of the iteration: u, t, ext
    T* s_t = s_u + Ep;
    T* s_ext = s_t + Ep;
    T* s_xv = s_ext + Ep;                    // [E] x_{v(e)}  (prior of the edge's variable)
    T* s_sc = s_xv + Ep;                     // [E] s_{c(e)}  (syndrome of the edge's check)
    T* s_ge = s_sc + Ep;                     // [E] dext (sibling path: pass C's output)
    // fused loss (lossp.y): [V] y + p, p, d loss / d p; [C + nl] row gradients, row terms;
    // int [V] logical masks, [nl] row lengths, [nl][V] row variable lists
    const bool floss = lossp.y != nullptr;
    const int nl = floss ? lossp.nl : 0, nr = C + nl;
    T* s_ls = s_ge + Ep;
    T* s_pv = s_ls + V;
    T* s_gpv = s_pv + V;
    T* s_lg = s_gpv + V;
    T* s_lt = s_lg + nr;
    uint32_t* s_lmask = (uint32_t*)(s_lt + nr);
    int* s_lcnt = (int*)(s_lmask + V);
    int* s_lvar = s_lcnt + nl;
    // sibs (checks and variables of degree <= 4): per edge its check's edges (cedge order) and
    // its variable's edges (var_ptr order), -1 padded: [E][8] ints built once per launch, so
    // the leave-one-out phases read their operands in two LDS round trips instead of walking
    // evc -> ptr -> edge chains
    // (after the fused-loss arrays when they exist, else right after the per-edge arrays; offset
    // arithmetic on the __shared__ base keeps ds_* accesses)
    const char* sib_end = floss ? (const char*)(s_lvar + (size_t)nl * V) : (const char*)s_ls;
    int* s_sib = (int*)(smem + (((sib_end - smem) + 15) & ~(ptrdiff_t)15));
    // fp32: the three MLPs' parked pass constants [3][10][64] after the sibling tables (or where
    // they would start; train_lds reserves it; dead before the gradient flush reuses the space)
    float* s_wp = (float*)(smem + (((((const char*)s_sib - smem) + (sibs ? 32 * (ptrdiff_t)E : 0)) + 15) &
                                   ~(ptrdiff_t)15));

    const int* gtab = (const int*)g.edge_vc;
    Units<T> uv, uc, uo;                     // ggc1.mlp, ggc2.mlp, mlp
    uv.load2(w + kV24Ggc1, lane);
    uc.load1(w + kV24Ggc2, lane);
    uo.load1(w + kV24Mlp, lane);
    if constexpr (kParkF32) {
        if (wave == 0) {
            uv.park(s_wp, lane);
            uc.park(s_wp + 640, lane);
            uo.park(s_wp + 1280, lane);
        }
    }
    for (int i = tid; i < nints; i += kTrainThreads) s_tab[i] = gtab[i];
    if constexpr (kTabB > 0)
        for (int i = tid; i < kBwdTabDoubles; i += kTrainThreads) s_ftab[i] = bwd_tab_entry(i);
    for (int i = tid; i < 9 * (Ep - E); i += kTrainThreads) s_dm[(i / (Ep - E)) * Ep + E + i % (Ep - E)] = T(0);
    if (floss) {
        for (int v = tid; v < V; v += kTrainThreads) s_lmask[v] = nl > 0 ? lossp.lmask[g.o0 + v] : 0u;
        __syncthreads();
        // logical row l as the list of its (local) variables, increasing: wave l, ballots
        for (int l = wave; l < nl; l += kTrainWaves) {
            int cnt = 0;
            for (int v0 = 0; v0 < V; v0 += 64) {
                const int v = v0 + lane;
                const bool in = v < V && ((s_lmask[v] >> l) & 1u);
                const uint64_t bal = __ballot(in);
                if (in) s_lvar[l * V + cnt + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                               __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u))] = v;
                cnt += __builtin_popcountll(bal);
            }
            if (lane == 0) s_lcnt[l] = cnt;
        }
    }
    __syncthreads();
    if (sibs) {
        for (int f = tid; f < E; f += kTrainThreads) {
            const uint32_t vc = s_evc[f];
            const int c = (int)(vc >> 16), v = (int)(vc & 0xffffu);
            const int c0 = s_cptr[c], cn = s_cptr[c + 1] - c0;
            const int v0 = s_vptr[v], vn = s_vptr[v + 1] - v0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                s_sib[8 * f + j] = j < cn ? s_cedge[c0 + j] : -1;
                s_sib[8 * f + 4 + j] = j < vn ? v0 + j : -1;
            }
        }
        __syncthreads();
    }
    GNND_PMARK(pf, 12);

    // unit-parallel pass over the codeword's edges, two per wave step:
    // out[f] = d/d in of MLP at (in0[f], in1[f]) for upstream dy(f)
    // The uniform results of step k go to lane k of two VGPRs (compare + select), stored by the
    // lanes after every 64 steps (no per-step exec-masked lane-0 stores).
    // issue fairness between the waves of a SIMD in the unit passes (GNND_BWD_FAIR, default 1): the
    // arbiter issues oldest-first, so a SIMD's older wave finishes its share of a pass well before
    // the younger ones, which then run alone with their latencies exposed (per-wave phase
    // profile r05h: fp64 pass A 145k vs 233k cycles, fp32 38k / 57k / 80k / 99k by age).  Each
    // wave lowers its priority as it completes its steps (3 -> 1 over the pass), so a lagging
    // wave takes the issue slots until it has caught up.  Same-box A/B (r05j): config-5 step at
    // B = 128 fp32 0.1801 -> 0.1773 ms, fp64 0.3926 -> 0.3888 ms.
#ifndef GNND_BWD_FAIR
#define GNND_BWD_FAIR 1
#endif
    const int nsteps4 = ((E + 3) / 4 + kTrainWaves - 1) / kTrainWaves;   // wave steps per pass
    auto fair_prio = [&](int k) {
        if constexpr (GNND_BWD_FAIR) {
            const int q = 3 * k / nsteps4;               // wave-uniform
            if (q == 0) __builtin_amdgcn_s_setprio(3);
            else if (q == 1) __builtin_amdgcn_s_setprio(2);
            else __builtin_amdgcn_s_setprio(1);
        }
    };
    auto fair_end = [&]() {
        if constexpr (GNND_BWD_FAIR) __builtin_amdgcn_s_setprio(0);
    };
    auto unit_pass = [&](auto& U, auto two_tag, const T* in0, const T* in1, auto dy_of, auto dy4_of,
                         T* outp) {
        constexpr bool TWO = decltype(two_tag)::value;
        if constexpr (sizeof(T) == 4) {
            // fp32: four edges f + i W (i = 0..3) per wave step, one shared reduction; the next
            // step's inputs are read from LDS before this step's unit work (latency hidden)
            constexpr int W = kTrainWaves, kStride4 = 4 * kTrainWaves;
            // 8-wave workgroups (256 VGPRs per lane): the per-half partials are pass-local and the
            // next step's inputs are read ahead; 16-wave ones (128 VGPRs) keep every MLP's
            // partials resident and read each step's inputs in place (no register spills)
            constexpr bool kPipe = kTrainThreads <= 512 && kMinWaves == 1;
            if constexpr (kPipe) U.zero_pg();
            auto load = [&](int f, float (&a0)[4], float (&a1)[4], float (&dy)[4]) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int fi = f + i * W;
                    const bool ok = fi < E;
                    const int fc = ok ? fi : f;
                    a0[i] = in0[fc];
                    a1[i] = TWO ? in1[fc] : 0.f;
                    dy[i] = ok ? dy_of(fc) : 0.f;
                }
            };
            for (int f0 = wave; f0 < E; f0 += 64 * kStride4) {
                float res[4] = {0.f, 0.f, 0.f, 0.f};
                int k = 0;
                if constexpr (kPipe) {
                    float a0[4], a1[4], dy[4];
                    load(f0, a0, a1, dy);
                    for (int f = f0; f < E && k < 64; f += kStride4, ++k) {
                        float b0[4], b1[4], dyn[4], r[4];
                        const int fn = f + kStride4;
                        if (fn < E && k + 1 < 64) load(fn, b0, b1, dyn);   // wave-uniform
                        U.template bwd4_f32<TWO>(a0, a1, dy, r);
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            res[i] = put_lane(res[i], r[i], k, lane);
                            a0[i] = b0[i];
                            a1[i] = b1[i];
                            dy[i] = dyn[i];
                        }
                    }
                } else {
                    // four CONSECUTIVE edges f..f+3 per wave step (f = 4 (wave + W k)): one
                    // ds_read_b128 per input array, the pairs {f, f+1}, {f+2, f+3} straight into
                    // the packed halves; the row-reduced d input stored by one lane per row
                    // the per-half partials are pass-local here too (zero_pg / fold around the
                    // pass): only the active MLP's 16 partial VGPRs live, not all three MLPs' 48
                    const int eo = row_edge(lane >> 4);
                    U.zero_pg();
                    for (int f = 4 * f0, ks = 0; f < E; f += 4 * kTrainWaves, ++ks) {
                        fair_prio(ks);
                        const f32x4 v0 = *(const f32x4*)(in0 + f);
                        const f32x4 v1 = TWO ? *(const f32x4*)(in1 + f) : f32x4{0.f, 0.f, 0.f, 0.f};
                        const float r = U.template bwd4_rows<TWO>(v0, v1, dy4_of(f));
                        // every lane stores its row's total (16 identical writes per
                        // address, no exec-masked region inside the hot loop; f + eo < Ep, and
                        // the padding entries only ever meet dy = 0)
#ifdef GNND_W2_MASKED_STORE
                        // r03r experiment form (one lane per row stores under an exec mask)
                        if ((lane & 15) == 0) outp[f + eo] = r;
#else
                        outp[f + eo] = r;
#endif
                    }
                    U.fold();
                    fair_end();
                    break;                       // (one pass covers every edge)
                }
                const int fl = f0 + kStride4 * lane;
                if (kPipe && lane < k) {
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        if (fl + i * W < E) outp[fl + i * W] = res[i];
                }
            }
            if constexpr (kPipe) U.fold();
            return;
        }
        if constexpr (sizeof(T) == 8) {
            // fp64: four consecutive edges f..f+3 per wave step (f = 4 (wave + W k)); padding
            // entries E..Ep-1 are zero inputs with dy = 0, and every lane stores its row's total
            const int eo = row_edge(lane >> 4);
            for (int f = 4 * wave, ks = 0; f < E; f += 4 * kTrainWaves, ++ks) {
                fair_prio(ks);
                double a0[4], a1[4], dy[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    a0[i] = in0[f + i];
                    a1[i] = TWO ? in1[f + i] : 0.0;
                    dy[i] = dy_of(f + i);
                }
                outp[f + eo] = U.template bwd4_rows_f64<TWO>(a0, a1, dy, s_ftab);
            }
            fair_end();
        }
    };

    // the iteration's tape rows: the first kPF per thread are loaded into registers one
    // iteration ahead (their HBM latency hides behind the previous iteration's phases)
    constexpr int kPF = 1;
    T pu[kPF], pt[kPF], pe[kPF];
    // persistent over codewords b = blockIdx.x, blockIdx.x + gridDim.x, ...: the lanes'
    // gradient registers accumulate across all of them (one partial row per workgroup, any
    // batch size, LDS independent of B)
    for (int64_t b = blk; b < B; b += nblk) {
        auto prefetch = [&](int it) {
            const size_t trow = ((size_t)it * B + b) * g.es + g.e0;
#pragma unroll
            for (int i = 0; i < kPF; ++i) {
                const int f = tid + i * kTrainThreads;
                if (f < E) { pu[i] = tape.u[trow + f]; pt[i] = tape.t[trow + f]; pe[i] = tape.ext[trow + f]; }
            }
        };
        auto stage = [&](int it) {
#pragma unroll
            for (int i = 0; i < kPF; ++i) {
                const int f = tid + i * kTrainThreads;
                if (f < E) { s_u[f] = pu[i]; s_t[f] = pt[i]; s_ext[f] = pe[i]; }
            }
            const size_t trow = ((size_t)it * B + b) * g.es + g.e0;
            for (int f = tid + kPF * kTrainThreads; f < E; f += kTrainThreads) {
                s_u[f] = tape.u[trow + f];
                s_t[f] = tape.t[trow + f];
                s_ext[f] = tape.ext[trow + f];
            }
        };
        if (iters > 0) prefetch(iters - 1);
        // readout inputs: m^T into s_u, d loss / d r per edge into s_da; per-edge x_v, s_c
        const T* xb = x + (size_t)b * g.xs;
        if (floss) {
            // quantum/decoder_v2_4.py:297-317 on this component: s = y + p; rows -> |sin| terms
            // and d|sin(pi/2 s_r)| / d s_r; d loss / d p_v = sum over v's rows
            const size_t ob = (size_t)b * g.os + g.o0;
            for (int v = tid; v < V; v += kTrainThreads) {
                const T pv = p[ob + v];
                s_pv[v] = pv;
                s_ls[v] = lossp.y[ob + v] + pv;
            }
            GNND_PMARK(pf, 13);
            __syncthreads();
            GNND_PMARK(pf, 14);
            const T kPi = T(M_PI);
            for (int r = tid; r < nr; r += kTrainThreads) {
                T sr = T(0);
                if (r < C) {
                    for (int k = s_cptr[r]; k < s_cptr[r + 1]; ++k) sr += s_ls[s_evc[s_cedge[k]] & 0xffffu];
                } else {
                    const int l = r - C;
                    for (int i = 0; i < s_lcnt[l]; ++i) sr += s_ls[s_lvar[l * V + i]];
                }
                const T xr = sr * kPi / T(2);
                const T sn = sin(xr);
                const T gr = (sn > T(0) ? T(1) : sn < T(0) ? T(-1) : T(0)) * cos(xr) * (kPi / T(2));
                const bool on = r >= C || !lossp.logical_only;
                s_lg[r] = on ? gr : T(0);
                s_lt[r] = on ? (sn < T(0) ? -sn : sn) : T(0);
            }
            GNND_PMARK(pf, 15);
            __syncthreads();
            for (int v = tid; v < V; v += kTrainThreads) {
                T d = T(0);
                for (int k = s_vptr[v]; k < s_vptr[v + 1]; ++k) d += s_lg[s_evc[k] >> 16];
                const uint32_t m = s_lmask[v];
                for (int l = 0; l < nl; ++l)
                    if ((m >> l) & 1u) d += s_lg[C + l];
                s_gpv[v] = d;
            }
            if (wave == 0) {                  // the component's loss, fixed order
                T t = T(0);
                for (int r = lane; r < nr; r += 64) t += s_lt[r];
                t = wave_sum(t);
                if (lane == 0) lossp.loss_b[(size_t)b * lossp.ncomp + comp] = t;
            }
            __syncthreads();
        }
        for (int f = tid; f < E; f += kTrainThreads) {
            const uint32_t vc = s_evc[f];
            const int v = (int)(vc & 0xffffu);
            const size_t bv = (size_t)b * g.os + g.o0 + v;
            const T pv = floss ? s_pv[v] : p[bv];
            const T gv = floss ? s_gpv[v] : gp[bv];
            s_xv[f] = xb[g.xv0 + v];
            s_sc[f] = xb[g.xc0 + (int)(vc >> 16)];
            s_u[f] = tape.mT[(size_t)b * g.es + g.e0 + f];
            s_da[f] = -((gv * (T(1) - pv)) * pv);     // p = sigmoid(-r)
        }
        GNND_PMARK(pf, 19);
        __syncthreads();

        // readout: r_v = sum_e MLP_o(m^T_e) + x_v  ->  dm
        auto ld4 = [](const T* a, int f) -> f32x4 {
            if constexpr (sizeof(T) == 4) return *(const f32x4*)(a + f);
            else return f32x4{0.f, 0.f, 0.f, 0.f};
        };
        GNND_PMARK(pf, 0);
        if constexpr (kParkF32) uo.unpark(s_wp + 1280, lane);
        unit_pass(uo, std::false_type{}, s_u, nullptr, [&](int f) { return s_da[f]; },
                  [&](int f) { return ld4(s_da, f); }, s_dm);
        __syncthreads();
        GNND_PMARK(pf, 1);

#ifndef GNND_BWD_EXP
#define GNND_BWD_EXP 0   // timing experiments only (wrong gradients): 1 no LOO compute,
#endif                   // 2 no LOO phases or their barriers, 3 no unit passes
        // With the sibling tables the two leave-one-out phases need no edge-parallel phase and
        // no barrier of their own: each wave first forms, lane-parallel, the values of the edges
        // its own unit-pass steps will read (phase D's dm += S_v(dext) - dext before pass A,
        // phase B's da = ((S_c(du) - du)(1 - t^2)) / 2 before pass C), and LDS keeps a wave's
        // accesses in order, so its unit pass sees them.  du and dext live in separate buffers
        // (s_g, and s_da's twin s_ge) so a prologue never reads what another wave's pass of the
        // same phase writes.  The same operations in the same order as the phases: bit-identical.
        if constexpr (sibs) {
            // the unit pass's edge set of this wave: four consecutive edges per step (fp32
            // 16-wave shape, fp64) or edges = wave mod W (fp32 pipelined 8-wave shape)
            constexpr bool kPipeSet = sizeof(T) == 4 && kTrainThreads <= 512 && kMinWaves == 1;
            auto my_edge = [&](int j) -> int {
                return kPipeSet ? wave + kTrainWaves * j : 4 * (wave + kTrainWaves * (j >> 2)) + (j & 3);
            };
            for (int it = iters - 1; it >= 0; --it) {
                stage(it);
                __syncthreads();
                GNND_PMARK(pf, 2);
                if (it > 0) prefetch(it - 1);
                if (it < iters - 1) {          // D of the previous step, for this wave's edges
                    for (int j = lane;; j += 64) {
                        const int f = my_edge(j);
                        if (f >= E) break;
                        T sv = T(0);
                        const int4 vs = *(const int4*)(s_sib + 8 * f + 4);
                        const T g0 = s_ge[vs.x < 0 ? 0 : vs.x], g1 = s_ge[vs.y < 0 ? 0 : vs.y];
                        const T g2 = s_ge[vs.z < 0 ? 0 : vs.z], g3 = s_ge[vs.w < 0 ? 0 : vs.w];
                        if (vs.x >= 0) sv += g0;
                        if (vs.y >= 0) sv += g1;
                        if (vs.z >= 0) sv += g2;
                        if (vs.w >= 0) sv += g3;
                        s_dm[f] += sv - s_ge[f];
                    }
                }
                GNND_PMARK(pf, 9);
                // A: m^{t+1} = MLP_c(u) s_c + m^t
                if constexpr (kParkF32) uc.unpark(s_wp + 640, lane);
                unit_pass(uc, std::false_type{}, s_u, nullptr, [&](int f) { return s_dm[f] * s_sc[f]; },
                          [&](int f) { return ld4(s_dm, f) * ld4(s_sc, f); }, s_g);
                GNND_PMARK(pf, 3);
                __syncthreads();
                GNND_PMARK(pf, 4);
                for (int j = lane;; j += 64) {   // B, for this wave's edges
                    const int f = my_edge(j);
                    if (f >= E) break;
                    T sc = T(0);
                    const int4 cs = *(const int4*)(s_sib + 8 * f);
                    const T g0 = s_g[cs.x < 0 ? 0 : cs.x], g1 = s_g[cs.y < 0 ? 0 : cs.y];
                    const T g2 = s_g[cs.z < 0 ? 0 : cs.z], g3 = s_g[cs.w < 0 ? 0 : cs.w];
                    if (cs.x >= 0) sc += g0;
                    if (cs.y >= 0) sc += g1;
                    if (cs.z >= 0) sc += g2;
                    if (cs.w >= 0) sc += g3;
                    const T t = s_t[f];
                    s_da[f] = ((sc - s_g[f]) * (T(1) - t * t)) / T(2);
                }
                GNND_PMARK(pf, 5);
                // C: a = MLP_v(ext, x_v)
                if constexpr (kParkF32) uv.unpark(s_wp, lane);
                unit_pass(uv, std::true_type{}, s_ext, s_xv, [&](int f) { return s_da[f]; },
                          [&](int f) { return ld4(s_da, f); }, s_ge);
                GNND_PMARK(pf, 7);
                __syncthreads();
                GNND_PMARK(pf, 8);
            }
        } else {
        for (int it = iters - 1; it >= 0; --it) {
            stage(it);
            __syncthreads();
            GNND_PMARK(pf, 2);
            if (it > 0) prefetch(it - 1);
            // A: m^{t+1} = MLP_c(u) s_c + m^t
            if (GNND_BWD_EXP != 3)
            {
                if constexpr (kParkF32) uc.unpark(s_wp + 640, lane);
                unit_pass(uc, std::false_type{}, s_u, nullptr, [&](int f) { return s_dm[f] * s_sc[f]; },
                          [&](int f) { return ld4(s_dm, f) * ld4(s_sc, f); }, s_g);
            }
            GNND_PMARK(pf, 3);
            __syncthreads();
            GNND_PMARK(pf, 4);
            // B: u = S_c(t) - t  ->  dt = S_c(du) - du;  t = tanh(a/2)
            for (int f = tid; f < E; f += kTrainThreads) {
                T s = T(0);
                if (sibs) {           // the same order: the check's edges in cedge order
                    const int4 cs = *(const int4*)(s_sib + 8 * f);
                    const T g0 = s_g[cs.x < 0 ? 0 : cs.x], g1 = s_g[cs.y < 0 ? 0 : cs.y];
                    const T g2 = s_g[cs.z < 0 ? 0 : cs.z], g3 = s_g[cs.w < 0 ? 0 : cs.w];
                    if (cs.x >= 0) s += g0;
                    if (cs.y >= 0) s += g1;
                    if (cs.z >= 0) s += g2;
                    if (cs.w >= 0) s += g3;
                } else {
                    const int c = (int)(s_evc[f] >> 16);
                    if (GNND_BWD_EXP == 0 || GNND_BWD_EXP == 3)
                        for (int k = s_cptr[c], ke = s_cptr[c + 1]; k < ke; ++k) s += s_g[s_cedge[k]];
                }
                const T t = s_t[f];
                s_da[f] = ((s - s_g[f]) * (T(1) - t * t)) / T(2);
            }
            GNND_PMARK(pf, 5);
            if (GNND_BWD_EXP != 2) __syncthreads();
            GNND_PMARK(pf, 6);
            // C: a = MLP_v(ext, x_v)
            if (GNND_BWD_EXP != 3)
            {
                if constexpr (kParkF32) uv.unpark(s_wp, lane);
                unit_pass(uv, std::true_type{}, s_ext, s_xv, [&](int f) { return s_da[f]; },
                          [&](int f) { return ld4(s_da, f); }, s_g);
            }
            GNND_PMARK(pf, 7);
            __syncthreads();
            GNND_PMARK(pf, 8);
            // D: ext = S_v(m) - m  ->  dm += S_v(dext) - dext  (variable edges are contiguous)
            for (int f = tid; f < E; f += kTrainThreads) {
                T s = T(0);
                if (sibs) {           // the same order: the variable's edges ascending
                    const int4 vs = *(const int4*)(s_sib + 8 * f + 4);
                    const T g0 = s_g[vs.x < 0 ? 0 : vs.x], g1 = s_g[vs.y < 0 ? 0 : vs.y];
                    const T g2 = s_g[vs.z < 0 ? 0 : vs.z], g3 = s_g[vs.w < 0 ? 0 : vs.w];
                    if (vs.x >= 0) s += g0;
                    if (vs.y >= 0) s += g1;
                    if (vs.z >= 0) s += g2;
                    if (vs.w >= 0) s += g3;
                } else {
                    const int v = (int)(s_evc[f] & 0xffffu);
                    if (GNND_BWD_EXP == 0 || GNND_BWD_EXP == 3)
                        for (int k = s_vptr[v], ke = s_vptr[v + 1]; k < ke; ++k) s += s_g[k];
                }
                s_dm[f] += s - s_g[f];
            }
            GNND_PMARK(pf, 9);
            if (GNND_BWD_EXP != 2) __syncthreads();
            GNND_PMARK(pf, 10);
        }
        }
    }

    // workgroup gradient: every wave stores its gradients into its own row of a per-wave
    // buffer (aliasing the per-edge arrays, dead now), then each parameter is summed over the
    // waves in wave order from 0 (deterministic; the same bits as adding the waves one by one
    // into a zeroed accumulator) — one barrier instead of one per wave
    T* s_red = s_dm;                         // [kTrainWaves][kV24W] (train_lds reserves it)
    __syncthreads();
    GNND_PMARK(pf, 16);
    {
        constexpr bool kFolded = true;       // fp32: every unit_pass folds its partials
        T* my = s_red + (size_t)wave * kV24W;
        uv.template flush<true>(my + kV24Ggc1, lane, kFolded);
        uc.template flush<false>(my + kV24Ggc2, lane, kFolded);
        uo.template flush<false>(my + kV24Mlp, lane, kFolded);
    }
    GNND_PMARK(pf, 17);
    __syncthreads();
    GNND_PMARK(pf, 18);
    T* row = gpart + (size_t)blockIdx.x * kV24W;
    for (int i = tid; i < kV24W; i += kTrainThreads) {
        T a = T(0);
#pragma unroll
        for (int wv = 0; wv < kTrainWaves; ++wv) a += s_red[(size_t)wv * kV24W + i];
        row[i] = a;
    }
    GNND_PMARK(pf, 11);
    GNND_PREPORT(pf, "bwd", kTrainThreads, iters);
}

// sum of the per-workgroup rows, fixed order (8 interleaved partial chains, then combined)
template <typename T>
__global__ void grad_reduce_kernel(const T* __restrict__ gpart, int rows, T* __restrict__ gw,
                                   int n = kV24W) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    T s[8] = {};
    int r = 0;
    for (; r + 8 <= rows; r += 8)
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] += gpart[(size_t)(r + j) * n + i];
    for (int j = 0; r < rows; ++r, ++j) s[j] += gpart[(size_t)r * n + i];
    gw[i] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
}

// fp32 reverse-pass workgroup shape: 1024 = 16 waves, one workgroup per CU; 5122 = 8 waves,
// two workgroups per CU; 2564 = 4 waves, four per CU (all 128 VGPRs, 4 waves per SIMD);
// 512 = 8 waves with 256 VGPRs.  Default by grid: the 16-wave shape while the workgroups do
// not fill the CUs twice (B = 128: 0.274 vs 0.284 ms/step for 5122), the two-per-CU shape
// above (B = 8 192: 9.29 vs 10.09 ms, r03o: independent barriers hide each other's phases).
// GNND_TRAIN_THREADS forces one (A/B).
int train_threads_f32(int64_t blocks) {
    static int forced = [] {
        const char* e = gnnd_tune_env("GNND_TRAIN_THREADS");
        const int n = e ? atoi(e) : 0;
        return n == 512 || n == 5122 || n == 2564 || n == 1024 ? n : 0;
    }();
    if (forced) return forced;
    return blocks >= 2 * (int64_t)device_cus() ? 5122 : 1024;
}
// workgroups of the reverse pass: one codeword each up to 1024 (the partial-row count),
// larger batches loop (each workgroup a fixed, strided set of codewords: deterministic)
constexpr int64_t kTrainMaxBlocks = 1024;
int64_t train_blocks(int64_t B) { return B < kTrainMaxBlocks ? B : kTrainMaxBlocks; }
// the reverse pass on a split graph: each component of a codeword in its own workgroup
bool train_split(const gnnd_graph* g, int64_t B) {
    return g->ncomp > 1 && g->dcomp && !g->nosplit && !split_disabled() && split_pays(B);
}
// workgroups per component and in all (<= kTrainMaxBlocks gradient rows)
int64_t train_cblk(const gnnd_graph* g, int64_t B) {
    if (!train_split(g, B)) return train_blocks(B);
    const int64_t per = kTrainMaxBlocks / g->ncomp;
    return B < per ? B : per;
}
int64_t train_rows(const gnnd_graph* g, int64_t B) {
    return train_split(g, B) ? train_cblk(g, B) * g->ncomp : train_blocks(B);
}
// waves: the workgroup's waves (the final per-wave gradient buffer aliases the arrays after
// the graph tables: [waves][kV24W] values)
size_t train_lds(const gnnd_graph* g, int esz, int nl = -1, int waves = 0, bool sibs = false) {   // nl >= 0: fused loss
    const GraphView& v = g->view;
    const size_t tab = (esz == 8 ? bwd_tab_bytes<double>() : 0) +
                       (((size_t)graph_table_ints(v.V, v.C, v.E) * 4 + 15) & ~(size_t)15);
    size_t n = tab + (size_t)esz * 9 * (((size_t)v.E + 3) & ~(size_t)3);
    if (nl >= 0)
        n += (size_t)esz * (3 * (size_t)v.V + 2 * ((size_t)v.C + nl)) +
             4 * ((size_t)v.V + nl + (size_t)nl * v.V);
    if (sibs) n = ((n + 15) & ~(size_t)15) + 32 * (size_t)v.E;
    if (esz == 4) n = ((n + 15) & ~(size_t)15) + (size_t)3 * 10 * 64 * 4;   // parked constants
    const size_t red = tab + (size_t)esz * waves * kV24W;
    return n > red ? n : red;
}
// the sibling tables of the leave-one-out phases: checks and variables of degree <= 4, and room
bool train_sibs(const gnnd_graph* g, int esz, int nl, int waves) {
    const GraphView& v = g->view;
    return v.max_dc <= 4 && v.max_dv <= 4 && train_lds(g, esz, nl, waves, true) <= 160 * 1024;
}

// gw == nullptr: leave the per-workgroup partial rows in ws (gnnd_train_bwd_partial);
// lossp.y non-null: the syndrome loss fused in (gnnd_train_bwd_loss_partial)
template <typename T>
int launch_bwd(const gnnd_graph* g, const void* w, const void* x, const void* out,
               const void* gout, const void* tape, void* gw, void* ws, int64_t ws_bytes,
               int64_t B, int iters, hipStream_t st, BwdLoss<T> lossp = {}) {
    const bool split = train_split(g, B);
    const gnnd_graph* gk = split ? g->comp[0] : g;        // components share one shape
    const int64_t cblk = train_cblk(g, B), blocks = train_rows(g, B);
    if ((int64_t)blocks * kV24W * (int64_t)sizeof(T) > ws_bytes) return GNND_ERR_INVALID_ARG;
    lossp.ncomp = split ? g->ncomp : 1;
    // fp32: 16 waves (128 VGPRs) by default, GNND_TRAIN_THREADS=512 for 8 waves (A/B)
    const int shape = sizeof(T) == 4 ? train_threads_f32(blocks) : 0;
    // (5122: two 8-wave workgroups per CU = 4 waves per SIMD, 128 VGPRs; 2564: four 4-wave ones)
    const int nthreads = shape == 512 || shape == 5122 ? 512 : shape == 2564 ? 256 : train_threads<T>();
    const int nlf = lossp.y ? lossp.nl : -1;
    const bool sibs = train_sibs(gk, sizeof(T), nlf, nthreads / 64);
    auto kern = sibs ? (shape == 512 ? v24_bwd_kernel<T, 512> : shape == 5122 ? v24_bwd_kernel<T, 512, 4>
                        : shape == 2564 ? v24_bwd_kernel<T, 256, 4> : v24_bwd_kernel<T>)
                     : (shape == 512 ? v24_bwd_kernel<T, 512, 1, false>
                        : shape == 5122 ? v24_bwd_kernel<T, 512, 4, false>
                        : shape == 2564 ? v24_bwd_kernel<T, 256, 4, false>
                        : v24_bwd_kernel<T, train_threads<T>(), 1, false>);
    const size_t lds = train_lds(gk, sizeof(T), nlf, nthreads / 64, sibs);
    if (lds > 160 * 1024) return GNND_ERR_UNSUPPORTED;
    if (lds > 64 * 1024)
        GNND_HIP_CHECK(hipFuncSetAttribute((const void*)kern,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    const size_t n = (size_t)iters * B * g->view.E;
    T* base = (T*)tape;
    TapeView<T> tv{base, base + n, base + 2 * n, base + 3 * n};
    kern<<<(unsigned)blocks, nthreads, lds, st>>>(
        gk->view, (const T*)w, (const T*)x, (const T*)out, (const T*)gout, tv, (T*)ws, B, iters,
        split ? g->dcomp : nullptr, (int)cblk, lossp, sibs ? 1 : 0);   // dcomp[0..K): the components' `view`
    GNND_LAUNCH_CHECK();
    if (!gw) return GNND_OK;
    grad_reduce_kernel<T><<<(kV24W + 255) / 256, 256, 0, st>>>((const T*)ws, (int)blocks, (T*)gw);
    GNND_LAUNCH_CHECK();
    return GNND_OK;
}

bool is_wbp_train(int model) { return model == GNND_NBP || model == GNND_V22 || model == GNND_V10; }
// the 10-hidden-unit GNN decoders (CGNNI, QGNNI): gnnd_train_gnn.hip
bool is_gnn_train(int model) { return model == GNND_CGNNI || model == GNND_QGNNI; }
bool train_args_ok(const gnnd_graph* g, int model, int dtype, int64_t B, int32_t iters) {
    if (!g || B < 0 || iters < 0) return false;
    if (is_wbp_train(model)) return dtype == GNND_F64;       // the scripts' dtype only
    return (model == GNND_V24 || model == GNND_V30 || is_gnn_train(model)) &&
           (dtype == GNND_F32 || dtype == GNND_F64);
}
// per-edge weight tables of the weighted-BP models (gnnd.h NBP / V22 / V10 layouts)
int64_t wbp_weights(const gnnd_graph* g, int model, int iters) {
    return gnnd_wbp_weights(g, model, iters);
}
// trainable weights of a fused-training model (the packed layout of gnnd.h)
int train_weights(int model) { return model == GNND_V30 ? kV30Count : is_gnn_train(model) ? 62 : kV24W; }
// gradient rows of the reverse pass
int64_t model_train_rows(const gnnd_graph* g, int model, int64_t B) {
    if (is_wbp_train(model)) return gnnd_wbp_train_rows(B);
    if (is_gnn_train(model)) return gnnd_gnn_train_rows(B);
    return model == GNND_V30 ? gnnd_v30_train_rows(B) : train_rows(g, B);
}

// ---------------------------------------------------------------------------------------
// syndrome loss of the quantum training scripts with its gradient
// ---------------------------------------------------------------------------------------
// quantum/decoder_v2_4.py:297-317 (QGNNI.py:255-290 with logical_only): per codeword
//   s = y + p;  loss = sum_c |sin(pi/2 (H^T s)_c)| + sum_l |sin(pi/2 (Lambda s)_l)|
//   d loss / d p_v = sum_{rows r containing v} (pi/2) cos(x_r) sign(sin(x_r)),  x_r = (s_r pi) / 2
// (torch: d|u|/du = sign(u), sign(0) = 0).  One wave per codeword: lanes over variables
// (s into LDS), lanes over rows (check rows from the graph CSR, logical rows from the dense
// 0/1 table) -> |sin| terms and row gradients in LDS, wave-reduced loss, lanes over
// variables for the gradient (variable CSR).  Replaces ~30 small torch kernels per step.
// The workgroup first stages the graph's row and column lists (check -> variables, variable
// -> checks) and the logical rows as per-variable bit masks in LDS, so the per-codeword
// gathers are LDS reads instead of chains of dependent global loads (a small training batch
// is latency-bound here: 13.9 us at B = 128 with global gathers).
template <typename T>
__global__ void __launch_bounds__(256)
syndrome_loss_kernel(GraphView g, const int32_t* __restrict__ lg, int nl, int logical_only,
                     const T* __restrict__ pred, const T* __restrict__ y, T* __restrict__ loss_b,
                     T* __restrict__ dpred, int64_t B) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int V = g.V, C = g.C, E = g.E;
    const int nr = C + nl;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    // graph image: chk_ptr[C+1], chk_var[E], var_ptr[V+1], var_chk[E], lmask[V]
    int* t_cptr = (int*)smem;
    int* t_cvar = t_cptr + C + 1;
    int* t_vptr = t_cvar + E;
    int* t_vchk = t_vptr + V + 1;
    uint32_t* t_lmask = (uint32_t*)(t_vchk + E);
    const size_t toff = ((size_t)(2 * E + C + 2 * V + 2) * 4 + 15) & ~(size_t)15;
    for (int i = threadIdx.x; i <= C; i += 256) t_cptr[i] = g.chk_ptr[i];
    for (int i = threadIdx.x; i <= V; i += 256) t_vptr[i] = g.var_ptr[i];
    for (int k = threadIdx.x; k < E; k += 256) {
        t_cvar[k] = (int)(g.edge_vc[g.chk_edge[k]] & 0xffffu);
        t_vchk[k] = (int)(g.edge_vc[k] >> 16);
    }
    for (int v = threadIdx.x; v < V; v += 256) {
        uint32_t m = 0;
        for (int l = 0; l < nl; ++l) m |= (lg[(size_t)l * V + v] != 0 ? 1u : 0u) << l;
        t_lmask[v] = m;
    }
    __syncthreads();
    T* s_s = (T*)(smem + toff) + (size_t)wave * (V + nr);
    T* s_g = s_s + V;
    const int64_t b = (int64_t)blockIdx.x * 4 + wave;
    if (b >= B) return;                          // whole wave exits (no block barrier below)
    const T* pb = pred + b * V;
    const T* yb = y + b * V;
    for (int v = lane; v < V; v += 64) s_s[v] = yb[v] + pb[v];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    T term = T(0);
    const T kPi = T(M_PI);
    auto row_grad = [&](T sr, int r, bool on) {     // |sin| term and d|sin(x_r)|/ds_r
        const T xr = sr * kPi / T(2);
        const T sn = sin(xr);
        const T gr = (sn > T(0) ? T(1) : sn < T(0) ? T(-1) : T(0)) * cos(xr) * (kPi / T(2));
        s_g[r] = on ? gr : T(0);
        if (on) term += sn < T(0) ? -sn : sn;
    };
    for (int r = lane; r < C; r += 64) {            // check rows: lanes over checks
        T sr = T(0);
        for (int k = t_cptr[r]; k < t_cptr[r + 1]; ++k) sr += s_s[t_cvar[k]];
        row_grad(sr, r, !logical_only);
    }
    for (int l = 0; l < nl; ++l) {                  // logical rows: the wave sums each one
        T part = T(0);
        for (int v = lane; v < V; v += 64)
            if ((t_lmask[v] >> l) & 1u) part += s_s[v];
        for (int o = 32; o >= 1; o >>= 1) part += __shfl_xor(part, o);
        if (lane == l % 64) row_grad(part, C + l, true);
    }
    // wave sum of the row terms, fixed butterfly order
    for (int o = 32; o >= 1; o >>= 1) term += __shfl_xor(term, o);
    if (lane == 0) loss_b[b] = term;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int v = lane; v < V; v += 64) {
        T d = T(0);
        for (int k = t_vptr[v]; k < t_vptr[v + 1]; ++k) d += s_g[t_vchk[k]];
        const uint32_t m = t_lmask[v];
        for (int l = 0; l < nl; ++l)
            if ((m >> l) & 1u) d += s_g[C + l];
        dpred[b * V + v] = d;
    }
}

template <typename T>
int launch_syndrome_loss(const gnnd_graph* g, const int32_t* lg, int nl, int logical_only,
                         const void* pred, const void* y, void* loss_b, void* dpred, int64_t B,
                         hipStream_t st) {
    const GraphView& v = g->view;
    if (nl > 32) return GNND_ERR_UNSUPPORTED;    // logical rows as per-variable bit masks
    const size_t tab = ((size_t)(2 * v.E + v.C + 2 * v.V + 2) * 4 + 15) & ~(size_t)15;
    const size_t lds = tab + 4 * (size_t)(v.V + v.C + nl) * sizeof(T);
    if (lds > 160 * 1024) return GNND_ERR_UNSUPPORTED;   // SyndromeLoss falls back to torch
    if (lds > 64 * 1024)
        GNND_HIP_CHECK(hipFuncSetAttribute((const void*)syndrome_loss_kernel<T>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    const int64_t blocks = (B + 3) / 4;
    syndrome_loss_kernel<T><<<(unsigned)blocks, 256, lds, st>>>(
        v, lg, nl, logical_only, (const T*)pred, (const T*)y, (T*)loss_b, (T*)dpred, B);
    GNND_LAUNCH_CHECK();
    return GNND_OK;
}

// ---------------------------------------------------------------------------------------
// hard-decision metrics: bit/frame error counts (the bench's BER/FER; the
// reference reports losses only) and the toric failure rule of quantum/neural_BP.py:333-348
// (residual syndrome failure, else logical failure) on the device, one wave per codeword,
// integer counts (atomics on integers: exact, order-free)
// ---------------------------------------------------------------------------------------
// counts[0] bit errors (pred > 0.5 != y), [1] codewords with a bit error, [2] codewords whose
// residual e = y xor hat(e) violates a check, [3] codewords with zero residual syndrome but
// odd overlap with a logical row
template <typename T>
__global__ void __launch_bounds__(256)
decision_errors_kernel(GraphView g, const int32_t* __restrict__ lg, int nl,
                       const T* __restrict__ pred, const T* __restrict__ y,
                       unsigned long long* __restrict__ counts, int64_t B) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int V = g.V, C = g.C;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint8_t* s_e = (uint8_t*)smem + (size_t)wave * ((V + 15) & ~15);
    // each wave loops over codewords (grid-stride) and keeps its counts in registers: one
    // set of atomics per wave, not per codeword (65 536 codewords on 4 addresses contended)
    unsigned long long c_bit = 0, c_frame = 0, c_syn = 0, c_log = 0;
    for (int64_t b = (int64_t)blockIdx.x * 4 + wave; b < B; b += (int64_t)gridDim.x * 4) {
        const T* pb = pred + b * V;
        const T* yb = y + b * V;
        int nerr = 0;
        for (int v = lane; v < V; v += 64) {
            const int e = (pb[v] > T(0.5)) != (yb[v] > T(0.5));
            s_e[v] = (uint8_t)e;
            nerr += e;
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        int bad_chk = 0;
        for (int r = lane; r < C; r += 64) {     // lanes over checks (graph CSR)
            int par = 0;
            for (int k = g.chk_ptr[r]; k < g.chk_ptr[r + 1]; ++k)
                par ^= s_e[g.edge_vc[g.chk_edge[k]] & 0xffffu];
            bad_chk |= par;
        }
        int bad_log = 0;
        for (int l = 0; l < nl; ++l) {           // logical rows: wave parity
            const int32_t* row = lg + (size_t)l * V;
            int par = 0;
            for (int v = lane; v < V; v += 64) par ^= row[v] ? s_e[v] : 0;
            bad_log |= __builtin_popcountll(__ballot(par)) & 1;
        }
        const unsigned long long any_chk = __ballot(bad_chk);
        for (int o = 32; o >= 1; o >>= 1) nerr += __shfl_xor(nerr, o);
        c_bit += (unsigned)nerr;
        c_frame += nerr != 0;
        c_syn += any_chk != 0;
        c_log += any_chk == 0 && bad_log;
        __builtin_amdgcn_wave_barrier();         // s_e reads done before the next writes
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (lane == 0) {
        if (c_bit) atomicAdd(&counts[0], c_bit);
        if (c_frame) atomicAdd(&counts[1], c_frame);
        if (c_syn) atomicAdd(&counts[2], c_syn);
        if (c_log) atomicAdd(&counts[3], c_log);
    }
}

template <typename T>
int launch_decision_errors(const gnnd_graph* g, const int32_t* lg, int nl, const void* pred,
                           const void* y, int64_t* counts, int64_t B, hipStream_t st) {
    const GraphView& v = g->view;
    const size_t lds = 4 * (size_t)((v.V + 15) & ~15);
    GNND_HIP_CHECK(hipMemsetAsync(counts, 0, 4 * sizeof(int64_t), st));
    if (B == 0) return GNND_OK;
    const int64_t want = (B + 3) / 4;
    const int64_t blocks = want < 2048 ? want : 2048;     // 8 waves per CU, grid-stride
    decision_errors_kernel<T><<<(unsigned)blocks, 256, lds, st>>>(
        v, lg, nl, (const T*)pred, (const T*)y, (unsigned long long*)counts, B);
    GNND_LAUNCH_CHECK();
    return GNND_OK;
}

// ---------------------------------------------------------------------------------------
// Adam on one flat parameter buffer (torch.optim.Adam, amsgrad/maximize off, the
// non-capturable update order), device-resident step counter: graph-capturable
// ---------------------------------------------------------------------------------------
// g' = g + wd p;  m = m + (1 - b1)(g' - m)  (lerp, weight < 0.5);  v = v b2; v += ((1 - b2) g') g';
// t = step + 1;  p += -(lr / (1 - b1^t)) * (m / (sqrt(v) / sqrt(1 - b2^t) + eps)).
// Bias corrections in double (torch computes them as Python floats).  ONE workgroup: the
// counter is read by every thread and written back after a barrier.
// one parameter's update (shared by adam_kernel and train_update_kernel: same code, same bits)
template <typename T> struct AdamCoef {
    T step_size, bc2s, w1, tb2, w2, te, twd;
    bool decay;
    // bias corrections of step t (double pow, as torch computes them on the host)
    __device__ static T step_size_of(double t, double lr, double b1) { return (T)(lr / (1.0 - pow(b1, t))); }
    __device__ static T bc2s_of(double t, double b2) { return (T)sqrt(1.0 - pow(b2, t)); }
    __device__ AdamCoef(T ss, T bc, double b1, double b2, double eps, double wd)
        : step_size(ss), bc2s(bc), w1((T)(1.0 - b1)), tb2((T)b2), w2((T)(1.0 - b2)), te((T)eps),
          twd((T)wd), decay(wd != 0.0) {}
};
template <typename T>
__device__ __forceinline__ T adam_one(const AdamCoef<T>& c, T pi, T gi, T& mi_io, T& vi_io) {
    if (c.decay) gi = __builtin_fma(c.twd, pi, gi);
    const T mi = __builtin_fma(c.w1, gi - mi_io, mi_io);
    const T vi = __builtin_fma(c.w2 * gi, gi, vi_io * c.tb2);
    mi_io = mi;
    vi_io = vi;
    const T denom = sqrt(vi) / c.bc2s + c.te;
    return __builtin_fma(-c.step_size, mi / denom, pi);
}

template <typename T>
__global__ void __launch_bounds__(1024)
adam_kernel(T* __restrict__ p, const T* __restrict__ g, T* __restrict__ m, T* __restrict__ v,
            double* __restrict__ step, int64_t n, double lr, double b1, double b2, double eps,
            double wd) {
    const double t = step[0] + 1.0;
    const AdamCoef<T> c(AdamCoef<T>::step_size_of(t, lr, b1), AdamCoef<T>::bc2s_of(t, b2), b1, b2,
                        eps, wd);
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
        T mi = m[i], vi = v[i];
        p[i] = adam_one(c, p[i], g[i], mi, vi);
        m[i] = mi;
        v[i] = vi;
    }
    __syncthreads();
    if (threadIdx.x == 0) step[0] = t;
}

// ---------------------------------------------------------------------------------------
// fused optimizer epilogue of a training step (gnnd_train_update): per parameter i
//   REDUCE  g_i = fixed-order sum of the reverse pass's per-workgroup rows (a block = 64
//           parameters x 16 waves: wave w sums rows w, w+16, ... in order with coalesced row
//           reads, then a fixed LDS tree), written to grad (if given); otherwise g_i = grad[i]
//           (an all-reduced gradient)
//   LOSS    block 0 also sums the per-codeword losses in a fixed order -> loss[0]
//   ADAM    torch.optim.Adam's update (adam_kernel's order) of param/exp_avg/exp_avg_sq, then
//           the kernel-layout copy of the updated weight (gnnd_prepare_weights' mapping) into
//           prepared, so the next step's forward needs no prepare launch
// The step count is read by one lane per block before that block arrives on `sync` (an
// agent-scope atomic counter); the last block to arrive writes step + 1 and re-arms the
// counter.  Nothing else crosses workgroups: one launch replaces grad_reduce, the loss sum,
// Adam and prepare (four ~5 us launches of the single-rank step).
// ---------------------------------------------------------------------------------------
constexpr int kUpdThreads = 1024;           // 16 row groups x 64 parameters per block

// plain packed index i of decoder_v2_4 -> (prepared index, scale) of the fp32 kernel layout
// (prepare_v24_f32_kernel in gnnd_decode.hip)
__device__ __forceinline__ int v24_prep_index(int i, float& scale) {
    if (i < kV24Ggc2) {                       // ggc1.mlp: W1a, W1b, b1, W2, b2
        const int k = i & 127;
        if (i < 128) { scale = kLog2e; return 256 + k; }
        if (i < 256) { scale = kLog2e; return 2 * k; }
        if (i < 384) { scale = kLog2e; return 2 * k + 1; }
        scale = i < 512 ? kLn2 : 1.f;
        return i;
    }
    const int base = i < kV24Mlp ? kV24Ggc2 : kV24Mlp;   // ggc2.mlp / mlp: W1, b1, W2, b2
    const int l = i - base, k = l & 127;
    if (l < 128) { scale = kLog2e; return base + 2 * k; }
    if (l < 256) { scale = kLog2e; return base + 2 * k + 1; }
    scale = l < 384 ? kLn2 : 1.f;
    return i;
}

template <typename T>
__global__ void __launch_bounds__(kUpdThreads)
train_update_kernel(const T* __restrict__ rows, int nrows, T* __restrict__ grad,
                    const T* __restrict__ loss_b, int64_t nloss, T* __restrict__ loss,
                    T* __restrict__ p, T* __restrict__ m, T* __restrict__ v,
                    double* __restrict__ step, uint32_t* __restrict__ sync, int n, double lr,
                    double b1, double b2, double eps, double wd, T* __restrict__ prepared,
                    int prep_v24_f32) {
    __shared__ T s_red[kUpdThreads];
    __shared__ double s_t;
    __shared__ T s_coef[2];
    constexpr int kGroups = kUpdThreads / 64;          // row groups (waves)
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int i = blockIdx.x * 64 + lane;               // this lane's parameter
    const bool adam = p != nullptr;
    if (adam && tid == 0) {                   // bias corrections once per block (double pow)
        s_t = step[0] + 1.0;
        s_coef[0] = AdamCoef<T>::step_size_of(s_t, lr, b1);
        s_coef[1] = AdamCoef<T>::bc2s_of(s_t, b2);
    }
    T gi = T(0);
    if (rows) {
        // wave w sums rows w, w + 16, ... of 64 consecutive parameters (coalesced rows),
        // then a fixed tree over the 16 waves' partials
        // (16 rows' loads issued before their adds: the same order, without one dependent
        // L2 round trip per row)
        T s = T(0);
        if (i < n) {
            int r = wv;
            for (; r + 15 * kGroups < nrows; r += 16 * kGroups) {
                T v[16];
#pragma unroll
                for (int j = 0; j < 16; ++j) v[j] = rows[(size_t)(r + j * kGroups) * n + i];
#pragma unroll
                for (int j = 0; j < 16; ++j) s += v[j];
            }
            for (; r < nrows; r += kGroups) s += rows[(size_t)r * n + i];
        }
        s_red[tid] = s;
        __syncthreads();
        for (int o = kGroups / 2; o >= 1; o >>= 1) {
            if (wv < o) s_red[tid] += s_red[tid + 64 * o];
            __syncthreads();
        }
        gi = s_red[lane];
        if (grad && wv == 0 && i < n) grad[i] = gi;
    } else if (i < n && wv == 0) {
        gi = grad[i];
    }
    if (loss_b && blockIdx.x == 0) {          // per-codeword losses, fixed order
        __syncthreads();
        T s = T(0);
        for (int64_t b = tid; b < nloss; b += kUpdThreads) s += loss_b[b];
        s_red[tid] = s;
        __syncthreads();
        for (int o = kUpdThreads / 2; o >= 1; o >>= 1) {
            if (tid < o) s_red[tid] += s_red[tid + o];
            __syncthreads();
        }
        if (tid == 0) loss[0] = s_red[0];
    }
    if (!adam) return;
    __syncthreads();                          // s_t (and every use of step) before arrival
    const double t = s_t;
    if (wv == 0 && i < n) {
        const AdamCoef<T> c(s_coef[0], s_coef[1], b1, b2, eps, wd);
        T mi = m[i], vi = v[i];
        const T np = adam_one(c, p[i], gi, mi, vi);
        m[i] = mi;
        v[i] = vi;
        p[i] = np;
        if (prepared) {
            if (prep_v24_f32) {
                float sc;
                const int k = v24_prep_index(i, sc);
                prepared[k] = (T)((float)np * sc);
            } else {
                prepared[i] = np;
            }
        }
    }
    if (tid == 0) {
        const uint32_t prev = __hip_atomic_fetch_add(sync, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == gridDim.x - 1) {          // every block has read the step count
            step[0] = t;
            __hip_atomic_store(sync, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

}  // namespace

extern "C" int gnnd_train_tape_bytes(const gnnd_graph* g, int model, int dtype, int64_t batch,
                                     int32_t iters, int64_t* h_bytes) {
    if (!train_args_ok(g, model, dtype, batch, iters) || !h_bytes) return GNND_ERR_INVALID_ARG;
    const int64_t esz = dtype == GNND_F64 ? 8 : 4;
    *h_bytes = model == GNND_V30 ? esz * gnnd_v30_tape_elems(g, batch, iters)
               : is_wbp_train(model) ? esz * gnnd_wbp_tape_elems(g, batch, iters)
               : is_gnn_train(model) ? esz * gnnd_gnn_tape_elems(g, batch, iters)
                                     : esz * batch * g->view.E * (3 * (int64_t)iters + 1);
    return GNND_OK;
}

extern "C" int gnnd_train_fwd(const gnnd_graph* g, int model, int dtype, const void* d_w,
                              const void* d_x, void* d_out, void* d_tape, int64_t batch,
                              int32_t iters, void* stream) {
    if (!train_args_ok(g, model, dtype, batch, iters)) return GNND_ERR_INVALID_ARG;
    if (batch == 0) return GNND_OK;
    if (!d_w || !d_x || !d_out || !d_tape) return GNND_ERR_INVALID_ARG;
    if (model == GNND_V30)
        return gnnd_launch_v30_tape(g, dtype, d_w, d_x, d_out, batch, iters, d_tape, (hipStream_t)stream);
    if (is_wbp_train(model))
        return gnnd_launch_wbp_tape(g, model, d_w, d_x, d_out, batch, iters, d_tape, (hipStream_t)stream);
    if (is_gnn_train(model))
        return gnnd_launch_gnn_tape(g, model, dtype, d_w, d_x, d_out, batch, iters, d_tape,
                                    (hipStream_t)stream);
    return gnnd_launch_v24_tape(g, dtype, d_w, d_x, d_out, batch, iters, d_tape,
                                (hipStream_t)stream);
}

extern "C" int gnnd_train_fwd_loss(const gnnd_graph* g, int model, int dtype, const void* d_w,
                                   const void* d_x, void* d_out, void* d_tape, const void* d_y,
                                   const uint32_t* d_logical_mask, int32_t n_logical,
                                   int32_t logical_only, void* d_grad_out, void* d_loss_b,
                                   int64_t batch, int32_t iters, void* stream) {
    if (!train_args_ok(g, model, dtype, batch, iters)) return GNND_ERR_INVALID_ARG;
    if (model != GNND_V24 || dtype != GNND_F32) return GNND_ERR_UNSUPPORTED;
    if (n_logical < 0 || n_logical > 32 || (n_logical > 0 && !d_logical_mask)) return GNND_ERR_INVALID_ARG;
    if (batch == 0) return GNND_OK;
    if (!d_w || !d_x || !d_out || !d_tape || !d_y || !d_grad_out || !d_loss_b) return GNND_ERR_INVALID_ARG;
    // the losses' layout is the reverse pass's (gnnd_train_loss_count): the forward must split
    // a codeword into the same components
    const int need = train_split(g, batch) ? g->ncomp : 1;
    return gnnd_launch_v24_tape_loss(g, dtype, d_w, d_x, d_out, batch, iters, d_tape, d_y,
                                     d_logical_mask, n_logical, logical_only, need, d_grad_out,
                                     d_loss_b, (hipStream_t)stream);
}

extern "C" int gnnd_train_workspace_bytes(const gnnd_graph* g, int model, int dtype,
                                          int64_t batch, int32_t iters, int64_t* h_bytes) {
    if (!train_args_ok(g, model, dtype, batch, iters) || !h_bytes) return GNND_ERR_INVALID_ARG;
    const int64_t n = is_wbp_train(model) ? wbp_weights(g, model, iters) : train_weights(model);
    *h_bytes = model_train_rows(g, model, batch) * n * (dtype == GNND_F64 ? 8 : 4);
    return GNND_OK;
}

extern "C" int gnnd_train_bwd_workspace(const gnnd_graph* g, int model, int dtype,
                                        int64_t batch, int64_t* h_bytes) {
    if (!train_args_ok(g, model, dtype, batch, 0) || !h_bytes) return GNND_ERR_INVALID_ARG;
    if (is_wbp_train(model)) return GNND_ERR_UNSUPPORTED;    // depends on iters: the call above
    *h_bytes = model_train_rows(g, model, batch) * (int64_t)train_weights(model) * (dtype == GNND_F64 ? 8 : 4);
    return GNND_OK;
}

extern "C" int gnnd_train_bwd(const gnnd_graph* g, int model, int dtype, const void* d_w,
                              const void* d_x, const void* d_out, const void* d_grad_out,
                              const void* d_tape, void* d_grad_w, void* d_workspace,
                              int64_t workspace_bytes, int64_t batch, int32_t iters,
                              void* stream) {
    if (!train_args_ok(g, model, dtype, batch, iters)) return GNND_ERR_INVALID_ARG;
    if (!d_w || !d_grad_w) return GNND_ERR_INVALID_ARG;
    hipStream_t st = (hipStream_t)stream;
    const int64_t nw = is_wbp_train(model) ? wbp_weights(g, model, iters) : train_weights(model);
    if (batch == 0) {
        GNND_HIP_CHECK(hipMemsetAsync(d_grad_w, 0, (size_t)nw * (dtype == GNND_F64 ? 8 : 4), st));
        return GNND_OK;
    }
    if (!d_x || !d_out || !d_grad_out || !d_tape || !d_workspace) return GNND_ERR_INVALID_ARG;
    if (is_wbp_train(model)) {
        const int rc = gnnd_launch_wbp_bwd(g, model, d_w, d_x, d_out, d_grad_out, d_tape, d_workspace,
                                           workspace_bytes, batch, iters, st);
        if (rc != GNND_OK) return rc;
        if (nw > 0x7fffffff) return GNND_ERR_UNSUPPORTED;
        grad_reduce_kernel<double><<<(unsigned)((nw + 255) / 256), 256, 0, st>>>(
            (const double*)d_workspace, (int)gnnd_wbp_train_rows(batch), (double*)d_grad_w, (int)nw);
        GNND_LAUNCH_CHECK();
        return GNND_OK;
    }
    if (is_gnn_train(model)) {
        const int rc = gnnd_launch_gnn_bwd(g, model, dtype, d_w, d_x, d_grad_out, d_tape, d_workspace,
                                           workspace_bytes, batch, iters, st);
        if (rc != GNND_OK) return rc;
        const int rows = (int)gnnd_gnn_train_rows(batch);
        if (dtype == GNND_F32)
            grad_reduce_kernel<float><<<1, 256, 0, st>>>((const float*)d_workspace, rows, (float*)d_grad_w, 62);
        else
            grad_reduce_kernel<double><<<1, 256, 0, st>>>((const double*)d_workspace, rows, (double*)d_grad_w, 62);
        GNND_LAUNCH_CHECK();
        return GNND_OK;
    }
    if (model == GNND_V30) {
        const int rc = gnnd_launch_v30_bwd(g, dtype, d_w, d_x, d_out, d_grad_out, d_tape, d_workspace,
                                           workspace_bytes, batch, iters, st);
        if (rc != GNND_OK) return rc;
        const int rows = (int)gnnd_v30_train_rows(batch);
        if (dtype == GNND_F32)
            grad_reduce_kernel<float><<<1, 256, 0, st>>>((const float*)d_workspace, rows, (float*)d_grad_w, kV30Count);
        else
            grad_reduce_kernel<double><<<1, 256, 0, st>>>((const double*)d_workspace, rows, (double*)d_grad_w, kV30Count);
        GNND_LAUNCH_CHECK();
        return GNND_OK;
    }
    if (dtype == GNND_F32)
        return launch_bwd<float>(g, d_w, d_x, d_out, d_grad_out, d_tape, d_grad_w, d_workspace,
                                 workspace_bytes, batch, iters, st);
    return launch_bwd<double>(g, d_w, d_x, d_out, d_grad_out, d_tape, d_grad_w, d_workspace,
                              workspace_bytes, batch, iters, st);
}

extern "C" int gnnd_train_bwd_rows(const gnnd_graph* g, int model, int dtype, int64_t batch,
                                   int64_t* h_rows) {
    if (!train_args_ok(g, model, dtype, batch, 0) || !h_rows) return GNND_ERR_INVALID_ARG;
    *h_rows = batch > 0 ? model_train_rows(g, model, batch) : 0;
    return GNND_OK;
}

extern "C" int gnnd_train_bwd_partial(const gnnd_graph* g, int model, int dtype, const void* d_w,
                                      const void* d_x, const void* d_out, const void* d_grad_out,
                                      const void* d_tape, void* d_workspace, int64_t workspace_bytes,
                                      int64_t batch, int32_t iters, void* stream) {
    if (!train_args_ok(g, model, dtype, batch, iters)) return GNND_ERR_INVALID_ARG;
    if (batch == 0) return GNND_OK;
    if (!d_w || !d_x || !d_out || !d_grad_out || !d_tape || !d_workspace) return GNND_ERR_INVALID_ARG;
    hipStream_t st = (hipStream_t)stream;
    if (model == GNND_V30)
        return gnnd_launch_v30_bwd(g, dtype, d_w, d_x, d_out, d_grad_out, d_tape, d_workspace,
                                   workspace_bytes, batch, iters, st);
    if (is_wbp_train(model))
        return gnnd_launch_wbp_bwd(g, model, d_w, d_x, d_out, d_grad_out, d_tape, d_workspace,
                                   workspace_bytes, batch, iters, st);
    if (is_gnn_train(model))
        return gnnd_launch_gnn_bwd(g, model, dtype, d_w, d_x, d_grad_out, d_tape, d_workspace,
                                   workspace_bytes, batch, iters, st);
    if (dtype == GNND_F32)
        return launch_bwd<float>(g, d_w, d_x, d_out, d_grad_out, d_tape, nullptr, d_workspace,
                                 workspace_bytes, batch, iters, st);
    return launch_bwd<double>(g, d_w, d_x, d_out, d_grad_out, d_tape, nullptr, d_workspace,
                              workspace_bytes, batch, iters, st);
}

extern "C" int gnnd_train_loss_count(const gnnd_graph* g, int64_t batch, int64_t* h_count) {
    if (!g || batch < 0 || !h_count) return GNND_ERR_INVALID_ARG;
    *h_count = batch * (train_split(g, batch) ? g->ncomp : 1);
    return GNND_OK;
}

extern "C" int gnnd_train_bwd_loss_partial(const gnnd_graph* g, int model, int dtype,
                                           const void* d_w, const void* d_x, const void* d_out,
                                           const void* d_y, const uint32_t* d_logical_mask,
                                           int32_t n_logical, int32_t logical_only,
                                           const void* d_tape, void* d_loss_b, void* d_workspace,
                                           int64_t workspace_bytes, int64_t batch, int32_t iters,
                                           void* stream) {
    if (!train_args_ok(g, model, dtype, batch, iters)) return GNND_ERR_INVALID_ARG;
    if (model != GNND_V24) return GNND_ERR_UNSUPPORTED;    // decoder_v2_4's syndrome loss only
    if (n_logical < 0 || n_logical > 32 || (n_logical > 0 && !d_logical_mask)) return GNND_ERR_INVALID_ARG;
    if (batch == 0) return GNND_OK;
    if (!d_w || !d_x || !d_out || !d_y || !d_tape || !d_loss_b || !d_workspace) return GNND_ERR_INVALID_ARG;
    hipStream_t st = (hipStream_t)stream;
    if (dtype == GNND_F32)
        return launch_bwd<float>(g, d_w, d_x, d_out, d_out, d_tape, nullptr, d_workspace,
                                 workspace_bytes, batch, iters, st,
                                 BwdLoss<float>{(const float*)d_y, d_logical_mask, n_logical,
                                                logical_only, 1, (float*)d_loss_b});
    return launch_bwd<double>(g, d_w, d_x, d_out, d_out, d_tape, nullptr, d_workspace,
                              workspace_bytes, batch, iters, st,
                              BwdLoss<double>{(const double*)d_y, d_logical_mask, n_logical,
                                              logical_only, 1, (double*)d_loss_b});
}

extern "C" int gnnd_train_update(int model, int dtype, const void* d_rows, int64_t n_rows,
                                 void* d_grad, const void* d_loss_b, int64_t batch, void* d_loss,
                                 void* d_param, void* d_exp_avg, void* d_exp_avg_sq,
                                 double* d_step, uint32_t* d_sync, double lr, double beta1,
                                 double beta2, double eps, double weight_decay, void* d_prepared,
                                 void* stream) {
    if ((model != GNND_V24 && model != GNND_V30 && !is_gnn_train(model)) ||
        (dtype != GNND_F32 && dtype != GNND_F64))
        return GNND_ERR_INVALID_ARG;
    if (n_rows < 0 || batch < 0 || n_rows > 0x7fffffff) return GNND_ERR_INVALID_ARG;
    if (n_rows > 0 && !d_rows) return GNND_ERR_INVALID_ARG;
    if (n_rows == 0 && !d_grad) return GNND_ERR_INVALID_ARG;          // nothing to update from
    if (batch > 0 && (!d_loss_b) != (!d_loss)) return GNND_ERR_INVALID_ARG;
    const bool adam = d_param != nullptr;
    if (adam && (!d_exp_avg || !d_exp_avg_sq || !d_step || !d_sync)) return GNND_ERR_INVALID_ARG;
    if (!adam && d_prepared) return GNND_ERR_INVALID_ARG;
    hipStream_t st = (hipStream_t)stream;
    const int nw = train_weights(model);
    const int blocks = (nw + 63) / 64;
    // V30's, CGNNI's and QGNNI's kernel layouts are the plain one
    const int prep_f32 = model == GNND_V24 ? 1 : 0;
    const bool lossb = batch > 0 && d_loss_b;
    if (dtype == GNND_F32)
        train_update_kernel<float><<<blocks, kUpdThreads, 0, st>>>(
            n_rows ? (const float*)d_rows : nullptr, (int)n_rows, (float*)d_grad,
            lossb ? (const float*)d_loss_b : nullptr, batch, (float*)d_loss, (float*)d_param,
            (float*)d_exp_avg, (float*)d_exp_avg_sq, d_step, d_sync, nw, lr, beta1, beta2, eps,
            weight_decay, (float*)d_prepared, prep_f32);
    else
        train_update_kernel<double><<<blocks, kUpdThreads, 0, st>>>(
            n_rows ? (const double*)d_rows : nullptr, (int)n_rows, (double*)d_grad,
            lossb ? (const double*)d_loss_b : nullptr, batch, (double*)d_loss, (double*)d_param,
            (double*)d_exp_avg, (double*)d_exp_avg_sq, d_step, d_sync, nw, lr, beta1, beta2,
            eps, weight_decay, (double*)d_prepared, 0);
    GNND_LAUNCH_CHECK();
    // fp64 decoder_v2_4: the check-MLP table of the updated weights (the prepared layout's tail)
    if (model == GNND_V24 && dtype == GNND_F64 && d_prepared)
        return launch_ctab_build((const double*)d_prepared, (double*)d_prepared, st);
    if (model == GNND_V24 && dtype == GNND_F32 && d_prepared && GNND_V24_CTAB)   // (from the plain weights)
        return launch_ctab_build((const float*)d_param, (float*)d_prepared, st);
    // fp32 CGNNI / QGNNI: the message MLP's piecewise-linear table
    if ((model == GNND_CGNNI || model == GNND_QGNNI) && dtype == GNND_F32 && d_prepared && GNND_MLP_PWL)
        return launch_pwl_build((const float*)d_prepared, (float*)d_prepared, st);
    return GNND_OK;
}

extern "C" int gnnd_syndrome_loss(const gnnd_graph* g, const int32_t* d_logical, int32_t n_logical,
                                  int32_t logical_only, int dtype, const void* d_pred,
                                  const void* d_y, void* d_loss_b, void* d_dpred, int64_t batch,
                                  void* stream) {
    if (!g || n_logical < 0 || (n_logical > 0 && !d_logical) || batch < 0) return GNND_ERR_INVALID_ARG;
    if (dtype != GNND_F32 && dtype != GNND_F64) return GNND_ERR_INVALID_ARG;
    if (batch == 0) return GNND_OK;
    if (!d_pred || !d_y || !d_loss_b || !d_dpred) return GNND_ERR_INVALID_ARG;
    hipStream_t st = (hipStream_t)stream;
    if (dtype == GNND_F32)
        return launch_syndrome_loss<float>(g, d_logical, n_logical, logical_only, d_pred, d_y,
                                           d_loss_b, d_dpred, batch, st);
    return launch_syndrome_loss<double>(g, d_logical, n_logical, logical_only, d_pred, d_y,
                                        d_loss_b, d_dpred, batch, st);
}

extern "C" int gnnd_decision_errors(const gnnd_graph* g, const int32_t* d_logical,
                                    int32_t n_logical, int dtype, const void* d_pred,
                                    const void* d_y, int64_t* d_counts, int64_t batch,
                                    void* stream) {
    if (!g || n_logical < 0 || (n_logical > 0 && !d_logical) || batch < 0 || !d_counts)
        return GNND_ERR_INVALID_ARG;
    if (dtype != GNND_F32 && dtype != GNND_F64) return GNND_ERR_INVALID_ARG;
    if (batch > 0 && (!d_pred || !d_y)) return GNND_ERR_INVALID_ARG;
    hipStream_t st = (hipStream_t)stream;
    if (dtype == GNND_F32)
        return launch_decision_errors<float>(g, d_logical, n_logical, d_pred, d_y, d_counts, batch, st);
    return launch_decision_errors<double>(g, d_logical, n_logical, d_pred, d_y, d_counts, batch, st);
}

extern "C" int gnnd_adam_step(int dtype, void* d_param, const void* d_grad, void* d_exp_avg,
                              void* d_exp_avg_sq, double* d_step, int64_t n, double lr,
                              double beta1, double beta2, double eps, double weight_decay,
                              void* stream) {
    if (dtype != GNND_F32 && dtype != GNND_F64) return GNND_ERR_INVALID_ARG;
    if (n < 0 || !d_step) return GNND_ERR_INVALID_ARG;
    if (n > 0 && (!d_param || !d_grad || !d_exp_avg || !d_exp_avg_sq)) return GNND_ERR_INVALID_ARG;
    hipStream_t st = (hipStream_t)stream;
    if (dtype == GNND_F32)
        adam_kernel<float><<<1, 1024, 0, st>>>((float*)d_param, (const float*)d_grad,
                                               (float*)d_exp_avg, (float*)d_exp_avg_sq, d_step, n,
                                               lr, beta1, beta2, eps, weight_decay);
    else
        adam_kernel<double><<<1, 1024, 0, st>>>((double*)d_param, (const double*)d_grad,
                                                (double*)d_exp_avg, (double*)d_exp_avg_sq, d_step,
                                                n, lr, beta1, beta2, eps, weight_decay);
    GNND_LAUNCH_CHECK();
    return GNND_OK;
}
