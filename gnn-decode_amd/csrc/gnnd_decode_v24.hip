// gnnd_decode_v24.hip — kernel instantiations for model GNND_V24 (see gnnd_decode_impl.h).
#include "gnnd_decode_impl.h"

GNND_DEBUG_TU(decode_v24)

int gnnd_launch_v24(const gnnd_graph* g, int dtype, const void* w, const void* x, void* out,
                       int64_t B, int iters, hipStream_t st) {
    return launch_model<GNND_V24>(g, dtype, w, x, out, B, iters, st);
}

int gnnd_launch_v24_tape(const gnnd_graph* g, int dtype, const void* w, const void* x, void* out,
                         int64_t B, int iters, void* tape, hipStream_t st) {
    if (dtype == GNND_F32) return launch_decode_r<GNND_V24, float>(g, w, x, out, B, iters, st, tape);
    return launch_decode_r<GNND_V24, double>(g, w, x, out, B, iters, st, tape);
}

int gnnd_launch_v24_tape_loss(const gnnd_graph* g, int dtype, const void* w, const void* x, void* out,
                              int64_t B, int iters, void* tape, const void* y, const uint32_t* lmask,
                              int nl, int logical_only, int need_ncomp, void* gp, void* loss_b,
                              hipStream_t st) {
    if (dtype != GNND_F32) return GNND_ERR_UNSUPPORTED;
    const FwdLoss fl{y, lmask, nl, logical_only, need_ncomp, gp, loss_b};
    return launch_decode_r<GNND_V24, float>(g, w, x, out, B, iters, st, tape, &fl);
}

// ---------------------------------------------------------------------------------------
// decoder_v2_4's check-side MLP through the table the fp64 decoder reads (ctab_build_kernel /
// ctab_valid / ctab_eval, gnnd_decode_impl.h): the same staged entries and evaluation, exposed
// so tests can hold it against the reference MLP (quantum/decoder_v2_4.py:241-243, :253-257)
// ---------------------------------------------------------------------------------------
namespace {
__global__ void __launch_bounds__(256)
ctab_eval_kernel(const double* __restrict__ w, int max_dc, const double* __restrict__ u,
                 double* __restrict__ y, int64_t n, int32_t* __restrict__ ok) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    double* tab = (double*)smem;
    const int R = max_dc > 1 ? max_dc - 1 : 0, R8 = kCtabInv * R;
    const bool valid = ctab_valid(w, R);
    if (blockIdx.x == 0 && threadIdx.x == 0) *ok = valid ? 1 : 0;
    if (!valid) return;                                       // (uniform)
    const double2* src = (const double2*)(w + kV24CtabOff + (size_t)(kCtabInv * kCtabRcap - R8) * kCtabNC);
    for (int i = threadIdx.x; i < ctab_entries(max_dc) * kCtabNC / 2; i += blockDim.x) ((double2*)tab)[i] = src[i];
    __syncthreads();
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        y[i] = ctab_eval(tab, u[i], R8);
}
}  // namespace

extern "C" int gnnd_v24_check_mlp_table(const gnnd_graph* g, const void* d_w, const void* d_u,
                                        void* d_y, int64_t n, int32_t* d_ok, void* stream) {
    if (!g || !d_w || !d_ok || n < 0 || (n > 0 && (!d_u || !d_y))) return GNND_ERR_INVALID_ARG;
    const int max_dc = g->view.max_dc;
    const size_t lds = (size_t)ctab_entries(max_dc < kCtabRcap + 1 ? max_dc : kCtabRcap + 1) * kCtabNC * 8;
    auto kern = ctab_eval_kernel;
    if (lds > 64 * 1024)
        GNND_HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    const int64_t blocks = n > 0 ? std::min<int64_t>((n + 255) / 256, 64) : 1;
    kern<<<(unsigned)blocks, 256, lds, (hipStream_t)stream>>>((const double*)d_w, max_dc, (const double*)d_u,
                                                               (double*)d_y, n, d_ok);
    GNND_LAUNCH_CHECK();
    return GNND_OK;
}

// the variable-side MLP through the channel-prior tables (vtab_eval, gnnd_decode_impl.h), for
// tests: y[i] = tanh(ggc1.mlp(u[i], x[i]) / 2) (the check step's pre-op, what the tables hold)
// and hit[i] = 1 where a table covers (u[i], x[i]), else hit[i] = 0 and y[i] untouched (the
// decoder evaluates the 128 units there); x = NULL: the readout MLP's table, y[i] = mlp(u[i])
namespace {
__global__ void __launch_bounds__(256)
vtab_eval_kernel(const double* __restrict__ w, const double* __restrict__ u, const double* __restrict__ xv,
                 double* __restrict__ y, int32_t* __restrict__ hit, int64_t n) {
    const int n_pt = (int)w[kV24PriorHdr];
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        int h = 0;
        if (!xv) {                                        // the readout MLP's table
            double v;
            if (n_pt > 0 && w[kV24PriorHdr + 1] != 0.0 &&
                vtab_eval<kVtInvR, false>(w + kV24PriorOff + (size_t)n_pt * kVtStride, u[i], 0.0, v)) {
                y[i] = v;
                h = 1;
            }
            hit[i] = h;
            continue;
        }
        const long long xb = __double_as_longlong(xv[i]);
        for (int t = 0; t < n_pt; ++t) {
            const double* tb = w + kV24PriorOff + (size_t)t * kVtStride;
            if (__double_as_longlong(tb[0]) != xb) continue;
            double v;
            if (vtab_eval<kVtInvG, true>(tb, u[i], xv[i], v)) {
                y[i] = v;
                h = 1;
            }
            break;
        }
        hit[i] = h;
    }
}
}  // namespace

extern "C" int gnnd_v24_var_mlp_table(const void* d_w, const void* d_u, const void* d_x, void* d_y,
                                      int32_t* d_hit, int64_t n, void* stream) {
    if (!d_w || n < 0 || (n > 0 && (!d_u || !d_y || !d_hit))) return GNND_ERR_INVALID_ARG;
    if (n == 0) return GNND_OK;
    const int64_t blocks = std::min<int64_t>((n + 255) / 256, 1024);
    vtab_eval_kernel<<<(unsigned)blocks, 256, 0, (hipStream_t)stream>>>(
        (const double*)d_w, (const double*)d_u, (const double*)d_x, (double*)d_y, d_hit, n);
    GNND_LAUNCH_CHECK();
    return GNND_OK;
}
