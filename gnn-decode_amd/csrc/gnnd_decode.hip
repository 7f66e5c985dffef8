// gnnd_decode.hip — C ABI of the fused decoder (kernels: gnnd_decode_impl.h, instantiated
// per model in gnnd_decode_<model>.hip) and the weight preparation kernel.
#include "gnnd_decode_impl.h"

GNND_DEBUG_TU(decode)

namespace {

// ---------------------------------------------------------------------------------------
// weights: fp32 V24 gets the paired-edge base-2 layout read by mlp128*_sp2 (gnnd_decode_impl.h)
// ---------------------------------------------------------------------------------------
__global__ void prepare_v24_f32_kernel(const float* __restrict__ in, float* __restrict__ o) {
    const int k = threadIdx.x;          // hidden unit, one block of 128 threads
    // ggc1.mlp (plain: W1a[128], W1b[128], b1[128], W2[128], b2) ->
    //   {W1b'_k, b1'_k}[128] | W1a'[128] | w2'[128] | b2
    const float* a = in + kV24Ggc1;
    float* q = o + kV24Ggc1;
    q[2 * k] = a[128 + k] * kLog2e;
    q[2 * k + 1] = a[256 + k] * kLog2e;
    q[256 + k] = a[k] * kLog2e;
    q[384 + k] = a[384 + k] * kLn2;
    if (k == 0) q[512] = a[512];
    // ggc2.mlp and mlp (plain: W1[128], b1[128], W2[128], b2) -> {W1'_k, b1'_k}[128] | w2' | b2
    for (int seg = 0; seg < 2; ++seg) {
        const float* s = in + (seg ? kV24Mlp : kV24Ggc2);
        float* d = o + (seg ? kV24Mlp : kV24Ggc2);
        d[2 * k] = s[k] * kLog2e;
        d[2 * k + 1] = s[128 + k] * kLog2e;
        d[256 + k] = s[256 + k] * kLn2;
        if (k == 0) d[384] = s[384];
    }
}


int dispatch_decode(const gnnd_graph* g, int model, int dtype, const void* w, const void* x,
                    void* out, int64_t B, int iters, hipStream_t st) {
    switch (model) {
        case GNND_V24: return gnnd_launch_v24(g, dtype, w, x, out, B, iters, st);
        case GNND_QGNNI: return gnnd_launch_qgnni(g, dtype, w, x, out, B, iters, st);
        case GNND_QBP: return gnnd_launch_qbp(g, dtype, w, x, out, B, iters, st);
        case GNND_CGNNI: return gnnd_launch_cgnni(g, dtype, w, x, out, B, iters, st);
        case GNND_CBP: return gnnd_launch_cbp(g, dtype, w, x, out, B, iters, st);
        case GNND_NBP: return gnnd_launch_nbp(g, dtype, w, x, out, B, iters, st);
        case GNND_V10: return gnnd_launch_v10(g, dtype, w, x, out, B, iters, st);
        case GNND_V30: return gnnd_launch_v30(g, dtype, w, x, out, B, iters, st);
        case GNND_V22: return gnnd_launch_v22(g, dtype, w, x, out, B, iters, st);
        default: return GNND_ERR_INVALID_ARG;
    }
}

}  // namespace

extern "C" int gnnd_weights_count(int model, int64_t* h_count) {
    int n = weights_count(model);
    if (n == -1 || !h_count) return GNND_ERR_INVALID_ARG;
    if (n < 0) return GNND_ERR_UNSUPPORTED;     // graph-dependent: gnnd_decode_weights_count
    *h_count = n;
    return GNND_OK;
}

extern "C" int gnnd_decode_weights_count(const gnnd_graph* g, int model, int32_t iters,
                                         int64_t* h_count) {
    if (!g || !h_count || iters < 0 || weights_count(model) == -1) return GNND_ERR_INVALID_ARG;
    *h_count = decode_weights_count(model, g->view.E, iters);
    return GNND_OK;
}

extern "C" int gnnd_prepare_weights(int model, int dtype, const void* d_w, void* d_prepared,
                                    void* stream) {
    int n = weights_count(model);
    if (n == -1 || (dtype != GNND_F32 && dtype != GNND_F64)) return GNND_ERR_INVALID_ARG;
    if (n < 0) return GNND_ERR_UNSUPPORTED;     // NBP/V10/V22: decode takes the packed layout as is
    if (n == 0) return GNND_OK;
    if (!d_w || !d_prepared || d_w == d_prepared) return GNND_ERR_INVALID_ARG;
    hipStream_t st = (hipStream_t)stream;
    if (model == GNND_V24 && dtype == GNND_F32) {
        prepare_v24_f32_kernel<<<1, 128, 0, st>>>((const float*)d_w, (float*)d_prepared);
        GNND_LAUNCH_CHECK();
        // [base-2 weights | bound, pad | check-MLP table (fp32)] (ctab_build_kernel)
        if (GNND_V24_CTAB) return launch_ctab_build((const float*)d_w, (float*)d_prepared, st);
        return GNND_OK;
    }
    size_t bytes = (size_t)n * (dtype == GNND_F64 ? 8 : 4);
    GNND_HIP_CHECK(hipMemcpyAsync(d_prepared, d_w, bytes, hipMemcpyDeviceToDevice, st));
    // fp64 decoder_v2_4: [plain | bound, R limit, pad | check-MLP table] (ctab_build_kernel)
    if (model == GNND_V24 && dtype == GNND_F64)
        return launch_ctab_build((const double*)d_w, (double*)d_prepared, st);
    // fp32 CGNNI / QGNNI: [plain | pad | header | message-MLP cells] (pwl_build_kernel)
    if ((model == GNND_CGNNI || model == GNND_QGNNI) && dtype == GNND_F32 && GNND_MLP_PWL)
        return launch_pwl_build((const float*)d_w, (float*)d_prepared, st);
    return GNND_OK;
}

extern "C" int gnnd_prepared_weights_count(int model, int dtype, int64_t* h_count) {
    int n = weights_count(model);
    if (n == -1 || !h_count || (dtype != GNND_F32 && dtype != GNND_F64)) return GNND_ERR_INVALID_ARG;
    if (n < 0) return GNND_ERR_UNSUPPORTED;
    *h_count = model == GNND_V24 && (dtype == GNND_F64 || GNND_V24_CTAB) ? kV24PriorOff
               : (model == GNND_CGNNI || model == GNND_QGNNI) && dtype == GNND_F32 && GNND_MLP_PWL
                   ? kGnnPreparedF32 : n;
    return GNND_OK;
}

extern "C" int gnnd_prepared_weights_count_priors(int model, int dtype, int32_t n_priors,
                                                  int64_t* h_count) {
    if (n_priors == 0) return gnnd_prepared_weights_count(model, dtype, h_count);
    if (!h_count || n_priors < 0 || n_priors > kVtMaxPriors || weights_count(model) == -1)
        return GNND_ERR_INVALID_ARG;
    if (model != GNND_V24 || dtype != GNND_F64) return GNND_ERR_UNSUPPORTED;
    *h_count = kV24PriorOff + (int64_t)n_priors * kVtStride + kVtStrideR;   // (+ the readout MLP's table)
    return GNND_OK;
}

extern "C" int gnnd_prepare_weights_priors(int model, int dtype, const void* d_w, void* d_prepared,
                                           const double* h_priors, int32_t n_priors, void* stream) {
    if (n_priors < 0 || n_priors > kVtMaxPriors || (n_priors > 0 && !h_priors)) return GNND_ERR_INVALID_ARG;
    if (n_priors > 0 && (model != GNND_V24 || dtype != GNND_F64)) return GNND_ERR_UNSUPPORTED;
    const int rc = gnnd_prepare_weights(model, dtype, d_w, d_prepared, stream);
    if (rc != GNND_OK || n_priors == 0) return rc;
    // (after gnnd_prepare_weights on the same stream: its check-MLP build zeroes the header,
    // the table build then writes the count)
    VtPriors pr{};
    for (int i = 0; i < n_priors; ++i) pr.x[i] = h_priors[i];
    vtab_build_kernel<0><<<dim3(vt_cells(kVtInvG), n_priors), 128, 0, (hipStream_t)stream>>>(
        (const double*)d_w, (double*)d_prepared, pr, n_priors, 0);
    GNND_LAUNCH_CHECK();
    // the readout MLP's table after them (same form, no prior, finer cells)
    vtab_build_kernel<1><<<dim3(vt_cells(kVtInvR), 1), 128, 0, (hipStream_t)stream>>>(
        (const double*)d_w, (double*)d_prepared, pr, n_priors, n_priors);
    GNND_LAUNCH_CHECK();
    return GNND_OK;
}

extern "C" int gnnd_decode_tile(const gnnd_graph* g, int model, int dtype, int32_t* h_cw,
                                int32_t* h_lds) {
    if (!g || !h_cw || !h_lds || weights_count(model) == -1) return GNND_ERR_INVALID_ARG;
    if (dtype != GNND_F32 && dtype != GNND_F64 && dtype != GNND_BF16) return GNND_ERR_INVALID_ARG;
    if (dtype == GNND_BF16) dtype = GNND_F32;          // fp32 arithmetic and LDS
    Plan p;
    int rc = plan_for(model, dtype, g, &p);
    if (rc != GNND_OK) return rc;
    *h_cw = p.cw;
    *h_lds = (int32_t)p.lds;
    return GNND_OK;
}

extern "C" int gnnd_decode_plan(const gnnd_graph* g, int model, int dtype, int32_t* h_plan) {
    if (!g || !h_plan || weights_count(model) == -1) return GNND_ERR_INVALID_ARG;
    if (dtype != GNND_F32 && dtype != GNND_F64 && dtype != GNND_BF16) return GNND_ERR_INVALID_ARG;
    if (dtype == GNND_BF16) dtype = GNND_F32;
    Plan p;
    int rc = plan_for(model, dtype, g, &p);
    if (rc != GNND_OK) return rc;
    h_plan[0] = p.cw;
    h_plan[1] = (int32_t)p.lds;
    h_plan[2] = p.resident ? 1 : 0;
    h_plan[3] = p.q;
    h_plan[4] = p.resident ? p.view->vgroup : 0;
    return GNND_OK;
}

extern "C" int gnnd_decode(const gnnd_graph* g, int model, int dtype, const void* d_w,
                           const void* d_x, void* d_out, int64_t batch, int32_t iters,
                           void* stream) {
    int nw = weights_count(model);
    if (!g || nw == -1 || batch < 0 || iters < 0) return GNND_ERR_INVALID_ARG;
    if (dtype != GNND_F32 && dtype != GNND_F64 && dtype != GNND_BF16) return GNND_ERR_INVALID_ARG;
    // nothing to write: an empty batch, or decoder_v2_2's per-layer readout list at T = 0
    if (batch == 0 || (model == GNND_V22 && iters == 0)) return GNND_OK;
    if (!d_x || !d_out || ((nw > 0 || nw == -2) && !d_w)) return GNND_ERR_INVALID_ARG;
    hipStream_t st = (hipStream_t)stream;
    return dispatch_decode(g, model, dtype, d_w, d_x, d_out, batch, iters, st);
}

// ---------------------------------------------------------------------------------------
// debug build: collect every translation unit's check word (gnnd_common.h GNND_DEBUG_TU)
// ---------------------------------------------------------------------------------------
#define GNND_TU_LIST(X) X(graph) X(propagate) X(decode) X(decode_v24) X(decode_qgnni) \
    X(decode_qbp) X(decode_cgnni) X(decode_cbp) X(decode_nbp) X(decode_v10) X(decode_v30) \
    X(decode_v22) X(train) X(sample)
#define GNND_DECL_TU(n) extern "C" unsigned gnnd_debug_take_##n(void);
GNND_TU_LIST(GNND_DECL_TU)

extern "C" int gnnd_debug_enabled(void) {
#ifdef GNND_DEBUG
    return 1;
#else
    return 0;
#endif
}

// OR of every translation unit's debug word (GnndDebugBit bits), cleared; synchronises the
// device first so pending kernels have recorded their checks
extern "C" int gnnd_debug_flags(uint32_t* h_flags) {
    if (!h_flags) return GNND_ERR_INVALID_ARG;
    GNND_HIP_CHECK(hipDeviceSynchronize());
    unsigned v = 0;
#define GNND_TAKE_TU(n) v |= gnnd_debug_take_##n();
    GNND_TU_LIST(GNND_TAKE_TU)
    *h_flags = v;
    return GNND_OK;
}
