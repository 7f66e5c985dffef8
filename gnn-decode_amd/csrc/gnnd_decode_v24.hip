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
