// gnnd_decode_qbp.hip — kernel instantiations for model GNND_QBP (see gnnd_decode_impl.h).
#include "gnnd_decode_impl.h"

GNND_DEBUG_TU(decode_qbp)

int gnnd_launch_qbp(const gnnd_graph* g, int dtype, const void* w, const void* x, void* out,
                       int64_t B, int iters, hipStream_t st) {
    return launch_model<GNND_QBP>(g, dtype, w, x, out, B, iters, st);
}
