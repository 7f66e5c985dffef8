// gnnd_decode_cbp.hip — kernel instantiations for model GNND_CBP (see gnnd_decode_impl.h).
#include "gnnd_decode_impl.h"

GNND_DEBUG_TU(decode_cbp)

int gnnd_launch_cbp(const gnnd_graph* g, int dtype, const void* w, const void* x, void* out,
                       int64_t B, int iters, hipStream_t st) {
    return launch_model<GNND_CBP>(g, dtype, w, x, out, B, iters, st);
}
