// gnnd_decode_nbp.hip — kernel instantiations for model GNND_NBP (see gnnd_decode_impl.h).
#include "gnnd_decode_impl.h"

GNND_DEBUG_TU(decode_nbp)

int gnnd_launch_nbp(const gnnd_graph* g, int dtype, const void* w, const void* x, void* out,
                       int64_t B, int iters, hipStream_t st) {
    return launch_model<GNND_NBP>(g, dtype, w, x, out, B, iters, st);
}
