// gnnd_decode_v10.hip — kernel instantiations for model GNND_V10 (see gnnd_decode_impl.h).
#include "gnnd_decode_impl.h"

GNND_DEBUG_TU(decode_v10)

int gnnd_launch_v10(const gnnd_graph* g, int dtype, const void* w, const void* x, void* out,
                       int64_t B, int iters, hipStream_t st) {
    return launch_model<GNND_V10>(g, dtype, w, x, out, B, iters, st);
}
