// gnnd_decode_v22.hip — kernel instantiations for model GNND_V22 (see gnnd_decode_impl.h).
#include "gnnd_decode_impl.h"

GNND_DEBUG_TU(decode_v22)

int gnnd_launch_v22(const gnnd_graph* g, int dtype, const void* w, const void* x, void* out,
                    int64_t B, int iters, hipStream_t st) {
    return launch_model<GNND_V22>(g, dtype, w, x, out, B, iters, st);
}
