// gnnd_decode_cgnni.hip — kernel instantiations for model GNND_CGNNI (see gnnd_decode_impl.h).
#include "gnnd_decode_impl.h"

GNND_DEBUG_TU(decode_cgnni)

int gnnd_launch_cgnni(const gnnd_graph* g, int dtype, const void* w, const void* x, void* out,
                       int64_t B, int iters, hipStream_t st) {
    return launch_model<GNND_CGNNI>(g, dtype, w, x, out, B, iters, st);
}
