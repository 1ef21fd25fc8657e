// conv1d_bf16g.hip — bf16 conv kernel with the weight fragments read from
// global memory (conv1d_impl.h GA: X-only double-buffered LDS, one barrier
// per K-chunk; the packed bf16 image is unchanged).
#include "conv1d_impl.h"

int vits_conv1d_dispatch_bf16g(const vits_conv::ConvGroup& g, hipStream_t s) {
  return vits_conv::conv1d_dispatch<VITS_WDT_BF16, true>(g, s);
}
