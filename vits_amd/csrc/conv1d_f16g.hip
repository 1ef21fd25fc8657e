// conv1d_f16g.hip — fp16 conv kernel with the weight fragments read from
// global memory (conv1d_impl.h GA), as conv1d_bf16g.hip.
#include "conv1d_impl.h"

int vits_conv1d_dispatch_f16g(const vits_conv::ConvGroup& g, hipStream_t s) {
  return vits_conv::conv1d_dispatch<VITS_WDT_F16, true>(g, s);
}
