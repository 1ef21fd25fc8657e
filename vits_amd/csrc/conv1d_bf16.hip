// conv1d_bf16.hip — bf16 instantiation of the conv kernel (conv1d_impl.h).
#include "conv1d_impl.h"

int vits_conv1d_dispatch_bf16(const vits_conv::ConvGroup& g, hipStream_t s) {
  return vits_conv::conv1d_dispatch<VITS_WDT_BF16>(g, s);
}
