// conv1d_f32.hip — f32 instantiation of the conv kernel (conv1d_impl.h).
#include "conv1d_impl.h"

int vits_conv1d_dispatch_f32(const vits_conv::ConvGroup& g, hipStream_t s) {
  return vits_conv::conv1d_dispatch<VITS_WDT_F32>(g, s);
}
