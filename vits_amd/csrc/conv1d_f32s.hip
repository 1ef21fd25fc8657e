// conv1d_f32s.hip — split-fp32 instantiation of the conv kernel
// (conv1d_impl.h, VITS_WDT_F32S): fp32 operands as three exact bf16 terms on
// the bf16 MFMA (six v_mfma_f32_32x32x16_bf16 per 16-deep k-step = 2.7x
// fewer MFMA cycles than the 32x32x2 f32 form for the same fp32-level error).
#include "conv1d_impl.h"

int vits_conv1d_dispatch_f32s(const vits_conv::ConvGroup& g, hipStream_t s) {
  return vits_conv::conv1d_dispatch<VITS_WDT_F32S>(g, s);
}
