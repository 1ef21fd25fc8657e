// conv1d_f32p.hip — split-fp32 instantiation with host-split weights
// (conv1d_impl.h, VITS_WDT_F32P): the weights arrive as three bf16 planes
// (hi, mid, lo; split once at pack time instead of per fragment in every
// workgroup), their A fragments are read from global memory into registers
// one k-step ahead, and the LDS holds only the (double-buffered) input
// window - one barrier per K-chunk.  Same six MFMAs in the same order as
// VITS_WDT_F32S, so the results are bitwise those of the F32S kernel.
#include "conv1d_impl.h"

int vits_conv1d_dispatch_f32p(const vits_conv::ConvGroup& g, hipStream_t s) {
  return vits_conv::conv1d_dispatch<VITS_WDT_F32P>(g, s);
}
