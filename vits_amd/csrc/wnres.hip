// wnres.hip — the residual / skip update between two WN layers of the
// fp16-autocast training step (modules.py:93-182, WN.forward):
//
//   x'      = (x + rs[:, :H]) * mask        (x fp32, rs the fp16 output of
//   out'    = out + rs[:, H:]                the res_skip conv, mask fp32;
//                                            out = 0 when not given)
//   x16'    = fp16(x')                      (the next in_layer conv's input:
//                                            autocast casts it there)
//
// and its gradient, given dx' (fp32), dx16' (fp16, from the next conv's data
// gradient) and dout' (fp32):
//
//   G        = dx' + dx16'                  (both reach x')
//   dx       = G * mask
//   drs      = fp16([G * mask ; dout'])     (the res_skip conv's dY, rows
//                                            :H / H: - one contiguous tensor)
//   dout     = dout'                        (passed through by the caller)
//
// PyTorch runs ~4 kernels forward (add, mul, add, cast) and ~7 backward
// (mul, two casts, the slice-gradient assembly, the fp16 -> fp32 cast of the
// conv's data gradient and two accumulations) per layer.  Tensors are
// contiguous [B][C][T].
#include "common.h"

namespace {

template <typename E>
__global__ __launch_bounds__(256) void wn_update_fwd_kernel(
    const float* __restrict__ x, const E* __restrict__ rs, const float* __restrict__ mask,
    const float* __restrict__ out, float* __restrict__ xn, E* __restrict__ x16,
    float* __restrict__ outn, int H, int T, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * 256) {
    const int64_t bh = i / T;
    const int t = (int)(i - bh * T);
    const int64_t b = bh / H;
    const int c = (int)(bh - b * H);
    const int64_t rrow = (b * 2 * H + c) * T + t;
    const float m = mask[b * T + t];
    const float v = (x[i] + (float)rs[rrow]) * m;
    xn[i] = v;
    x16[i] = (E)v;
    outn[i] = (out ? out[i] : 0.f) + (float)rs[rrow + (int64_t)H * T];
  }
}

template <typename E>
__global__ __launch_bounds__(256) void wn_update_bwd_kernel(
    const float* __restrict__ gx, const E* __restrict__ gx16, const float* __restrict__ gout,
    const float* __restrict__ mask, float* __restrict__ dx, E* __restrict__ drs, int H, int T,
    int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * 256) {
    const int64_t bh = i / T;
    const int t = (int)(i - bh * T);
    const int64_t b = bh / H;
    const int c = (int)(bh - b * H);
    const int64_t rrow = (b * 2 * H + c) * T + t;
    float g = gx ? gx[i] : 0.f;
    if (gx16) g += (float)gx16[i];
    const float d = g * mask[b * T + t];
    dx[i] = d;
    drs[rrow] = (E)d;
    drs[rrow + (int64_t)H * T] = (E)(gout ? gout[i] : 0.f);
  }
}

int grid_for(int64_t n) {
  const int64_t want = (n + 255) / 256;
  return (int)(want < 8192 ? want : 8192);
}

}  // namespace

extern "C" int vits_wn_update_forward(const float* x, const void* rs, const float* mask,
                                      const float* out, float* x_new, void* x16_new,
                                      float* out_new, int batch, int H, int T, int wdtype,
                                      void* stream) {
  VITS_CHECK_ARG(x && rs && mask && x_new && x16_new && out_new && batch > 0 && H > 0 && T > 0);
  VITS_CHECK_ARG(wdtype == VITS_WDT_F16 || wdtype == VITS_WDT_BF16);
  const int64_t n = (int64_t)batch * H * T;
  hipStream_t s = as_stream(stream);
  if (wdtype == VITS_WDT_F16)
    hipLaunchKernelGGL(wn_update_fwd_kernel<_Float16>, dim3(grid_for(n)), dim3(256), 0, s, x,
                       (const _Float16*)rs, mask, out, x_new, (_Float16*)x16_new, out_new, H, T, n);
  else
    hipLaunchKernelGGL(wn_update_fwd_kernel<__bf16>, dim3(grid_for(n)), dim3(256), 0, s, x,
                       (const __bf16*)rs, mask, out, x_new, (__bf16*)x16_new, out_new, H, T, n);
  return vits_launch_status();
}

extern "C" int vits_wn_update_backward(const float* gx, const void* gx16, const float* gout,
                                       const float* mask, float* dx, void* drs, int batch, int H,
                                       int T, int wdtype, void* stream) {
  VITS_CHECK_ARG(mask && dx && drs && batch > 0 && H > 0 && T > 0);
  VITS_CHECK_ARG(wdtype == VITS_WDT_F16 || wdtype == VITS_WDT_BF16);
  const int64_t n = (int64_t)batch * H * T;
  hipStream_t s = as_stream(stream);
  if (wdtype == VITS_WDT_F16)
    hipLaunchKernelGGL(wn_update_bwd_kernel<_Float16>, dim3(grid_for(n)), dim3(256), 0, s, gx,
                       (const _Float16*)gx16, gout, mask, dx, (_Float16*)drs, H, T, n);
  else
    hipLaunchKernelGGL(wn_update_bwd_kernel<__bf16>, dim3(grid_for(n)), dim3(256), 0, s, gx,
                       (const __bf16*)gx16, gout, mask, dx, (__bf16*)drs, H, T, n);
  return vits_launch_status();
}
