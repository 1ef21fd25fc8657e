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

// ---------------------------------------------------------------------------
// The rest of a mean-only coupling layer's element-wise work in the fp16-
// autocast training step (ResidualCouplingLayer.forward, modules.py:314-360;
// ResidualCouplingBlock.forward, models.py:219-235; PosteriorEncoder /
// coupling WN output, modules.py:182):
//
//  mask_cast:  h = pre(x0) * x_mask (the 16-bit conv output times the fp32
//              mask, fp32), and h rounded to the 16-bit type (the WN's first
//              in_layer conv input, which autocast would cast there).
//              backward: G = dh + dh16 (either NULL = 0), dy = fp16(G * mask)
//  wn_final:   the WN output (output + rs) * x_mask, returned rounded to the
//              16-bit type (its only consumer is the post / proj conv, which
//              autocast feeds fp16).  backward: d = dy16 * mask, dout = d
//              (fp32), drs = fp16(d)
//  coupling:   m = post(h) * x_mask; with logs = 0 (mean_only) the
//              reference's x1 * exp(logs) is x1 exactly, so
//                forward:  x1' = m + x1 * x_mask,   reverse: (x1 - m) * x_mask
//              and out = cat(x0, x1'), optionally channel-flipped (the Flip
//              module that follows, folded into the store).
//              backward (g = d out): gx0 = g0, gx1 = g1 * mask, dp = fp16(+-
//              g1 * mask) (the reverse direction's m enters with a minus).
// All tensors contiguous [B][C][T]; mask [B][1][T] fp32.
// ---------------------------------------------------------------------------

template <typename E>
__global__ __launch_bounds__(256) void mask_cast_fwd_kernel(
    const E* __restrict__ y, const float* __restrict__ mask, float* __restrict__ h,
    E* __restrict__ h16, int C, int T, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * 256) {
    const int64_t bc = i / T;
    const int t = (int)(i - bc * T);
    const int64_t b = bc / C;
    const float v = (float)y[i] * mask[b * T + t];
    h[i] = v;
    h16[i] = (E)v;
  }
}

template <typename E>
__global__ __launch_bounds__(256) void mask_cast_bwd_kernel(
    const float* __restrict__ gh, const E* __restrict__ gh16, const float* __restrict__ mask,
    E* __restrict__ dy, int C, int T, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * 256) {
    const int64_t bc = i / T;
    const int t = (int)(i - bc * T);
    const int64_t b = bc / C;
    float g = gh ? gh[i] : 0.f;
    if (gh16) g += (float)gh16[i];
    dy[i] = (E)(g * mask[b * T + t]);
  }
}

template <typename E>
__global__ __launch_bounds__(256) void wn_final_fwd_kernel(
    const float* __restrict__ out, const E* __restrict__ rs, const float* __restrict__ mask,
    E* __restrict__ o16, int C, int T, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * 256) {
    const int64_t bc = i / T;
    const int t = (int)(i - bc * T);
    const int64_t b = bc / C;
    const float v = ((out ? out[i] : 0.f) + (float)rs[i]) * mask[b * T + t];
    o16[i] = (E)v;
  }
}

template <typename E>
__global__ __launch_bounds__(256) void wn_final_bwd_kernel(
    const E* __restrict__ g16, const float* __restrict__ mask, float* __restrict__ dout,
    E* __restrict__ drs, int C, int T, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * 256) {
    const int64_t bc = i / T;
    const int t = (int)(i - bc * T);
    const int64_t b = bc / C;
    const float d = (float)g16[i] * mask[b * T + t];
    if (dout) dout[i] = d;
    drs[i] = (E)d;
  }
}

// i runs over [B][h][T]: each thread moves channel c of x0 and of x1
template <typename E>
__global__ __launch_bounds__(256) void coupling_fwd_kernel(
    const float* __restrict__ x, const E* __restrict__ p, const float* __restrict__ mask,
    float* __restrict__ out, int h, int T, int reverse, int flip, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * 256) {
    const int64_t bc = i / T;
    const int t = (int)(i - bc * T);
    const int64_t b = bc / h;
    const int c = (int)(bc - b * h);
    const float mk = mask[b * T + t];
    const float m = (float)p[i] * mk;
    const int64_t xb = b * 2 * h;
    const float x0 = x[(xb + c) * T + t];
    const float x1 = x[(xb + h + c) * T + t];
    const float v = reverse ? (x1 - m) * mk : m + x1 * mk;
    const int c0 = flip ? 2 * h - 1 - c : c;
    const int c1 = flip ? h - 1 - c : h + c;
    out[(xb + c0) * T + t] = x0;
    out[(xb + c1) * T + t] = v;
  }
}

template <typename E>
__global__ __launch_bounds__(256) void coupling_bwd_kernel(
    const float* __restrict__ g, const float* __restrict__ mask, float* __restrict__ gx,
    E* __restrict__ gp, int h, int T, int reverse, int flip, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * 256) {
    const int64_t bc = i / T;
    const int t = (int)(i - bc * T);
    const int64_t b = bc / h;
    const int c = (int)(bc - b * h);
    const float mk = mask[b * T + t];
    const int64_t xb = b * 2 * h;
    const int c0 = flip ? 2 * h - 1 - c : c;
    const int c1 = flip ? h - 1 - c : h + c;
    const float g0 = g[(xb + c0) * T + t];
    const float g1m = g[(xb + c1) * T + t] * mk;
    gx[(xb + c) * T + t] = g0;
    gx[(xb + h + c) * T + t] = g1m;
    gp[i] = (E)(reverse ? -g1m : g1m);
  }
}

extern "C" int vits_mask_cast_forward(const void* y, const float* mask, float* h, void* h16,
                                      int batch, int C, int T, int wdtype, void* stream) {
  VITS_CHECK_ARG(y && mask && h && h16 && batch > 0 && C > 0 && T > 0);
  VITS_CHECK_ARG(wdtype == VITS_WDT_F16 || wdtype == VITS_WDT_BF16);
  const int64_t n = (int64_t)batch * C * T;
  hipStream_t s = as_stream(stream);
  if (wdtype == VITS_WDT_F16)
    hipLaunchKernelGGL(mask_cast_fwd_kernel<_Float16>, dim3(grid_for(n)), dim3(256), 0, s,
                       (const _Float16*)y, mask, h, (_Float16*)h16, C, T, n);
  else
    hipLaunchKernelGGL(mask_cast_fwd_kernel<__bf16>, dim3(grid_for(n)), dim3(256), 0, s,
                       (const __bf16*)y, mask, h, (__bf16*)h16, C, T, n);
  return vits_launch_status();
}

extern "C" int vits_mask_cast_backward(const float* gh, const void* gh16, const float* mask,
                                       void* dy, int batch, int C, int T, int wdtype,
                                       void* stream) {
  VITS_CHECK_ARG(mask && dy && batch > 0 && C > 0 && T > 0);
  VITS_CHECK_ARG(wdtype == VITS_WDT_F16 || wdtype == VITS_WDT_BF16);
  const int64_t n = (int64_t)batch * C * T;
  hipStream_t s = as_stream(stream);
  if (wdtype == VITS_WDT_F16)
    hipLaunchKernelGGL(mask_cast_bwd_kernel<_Float16>, dim3(grid_for(n)), dim3(256), 0, s, gh,
                       (const _Float16*)gh16, mask, (_Float16*)dy, C, T, n);
  else
    hipLaunchKernelGGL(mask_cast_bwd_kernel<__bf16>, dim3(grid_for(n)), dim3(256), 0, s, gh,
                       (const __bf16*)gh16, mask, (__bf16*)dy, C, T, n);
  return vits_launch_status();
}

extern "C" int vits_wn_final_forward(const float* out, const void* rs, const float* mask,
                                     void* o16, int batch, int C, int T, int wdtype,
                                     void* stream) {
  VITS_CHECK_ARG(rs && mask && o16 && batch > 0 && C > 0 && T > 0);
  VITS_CHECK_ARG(wdtype == VITS_WDT_F16 || wdtype == VITS_WDT_BF16);
  const int64_t n = (int64_t)batch * C * T;
  hipStream_t s = as_stream(stream);
  if (wdtype == VITS_WDT_F16)
    hipLaunchKernelGGL(wn_final_fwd_kernel<_Float16>, dim3(grid_for(n)), dim3(256), 0, s, out,
                       (const _Float16*)rs, mask, (_Float16*)o16, C, T, n);
  else
    hipLaunchKernelGGL(wn_final_fwd_kernel<__bf16>, dim3(grid_for(n)), dim3(256), 0, s, out,
                       (const __bf16*)rs, mask, (__bf16*)o16, C, T, n);
  return vits_launch_status();
}

extern "C" int vits_wn_final_backward(const void* g16, const float* mask, float* dout, void* drs,
                                      int batch, int C, int T, int wdtype, void* stream) {
  VITS_CHECK_ARG(g16 && mask && drs && batch > 0 && C > 0 && T > 0);
  VITS_CHECK_ARG(wdtype == VITS_WDT_F16 || wdtype == VITS_WDT_BF16);
  const int64_t n = (int64_t)batch * C * T;
  hipStream_t s = as_stream(stream);
  if (wdtype == VITS_WDT_F16)
    hipLaunchKernelGGL(wn_final_bwd_kernel<_Float16>, dim3(grid_for(n)), dim3(256), 0, s,
                       (const _Float16*)g16, mask, dout, (_Float16*)drs, C, T, n);
  else
    hipLaunchKernelGGL(wn_final_bwd_kernel<__bf16>, dim3(grid_for(n)), dim3(256), 0, s,
                       (const __bf16*)g16, mask, dout, (__bf16*)drs, C, T, n);
  return vits_launch_status();
}

extern "C" int vits_coupling_forward(const float* x, const void* p, const float* mask, float* out,
                                     int batch, int half, int T, int reverse, int flip,
                                     int wdtype, void* stream) {
  VITS_CHECK_ARG(x && p && mask && out && out != x && batch > 0 && half > 0 && T > 0);
  VITS_CHECK_ARG(wdtype == VITS_WDT_F16 || wdtype == VITS_WDT_BF16);
  const int64_t n = (int64_t)batch * half * T;
  hipStream_t s = as_stream(stream);
  if (wdtype == VITS_WDT_F16)
    hipLaunchKernelGGL(coupling_fwd_kernel<_Float16>, dim3(grid_for(n)), dim3(256), 0, s, x,
                       (const _Float16*)p, mask, out, half, T, reverse, flip, n);
  else
    hipLaunchKernelGGL(coupling_fwd_kernel<__bf16>, dim3(grid_for(n)), dim3(256), 0, s, x,
                       (const __bf16*)p, mask, out, half, T, reverse, flip, n);
  return vits_launch_status();
}

extern "C" int vits_coupling_backward(const float* g, const float* mask, float* gx, void* gp,
                                      int batch, int half, int T, int reverse, int flip,
                                      int wdtype, void* stream) {
  VITS_CHECK_ARG(g && mask && gx && gp && gx != g && batch > 0 && half > 0 && T > 0);
  VITS_CHECK_ARG(wdtype == VITS_WDT_F16 || wdtype == VITS_WDT_BF16);
  const int64_t n = (int64_t)batch * half * T;
  hipStream_t s = as_stream(stream);
  if (wdtype == VITS_WDT_F16)
    hipLaunchKernelGGL(coupling_bwd_kernel<_Float16>, dim3(grid_for(n)), dim3(256), 0, s, g,
                       mask, gx, (_Float16*)gp, half, T, reverse, flip, n);
  else
    hipLaunchKernelGGL(coupling_bwd_kernel<__bf16>, dim3(grid_for(n)), dim3(256), 0, s, g, mask,
                       gx, (__bf16*)gp, half, T, reverse, flip, n);
  return vits_launch_status();
}
