// gate.hip — the WaveNet-style gate of the training step and its gradient.
//
//   acts[b][p][t] = tanh(x[b][p][t] + g[b][p]) * sigmoid(x[b][H+p][t] + g[b][H+p])
//
// modules.WN (modules.py:139-146, `commons.fused_add_tanh_sigmoid_multiply`
// in the reference's WN) and ResBlock2 (modules.py:253-255) run it on the
// output of a conv under autograd: ~5 elementwise kernels forward and ~8
// backward in PyTorch, here one each.  The backward also reduces the cond
// gradient dg[b][c] = sum_t dx[b][c][t] in the same pass (one workgroup per
// (b, p) row pair, no atomics).  fp32 in / out; the rows are time-contiguous
// with arbitrary batch / channel strides (channel slices of a larger
// buffer are fine).
#include "common.h"

namespace {

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + __expf(-x)); }

__global__ __launch_bounds__(256) void gate_fwd_kernel(const float* __restrict__ x, int64_t x_bs,
                                                      int x_cs, const float* __restrict__ g,
                                                      int64_t g_bs, float* __restrict__ y,
                                                      int64_t y_bs, int y_cs, int H, int T) {
  const int p = blockIdx.x;
  const int b = blockIdx.y;
  const float* xa = x + (int64_t)b * x_bs + (int64_t)p * x_cs;
  const float* xb = xa + (int64_t)H * x_cs;
  float* yr = y + (int64_t)b * y_bs + (int64_t)p * y_cs;
  const float ga = g ? g[(int64_t)b * g_bs + p] : 0.f;
  const float gb = g ? g[(int64_t)b * g_bs + H + p] : 0.f;
  for (int t = threadIdx.x; t < T; t += 256) {
    const float a = tanhf(xa[t] + ga);
    const float s = sigm(xb[t] + gb);
    yr[t] = a * s;
  }
}

__global__ __launch_bounds__(256) void gate_bwd_kernel(const float* __restrict__ dy, int64_t dy_bs,
                                                      int dy_cs, const float* __restrict__ x,
                                                      int64_t x_bs, int x_cs,
                                                      const float* __restrict__ g, int64_t g_bs,
                                                      float* __restrict__ dx, int64_t dx_bs,
                                                      int dx_cs, float* __restrict__ dg, int H,
                                                      int T) {
  __shared__ float red[2][4];
  const int p = blockIdx.x;
  const int b = blockIdx.y;
  const float* xa = x + (int64_t)b * x_bs + (int64_t)p * x_cs;
  const float* xb = xa + (int64_t)H * x_cs;
  const float* dyr = dy + (int64_t)b * dy_bs + (int64_t)p * dy_cs;
  float* dxa = dx + (int64_t)b * dx_bs + (int64_t)p * dx_cs;
  float* dxb = dxa + (int64_t)H * dx_cs;
  const float ga = g ? g[(int64_t)b * g_bs + p] : 0.f;
  const float gb = g ? g[(int64_t)b * g_bs + H + p] : 0.f;
  float sa = 0.f, sb = 0.f;
  for (int t = threadIdx.x; t < T; t += 256) {
    const float a = tanhf(xa[t] + ga);
    const float s = sigm(xb[t] + gb);
    const float d = dyr[t];
    const float da = d * s * (1.0f - a * a);
    const float db = d * a * s * (1.0f - s);
    dxa[t] = da;
    dxb[t] = db;
    sa += da;
    sb += db;
  }
  if (dg) {
    sa = wave_sum(sa);
    sb = wave_sum(sb);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
      red[0][w] = sa;
      red[1][w] = sb;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      dg[(int64_t)b * 2 * H + p] = red[0][0] + red[0][1] + red[0][2] + red[0][3];
      dg[(int64_t)b * 2 * H + H + p] = red[1][0] + red[1][1] + red[1][2] + red[1][3];
    }
  }
}

}  // namespace

extern "C" int vits_gate_forward(const float* x, int64_t x_bstride, int32_t x_cstride,
                                 const float* g, int64_t g_bstride, float* y, int64_t y_bstride,
                                 int32_t y_cstride, int batch, int half_channels, int t_len,
                                 void* stream) {
  VITS_CHECK_ARG(x && y && batch > 0 && half_channels > 0 && t_len > 0);
  VITS_CHECK_SHAPE(batch <= 65535);
  hipLaunchKernelGGL(gate_fwd_kernel, dim3(half_channels, batch), dim3(256), 0, as_stream(stream),
                     x, x_bstride, x_cstride, g, g_bstride, y, y_bstride, y_cstride, half_channels,
                     t_len);
  return vits_launch_status();
}

extern "C" int vits_gate_backward(const float* dy, int64_t dy_bstride, int32_t dy_cstride,
                                  const float* x, int64_t x_bstride, int32_t x_cstride,
                                  const float* g, int64_t g_bstride, float* dx, int64_t dx_bstride,
                                  int32_t dx_cstride, float* dg, int batch, int half_channels,
                                  int t_len, void* stream) {
  VITS_CHECK_ARG(dy && x && dx && batch > 0 && half_channels > 0 && t_len > 0);
  VITS_CHECK_SHAPE(batch <= 65535);
  hipLaunchKernelGGL(gate_bwd_kernel, dim3(half_channels, batch), dim3(256), 0, as_stream(stream),
                     dy, dy_bstride, dy_cstride, x, x_bstride, x_cstride, g, g_bstride, dx,
                     dx_bstride, dx_cstride, dg, half_channels, t_len);
  return vits_launch_status();
}
