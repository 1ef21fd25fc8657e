// gate.hip — the WaveNet-style gate of the training step and its gradient.
//
//   acts[b][p][t] = tanh(x[b][p][t] + g[b][p]) * sigmoid(x[b][H+p][t] + g[b][H+p])
//
// modules.WN (modules.py:139-146, `commons.fused_add_tanh_sigmoid_multiply`
// in the reference's WN) and ResBlock2 (modules.py:253-255) run it on the
// output of a conv under autograd: ~5 elementwise kernels forward and ~8
// backward in PyTorch, here one each.  The backward also reduces the cond
// gradient dg[b][c] = sum_t dx[b][c][t] in the same pass (one workgroup per
// (b, p) row pair, no atomics).  fp32 in / out, or (the *_io16 entry
// points) x / g / y / dy / dx of a 16-bit type with fp32 math and an fp32
// dg; the rows are time-contiguous with arbitrary batch / channel strides
// (channel slices of a larger buffer are fine).
#include "common.h"

namespace {

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + __expf(-x)); }

template <typename E>
__global__ __launch_bounds__(256) void gate_fwd_kernel(const E* __restrict__ x, int64_t x_bs,
                                                      int x_cs, const E* __restrict__ g,
                                                      int64_t g_bs, E* __restrict__ y,
                                                      int64_t y_bs, int y_cs, int H, int T) {
  const int p = blockIdx.x;
  const int b = blockIdx.y;
  const E* xa = x + (int64_t)b * x_bs + (int64_t)p * x_cs;
  const E* xb = xa + (int64_t)H * x_cs;
  E* yr = y + (int64_t)b * y_bs + (int64_t)p * y_cs;
  const float ga = g ? (float)g[(int64_t)b * g_bs + p] : 0.f;
  const float gb = g ? (float)g[(int64_t)b * g_bs + H + p] : 0.f;
  for (int t = threadIdx.x; t < T; t += 256) {
    const float a = tanhf((float)xa[t] + ga);
    const float s = sigm((float)xb[t] + gb);
    yr[t] = (E)(a * s);
  }
}

// V4: rows 4-element aligned (T % 4 == 0, strides and bases aligned): one
// 4-element load / store per row and thread - the element-wise map issued a
// 2-byte access per lane (half-width transactions) and left most of a
// T = 500 row's threads idle after two iterations.  One workgroup = one
// (b, p) row pair; dg[b * dg_bs + p] / [... + H + p] (dg_bs = 2H: the
// [B][2H] cond gradient; larger: a column slice of a wider buffer).
template <typename E, bool V4>
__device__ __forceinline__ void gate_bwd_rows(const E* __restrict__ dy, int64_t dy_bs, int dy_cs,
                                              const E* __restrict__ x, int64_t x_bs, int x_cs,
                                              const E* __restrict__ g, int64_t g_bs,
                                              E* __restrict__ dx, int64_t dx_bs, int dx_cs,
                                              float* __restrict__ dg, int64_t dg_bs, int H, int T,
                                              int p, int b) {
  __shared__ float red[2][4];
  const E* xa = x + (int64_t)b * x_bs + (int64_t)p * x_cs;
  const E* xb = xa + (int64_t)H * x_cs;
  const E* dyr = dy + (int64_t)b * dy_bs + (int64_t)p * dy_cs;
  E* dxa = dx + (int64_t)b * dx_bs + (int64_t)p * dx_cs;
  E* dxb = dxa + (int64_t)H * dx_cs;
  const float ga = g ? (float)g[(int64_t)b * g_bs + p] : 0.f;
  const float gb = g ? (float)g[(int64_t)b * g_bs + H + p] : 0.f;
  float sa = 0.f, sb = 0.f;
  if constexpr (V4) {
    typedef E e4 __attribute__((ext_vector_type(4)));
    for (int t = 4 * threadIdx.x; t < T; t += 1024) {
      const e4 xav = *reinterpret_cast<const e4*>(xa + t);
      const e4 xbv = *reinterpret_cast<const e4*>(xb + t);
      const e4 dv = *reinterpret_cast<const e4*>(dyr + t);
      e4 dav, dbv;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float a = tanhf((float)xav[i] + ga);
        const float s = sigm((float)xbv[i] + gb);
        const float d = (float)dv[i];
        dav[i] = (E)(d * s * (1.0f - a * a));
        dbv[i] = (E)(d * a * s * (1.0f - s));
        sa += (float)dav[i];
        sb += (float)dbv[i];
      }
      *reinterpret_cast<e4*>(dxa + t) = dav;
      *reinterpret_cast<e4*>(dxb + t) = dbv;
    }
  } else
  for (int t = threadIdx.x; t < T; t += 256) {
    const float a = tanhf((float)xa[t] + ga);
    const float s = sigm((float)xb[t] + gb);
    const float d = (float)dyr[t];
    // dg sums the gradients as stored (rounded to E, as the reference's
    // autocast sum of the fp16 gradient would see them)
    const E da = (E)(d * s * (1.0f - a * a));
    const E db = (E)(d * a * s * (1.0f - s));
    dxa[t] = da;
    dxb[t] = db;
    sa += (float)da;
    sb += (float)db;
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
      dg[(int64_t)b * dg_bs + p] = red[0][0] + red[0][1] + red[0][2] + red[0][3];
      dg[(int64_t)b * dg_bs + H + p] = red[1][0] + red[1][1] + red[1][2] + red[1][3];
    }
  }
}

template <typename E, bool V4 = false>
__global__ __launch_bounds__(256) void gate_bwd_kernel(const E* __restrict__ dy, int64_t dy_bs,
                                                      int dy_cs, const E* __restrict__ x,
                                                      int64_t x_bs, int x_cs,
                                                      const E* __restrict__ g, int64_t g_bs,
                                                      E* __restrict__ dx, int64_t dx_bs,
                                                      int dx_cs, float* __restrict__ dg, int H,
                                                      int T) {
  gate_bwd_rows<E, V4>(dy, dy_bs, dy_cs, x, x_bs, x_cs, g, g_bs, dx, dx_bs, dx_cs, dg, 2 * H, H,
                       T, blockIdx.x, blockIdx.y);
}

// up to GATE_JOBS independent gate backwards of one batch / length (the
// three ResBlock2 branches of a Generator stage) as one grid: blockIdx.z
// selects the job
constexpr int GATE_JOBS = 4;
struct GateJobs {
  vits_gate_bwd_job j[GATE_JOBS];
  int n;
};

template <typename E, bool V4>
__global__ __launch_bounds__(256) void gate_bwd_multi_kernel(const GateJobs J, int T) {
  const vits_gate_bwd_job& q = J.j[blockIdx.z];
  if ((int)blockIdx.x >= q.half_channels) return;
  gate_bwd_rows<E, V4>(static_cast<const E*>(q.dy), q.dy_bstride, q.dy_cstride,
                       static_cast<const E*>(q.x), q.x_bstride, q.x_cstride,
                       static_cast<const E*>(q.g), q.g_bstride, static_cast<E*>(q.dx),
                       q.dx_bstride, q.dx_cstride, q.dg, q.dg_bstride, q.half_channels, T,
                       blockIdx.x, blockIdx.y);
}

}  // namespace

extern "C" int vits_gate_forward(const float* x, int64_t x_bstride, int32_t x_cstride,
                                 const float* g, int64_t g_bstride, float* y, int64_t y_bstride,
                                 int32_t y_cstride, int batch, int half_channels, int t_len,
                                 void* stream) {
  VITS_CHECK_ARG(x && y && batch > 0 && half_channels > 0 && t_len > 0);
  VITS_CHECK_SHAPE(batch <= 65535);
  hipLaunchKernelGGL(gate_fwd_kernel<float>, dim3(half_channels, batch), dim3(256), 0, as_stream(stream),
                     x, x_bstride, x_cstride, g, g_bstride, y, y_bstride, y_cstride, half_channels,
                     t_len);
  return count_ok(vits_launch_status(), VITS_CNT_GATE_F32);
}

extern "C" int vits_gate_backward(const float* dy, int64_t dy_bstride, int32_t dy_cstride,
                                  const float* x, int64_t x_bstride, int32_t x_cstride,
                                  const float* g, int64_t g_bstride, float* dx, int64_t dx_bstride,
                                  int32_t dx_cstride, float* dg, int batch, int half_channels,
                                  int t_len, void* stream) {
  VITS_CHECK_ARG(dy && x && dx && batch > 0 && half_channels > 0 && t_len > 0);
  VITS_CHECK_SHAPE(batch <= 65535);
  hipLaunchKernelGGL(gate_bwd_kernel<float>, dim3(half_channels, batch), dim3(256), 0, as_stream(stream),
                     dy, dy_bstride, dy_cstride, x, x_bstride, x_cstride, g, g_bstride, dx,
                     dx_bstride, dx_cstride, dg, half_channels, t_len);
  return count_ok(vits_launch_status(), VITS_CNT_GATE_F32);
}

extern "C" int vits_gate_forward_io16(const void* x, int64_t x_bstride, int32_t x_cstride,
                                      const void* g, int64_t g_bstride, void* y,
                                      int64_t y_bstride, int32_t y_cstride, int batch,
                                      int half_channels, int t_len, int wdtype, void* stream) {
  VITS_CHECK_ARG(x && y && batch > 0 && half_channels > 0 && t_len > 0);
  VITS_CHECK_SHAPE(batch <= 65535);
  const dim3 grid(half_channels, batch);
  hipStream_t s = as_stream(stream);
#define VITS_GATE_FWD(E)                                                                           \
  hipLaunchKernelGGL(gate_fwd_kernel<E>, grid, dim3(256), 0, s, static_cast<const E*>(x),         \
                     x_bstride, x_cstride, static_cast<const E*>(g), g_bstride, static_cast<E*>(y), \
                     y_bstride, y_cstride, half_channels, t_len)
  if (wdtype == VITS_WDT_F16)
    VITS_GATE_FWD(_Float16);
  else if (wdtype == VITS_WDT_BF16)
    VITS_GATE_FWD(__bf16);
  else
    return VITS_E_ARG;
#undef VITS_GATE_FWD
  return count_ok(vits_launch_status(), VITS_CNT_GATE_16);
}

extern "C" int vits_gate_backward_io16(const void* dy, int64_t dy_bstride, int32_t dy_cstride,
                                       const void* x, int64_t x_bstride, int32_t x_cstride,
                                       const void* g, int64_t g_bstride, void* dx,
                                       int64_t dx_bstride, int32_t dx_cstride, float* dg, int batch,
                                       int half_channels, int t_len, int wdtype, void* stream) {
  VITS_CHECK_ARG(dy && x && dx && batch > 0 && half_channels > 0 && t_len > 0);
  VITS_CHECK_SHAPE(batch <= 65535);
  const dim3 grid(half_channels, batch);
  hipStream_t s = as_stream(stream);
  const bool v4 = (t_len & 3) == 0 && ((dy_bstride | dy_cstride | x_bstride | x_cstride |
                                        dx_bstride | dx_cstride | (int64_t)half_channels) & 3) == 0 &&
                  ((reinterpret_cast<uintptr_t>(dy) | reinterpret_cast<uintptr_t>(x) |
                    reinterpret_cast<uintptr_t>(dx)) & 7) == 0;
#define VITS_GATE_BWD(E)                                                                           \
  if (v4)                                                                                          \
    hipLaunchKernelGGL((gate_bwd_kernel<E, true>), grid, dim3(256), 0, s,                         \
                       static_cast<const E*>(dy), dy_bstride, dy_cstride,                          \
                       static_cast<const E*>(x), x_bstride, x_cstride, static_cast<const E*>(g),   \
                       g_bstride, static_cast<E*>(dx), dx_bstride, dx_cstride, dg, half_channels,  \
                       t_len);                                                                     \
  else                                                                                             \
    hipLaunchKernelGGL(gate_bwd_kernel<E>, grid, dim3(256), 0, s, static_cast<const E*>(dy),      \
                       dy_bstride, dy_cstride, static_cast<const E*>(x), x_bstride, x_cstride,    \
                       static_cast<const E*>(g), g_bstride, static_cast<E*>(dx), dx_bstride,     \
                       dx_cstride, dg, half_channels, t_len)
  if (wdtype == VITS_WDT_F16)
    VITS_GATE_BWD(_Float16);
  else if (wdtype == VITS_WDT_BF16)
    VITS_GATE_BWD(__bf16);
  else
    return VITS_E_ARG;
#undef VITS_GATE_BWD
  return count_ok(vits_launch_status(), VITS_CNT_GATE_16);
}

extern "C" int vits_gate_backward_io16_multi(const vits_gate_bwd_job* jobs, int n, int batch,
                                             int t_len, int wdtype, void* stream) {
  VITS_CHECK_ARG(jobs && n > 0 && n <= GATE_JOBS && batch > 0 && t_len > 0);
  VITS_CHECK_SHAPE(batch <= 65535);
  GateJobs J;
  J.n = n;
  int hmax = 0;
  bool v4 = (t_len & 3) == 0;
  for (int i = 0; i < n; ++i) {
    const vits_gate_bwd_job& q = jobs[i];
    VITS_CHECK_ARG(q.dy && q.x && q.dx && q.half_channels > 0);
    if (q.dg) VITS_CHECK_ARG(q.dg_bstride >= 2 * (int64_t)q.half_channels);
    J.j[i] = q;
    hmax = q.half_channels > hmax ? q.half_channels : hmax;
    v4 = v4 && ((q.dy_bstride | q.dy_cstride | q.x_bstride | q.x_cstride | q.dx_bstride |
                 q.dx_cstride | (int64_t)q.half_channels) & 3) == 0 &&
         ((reinterpret_cast<uintptr_t>(q.dy) | reinterpret_cast<uintptr_t>(q.x) |
           reinterpret_cast<uintptr_t>(q.dx)) & 7) == 0;
  }
  const dim3 grid(hmax, batch, n);
  hipStream_t s = as_stream(stream);
#define VITS_GATE_BWDM(E)                                                                          \
  if (v4)                                                                                          \
    hipLaunchKernelGGL((gate_bwd_multi_kernel<E, true>), grid, dim3(256), 0, s, J, t_len);        \
  else                                                                                             \
    hipLaunchKernelGGL((gate_bwd_multi_kernel<E, false>), grid, dim3(256), 0, s, J, t_len)
  if (wdtype == VITS_WDT_F16)
    VITS_GATE_BWDM(_Float16);
  else if (wdtype == VITS_WDT_BF16)
    VITS_GATE_BWDM(__bf16);
  else
    return VITS_E_ARG;
#undef VITS_GATE_BWDM
  return count_ok(vits_launch_status(), VITS_CNT_GATE_16);
}
