// layernorm.hip — channel LayerNorm on [B][C][T] (normalise over C per t).
//
// Replaces modules.LayerNorm (modules.py:41-44: transpose -> F.layer_norm
// over C, eps 1e-5 -> transpose) and, with the residual operand, the
// post-LN blocks x = LN(x + y) of attentions.Encoder (attentions.py:39-45,
// 50-53).  Workgroup = (utterance, 64 frames); each of the 4 waves sums a
// quarter of the channels for the 64 frames (lane = frame, so every load is
// a coalesced 256-byte row segment), partials meet in LDS.  Two-pass
// mean / biased variance in fp32 as F.layer_norm computes them.
#include "common.h"

namespace {

__global__ __launch_bounds__(256) void ln_channels_kernel(const float* x,
                                                          const float* r,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ beta,
                                                          float* y, int C, int T,
                                                          float eps,
                                                          const int32_t* __restrict__ lengths,
                                                          const float* __restrict__ post_add,
                                                          int64_t post_add_bstride, float scale,
                                                          const float* __restrict__ pos,
                                                          const float* __restrict__ pos_alpha) {
  __shared__ float part[4][64];
  __shared__ float stat[2][64];
  const int b = blockIdx.y;
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int t = blockIdx.x * 64 + lane;
  const bool valid = t < T;
  const int64_t base = (int64_t)b * C * T;
  const int c_per = (C + 3) / 4;
  const int c0 = wid * c_per;
  const int c1 = min(C, c0 + c_per);

  float s = 0.f;
  if (valid)
    for (int c = c0; c < c1; ++c) {
      const int64_t o = base + (int64_t)c * T + t;
      s += r ? x[o] + r[o] : x[o];
    }
  part[wid][lane] = s;
  __syncthreads();
  if (wid == 0) stat[0][lane] = (part[0][lane] + part[1][lane] + part[2][lane] + part[3][lane]) / (float)C;
  __syncthreads();
  const float mean = stat[0][lane];
  float v = 0.f;
  if (valid)
    for (int c = c0; c < c1; ++c) {
      const int64_t o = base + (int64_t)c * T + t;
      const float d = (r ? x[o] + r[o] : x[o]) - mean;
      v += d * d;
    }
  part[wid][lane] = v;
  __syncthreads();
  if (wid == 0) {
    const float var = (part[0][lane] + part[1][lane] + part[2][lane] + part[3][lane]) / (float)C;
    stat[1][lane] = 1.0f / sqrtf(var + eps);
  }
  __syncthreads();
  const float rstd = stat[1][lane];
  if (!valid) return;
  const bool zero = lengths && t >= lengths[b];
  const float* pa = post_add ? post_add + (int64_t)b * post_add_bstride : nullptr;
  const float alpha = pos ? *pos_alpha : 0.f;
  for (int c = c0; c < c1; ++c) {
    const int64_t o = base + (int64_t)c * T + t;
    const float xv = r ? x[o] + r[o] : x[o];
    float out = (xv - mean) * rstd;
    if (gamma) out = out * gamma[c];
    if (beta) out = out + beta[c];
    if (pa) out = out + pa[c];
    if (scale != 1.0f) out = out * scale;
    if (pos) out = out + pos[(int64_t)t * C + c] * alpha;
    y[o] = zero ? 0.f : out;
  }
}

// Backward of y = LN(x) * gamma + beta over C (the training step's
// modules.LayerNorm, modules.py:41-44; autocast runs it in fp32).  Same
// workgroup shape as the forward; mean / rstd are recomputed (two passes
// over the tile), then per frame  a = sum_c g dy,  q = sum_c g dy xhat,
//   dx = rstd (g dy - a / C - xhat q / C),
// and the tile's partial dgamma = sum_t dy xhat, dbeta = sum_t dy per
// channel (one wave reduction per channel) go to row (b, tile) of the
// [batch * tiles][C] partial buffers, summed by the caller.
__global__ __launch_bounds__(256) void ln_channels_bwd_kernel(
    const float* __restrict__ x, const float* __restrict__ gamma, const float* __restrict__ dy,
    float* __restrict__ dx, float* __restrict__ dgp, float* __restrict__ dbp, int C, int T,
    float eps) {
  __shared__ float part[4][64];
  __shared__ float part2[4][64];
  __shared__ float stat[4][64];
  const int b = blockIdx.y;
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int t = blockIdx.x * 64 + lane;
  const bool valid = t < T;
  const int64_t base = (int64_t)b * C * T;
  const int c_per = (C + 3) / 4;
  const int c0 = wid * c_per;
  const int c1 = min(C, c0 + c_per);
  float s = 0.f;
  if (valid)
    for (int c = c0; c < c1; ++c) s += x[base + (int64_t)c * T + t];
  part[wid][lane] = s;
  __syncthreads();
  if (wid == 0)
    stat[0][lane] = (part[0][lane] + part[1][lane] + part[2][lane] + part[3][lane]) / (float)C;
  __syncthreads();
  const float mean = stat[0][lane];
  float v = 0.f;
  if (valid)
    for (int c = c0; c < c1; ++c) {
      const float d = x[base + (int64_t)c * T + t] - mean;
      v += d * d;
    }
  part[wid][lane] = v;
  __syncthreads();
  if (wid == 0) {
    const float var = (part[0][lane] + part[1][lane] + part[2][lane] + part[3][lane]) / (float)C;
    stat[1][lane] = 1.0f / sqrtf(var + eps);
  }
  __syncthreads();
  const float rstd = stat[1][lane];
  float a = 0.f, q = 0.f;
  if (valid)
    for (int c = c0; c < c1; ++c) {
      const int64_t o = base + (int64_t)c * T + t;
      const float gd = (gamma ? gamma[c] : 1.f) * dy[o];
      a += gd;
      q += gd * (x[o] - mean) * rstd;
    }
  part[wid][lane] = a;
  part2[wid][lane] = q;
  __syncthreads();
  if (wid == 0) {
    stat[2][lane] = (part[0][lane] + part[1][lane] + part[2][lane] + part[3][lane]) / (float)C;
    stat[3][lane] = (part2[0][lane] + part2[1][lane] + part2[2][lane] + part2[3][lane]) / (float)C;
  }
  __syncthreads();
  const float am = stat[2][lane], qm = stat[3][lane];
  const int64_t prow = ((int64_t)b * gridDim.x + blockIdx.x) * C;
  for (int c = c0; c < c1; ++c) {
    const int64_t o = base + (int64_t)c * T + t;
    float gsum = 0.f, bsum = 0.f;
    if (valid) {
      const float d = dy[o];
      const float xh = (x[o] - mean) * rstd;
      dx[o] = rstd * ((gamma ? gamma[c] : 1.f) * d - am - xh * qm);
      gsum = d * xh;
      bsum = d;
    }
    gsum = wave_sum(gsum);
    bsum = wave_sum(bsum);
    if (lane == 0) {
      if (dgp) dgp[prow + c] = gsum;
      if (dbp) dbp[prow + c] = bsum;
    }
  }
}

}  // namespace

extern "C" int vits_layer_norm_channels_backward(const float* x, const float* gamma,
                                                 const float* dy, float* dx, float* dgamma_part,
                                                 float* dbeta_part, int batch, int channels,
                                                 int t_len, float eps, void* stream) {
  VITS_CHECK_ARG(x && dy && dx && batch > 0 && channels > 0 && t_len > 0);
  dim3 grid((t_len + 63) / 64, batch);
  hipLaunchKernelGGL(ln_channels_bwd_kernel, grid, dim3(256), 0, as_stream(stream), x, gamma, dy,
                     dx, dgamma_part, dbeta_part, channels, t_len, eps);
  return vits_launch_status();
}

extern "C" int vits_layer_norm_channels(const float* x, const float* r, const float* gamma,
                                        const float* beta, float* y, int batch, int channels,
                                        int t_len, float eps, const int32_t* lengths,
                                        const float* post_add, int64_t post_add_bstride,
                                        float scale, const float* pos, const float* pos_alpha,
                                        void* stream) {
  VITS_CHECK_ARG(x && y && batch > 0 && channels > 0 && t_len > 0);
  VITS_CHECK_ARG(!pos || pos_alpha);
  dim3 grid((t_len + 63) / 64, batch);
  hipLaunchKernelGGL(ln_channels_kernel, grid, dim3(256), 0, as_stream(stream), x, r, gamma, beta,
                     y, channels, t_len, eps, lengths, post_add, post_add_bstride, scale, pos,
                     pos_alpha);
  return vits_launch_status();
}
