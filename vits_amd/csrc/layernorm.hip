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

}  // namespace

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
