// negcent.hip — the alignment score matrix of SynthesizerTrn.forward
// (models.py:483-490) on gfx950 fp32 MFMA, one kernel instead of the
// reference's exp / 2 matmuls / 2 reductions / 3 adds:
//
//   s = exp(-2 logs_p)                                  [B][C][t_s]
//   neg_cent[b][y][x] = sum_d ( -0.5 log(2 pi) - logs_p[d][x]
//                               - 0.5 z_p[d][y]^2 s[d][x]
//                               + z_p[d][y] m_p[d][x] s[d][x]
//                               - 0.5 m_p[d][x]^2 s[d][x] )
//
// GEMM view per utterance: rows y (t_t, mel frames), columns x (t_s, text
// tokens), K = 2C: A = [-0.5 z^2 | z] (read from z_p [C][t_t], y contiguous),
// B = [s | m s] (computed on the fly from m_p / logs_p [C][t_s]).  The
// per-column constant sum_d(-0.5 log 2pi - logs - 0.5 m^2 s) is reduced by
// the same wave.  One wave = one 32x32 output tile; lane l holds column
// x0 + (l & 31), so every load and the store are 128-byte coalesced.
#include "common.h"

namespace {

__global__ __launch_bounds__(64) void neg_cent_kernel(const float* __restrict__ z,
                                                      const float* __restrict__ m,
                                                      const float* __restrict__ logs,
                                                      float* __restrict__ out, int C, int Tt,
                                                      int Ts) {
  const int lane = threadIdx.x;
  const int l32 = lane & 31;
  const int lhi = lane >> 5;
  const int x0 = blockIdx.x * 32;
  const int y0 = blockIdx.y * 32;
  const int b = blockIdx.z;
  const float* zb = z + (int64_t)b * C * Tt;
  const float* mb = m + (int64_t)b * C * Ts;
  const float* lb = logs + (int64_t)b * C * Ts;
  const int x = x0 + l32;
  const int y = y0 + l32;
  const bool xv = x < Ts;
  const bool yv = y < Tt;
  constexpr float kHalfLog2Pi = 0.918938533204672742f;  // 0.5 * log(2 pi)

  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  float colc = 0.f;  // this lane's half of the per-column constant
  for (int d0 = 0; d0 < C; d0 += 2) {
    const int d = d0 + lhi;
    float zv = 0.f, sv = 0.f, msv = 0.f;
    if (d < C) {
      if (yv) zv = zb[(int64_t)d * Tt + y];
      if (xv) {
        const float lv = lb[(int64_t)d * Ts + x];
        const float mv = mb[(int64_t)d * Ts + x];
        sv = expf(-2.0f * lv);
        msv = mv * sv;
        colc += -kHalfLog2Pi - lv - 0.5f * (mv * mv) * sv;
      }
    }
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(-0.5f * zv * zv, sv, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(zv, msv, acc, 0, 0, 0);
  }
  colc += __shfl_xor(colc, 32, 64);
  if (!xv) return;
  float* ob = out + (int64_t)b * Tt * Ts;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = y0 + (r & 3) + 8 * (r >> 2) + 4 * lhi;
    if (row < Tt) ob[(int64_t)row * Ts + x] = acc[r] + colc;
  }
}

}  // namespace

extern "C" int vits_neg_cent(const float* z_p, const float* m_p, const float* logs_p,
                             float* neg_cent, int batch, int channels, int t_t, int t_s,
                             void* stream) {
  VITS_CHECK_ARG(z_p && m_p && logs_p && neg_cent);
  VITS_CHECK_ARG(batch > 0 && channels > 0 && t_t > 0 && t_s > 0);
  dim3 grid((t_s + 31) / 32, (t_t + 31) / 32, batch);
  hipLaunchKernelGGL(neg_cent_kernel, grid, dim3(64), 0, as_stream(stream), z_p, m_p, logs_p,
                     neg_cent, channels, t_t, t_s);
  return vits_launch_status();
}
