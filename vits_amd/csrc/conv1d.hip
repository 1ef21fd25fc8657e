// conv1d.hip — implicit-GEMM dilated 1-D convolution on gfx950 fp32 MFMA
// (v_mfma_f32_32x32x2_f32), with the elementwise tails of the VITS blocks
// fused into the prologue/epilogue.
//
// GEMM view (one utterance b):
//   Y[m][n] = sum_{c<cin, j<k} W[m][c][j] * X[c][n - pad_left + j*dil]
// rows m = output channels (gate pairs interleaved / polyphase phases
// stacked, see vits_amd/engine.py), columns n = time positions.
//
// Layout in HBM: activations stay [B][C][T] (time contiguous, as the
// reference keeps them), packed weights are [cin_pad][k][m_pad] so a
// K-chunk of `kc` input channels is one contiguous slab whose rows the
// workgroup streams with 16-byte loads.
//
// One workgroup = 4 waves = one BM x BN output tile of one utterance.  Per
// K-chunk the workgroup stages W[kc][k][BM] and the input window
// X[kc][BN + (k-1)*dil] (leaky-relu prologue applied on the way in) into
// LDS once; every tap j then reads the same X rows shifted by j*dil, so the
// input is fetched once per chunk regardless of the kernel width.
//
// Reference call sites: modules.py:136,148 (WN in/res_skip convs),
// modules.py:252,257 (ResBlock2 convs1/convs2), models.py:307,310
// (conv_pre, ups), modules.py:363,366 (coupling pre/post).
#include "common.h"

namespace {

struct OutDesc {
  float* y;
  int64_t y_bstride;
  int y_cstride;
  int act;
  const float* res;
  int64_t res_bstride;
  int res_cstride;
  float res_scale;
  int accumulate;
  float post_div;
};

__device__ __forceinline__ float apply_act(float v, int act) {
  if (act == VITS_ACT_RELU) return v > 0.f ? v : 0.f;
  if (act == VITS_ACT_TANH) return tanhf(v);
  if (act == VITS_ACT_EXP) return expf(v);
  return v;
}

__device__ __forceinline__ void store_std(const OutDesc& o, int b, int ch, int t, float v,
                                          bool masked) {
  v = apply_act(v, o.act);
  if (o.res) v = o.res[(int64_t)b * o.res_bstride + (int64_t)ch * o.res_cstride + t] + o.res_scale * v;
  float* dst = o.y + (int64_t)b * o.y_bstride + (int64_t)ch * o.y_cstride + t;
  if (o.accumulate) v = *dst + v;
  if (o.post_div != 1.0f) v = v / o.post_div;
  if (masked) v = 0.f;
  *dst = v;
}

template <int BM, int BN, int WAVES_M, int WAVES_N, int EPI>
__global__ __launch_bounds__(256) void conv1d_mfma_kernel(const vits_conv1d_desc p) {
  constexpr int WM = BM / WAVES_M;
  constexpr int WN = BN / WAVES_N;
  constexpr int TM = WM / 32;
  constexpr int TN = WN / 32;
  static_assert(WAVES_M * WAVES_N == 4, "4 waves per workgroup");
  static_assert(TM >= 1 && TN >= 1, "wave tile >= 32x32");

  extern __shared__ float smem[];
  const int kc = p.kc;
  const int k = p.k;
  const int dil = p.dil;
  const int halo = (k - 1) * dil;
  const int xw = BN + halo;
  const int xw_pad = (xw + 3) & ~3;
  float* ws = smem;                  // [kc*k][BM]
  float* xs = smem + kc * k * BM;    // [kc][xw_pad]

  const int b = blockIdx.z;
  const int n0 = blockIdx.x * BN;
  const int m0 = blockIdx.y * BM;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = (wid / WAVES_N) * WM;
  const int wn = (wid % WAVES_N) * WN;
  const int l32 = lane & 31;
  const int lhi = lane >> 5;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const float* xb = p.x + (int64_t)b * p.x_bstride;
  const int64_t xts = p.x_tstride;
  const int xstart = n0 - p.pad_left;
  const float slope = p.in_slope;
  const bool act_in = slope != 1.0f;
  const int wrows = kc * k;
  constexpr int BM4 = BM / 4;

  for (int c0 = 0; c0 < p.cin_pad; c0 += kc) {
    // ---- stage packed weights W[c0 .. c0+kc)[0..k)[m0 .. m0+BM) ----------
    const float* wsrc = p.w + (int64_t)c0 * k * p.m_pad + m0;
    for (int i = tid; i < wrows * BM4; i += 256) {
      const int r = i / BM4;
      const int q = i - r * BM4;
      const float4 v = *reinterpret_cast<const float4*>(wsrc + (int64_t)r * p.m_pad + q * 4);
      *reinterpret_cast<float4*>(ws + r * BM + q * 4) = v;
    }
    // ---- stage input window with zero padding + leaky-relu prologue ------
    for (int c = 0; c < kc; ++c) {
      const int cc = c0 + c;
      const float* xr = xb + (int64_t)cc * p.x_cstride;
      const bool crow = cc < p.cin;
      for (int t = tid; t < xw_pad; t += 256) {
        const int tt = xstart + t;
        float v = 0.f;
        if (crow && t < xw && tt >= 0 && tt < p.tin) {
          v = xr[tt * xts];
          if (act_in) v = v < 0.f ? v * slope : v;
        }
        xs[c * xw_pad + t] = v;
      }
    }
    __syncthreads();

    // ---- MFMA over (tap, channel pair) -------------------------------------
    for (int j = 0; j < k; ++j) {
      const int xoff = wn + l32 + j * dil;
      for (int c = 0; c < kc; c += 2) {
        const int cr = c + lhi;
        float a[TM], bv[TN];
#pragma unroll
        for (int mi = 0; mi < TM; ++mi) a[mi] = ws[(cr * k + j) * BM + wm + mi * 32 + l32];
#pragma unroll
        for (int ni = 0; ni < TN; ++ni) bv[ni] = xs[cr * xw_pad + xoff + ni * 32];
#pragma unroll
        for (int mi = 0; mi < TM; ++mi)
#pragma unroll
          for (int ni = 0; ni < TN; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[mi], bv[ni], acc[mi][ni], 0, 0, 0);
      }
    }
    __syncthreads();
  }

  // ---- epilogue -----------------------------------------------------------
  const int len_b = p.lengths ? p.lengths[b] : 0x7fffffff;
  const float* cond = p.cond ? p.cond + (int64_t)b * p.cond_bstride : nullptr;
  OutDesc o0{p.out0.y, p.out0.y_bstride, p.out0.y_cstride, p.out0.act, p.out0.res,
             p.out0.res_bstride, p.out0.res_cstride, p.out0.res_scale, p.out0.accumulate,
             p.out0.post_div};

#pragma unroll
  for (int mi = 0; mi < TM; ++mi) {
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) {
      const int n = n0 + wn + ni * 32 + l32;
      const int rbase = m0 + wm + mi * 32 + 4 * lhi;
      if (EPI == VITS_EPI_GATE) {
        // packed rows 2q (tanh half) / 2q+1 (sigmoid half) live in the same
        // lane in registers r, r+1 (r even): no cross-lane traffic.
        const int H = p.m >> 1;
        if (n < p.n_out) {
#pragma unroll
          for (int r = 0; r < 16; r += 2) {
            const int row = rbase + (r & 3) + 8 * (r >> 2);
            if (row < p.m) {
              const int q = row >> 1;
              float va = acc[mi][ni][r];
              float vb = acc[mi][ni][r + 1];
              if (p.bias) {
                va += p.bias[q];
                vb += p.bias[H + q];
              }
              if (cond) {
                va += cond[q];
                vb += cond[H + q];
              }
              float v = tanhf(va) * (1.0f / (1.0f + expf(-vb)));
              store_std(o0, b, q, n, v, n >= len_b);
            }
          }
        }
      } else if (EPI == VITS_EPI_UPSAMPLE) {
        const int u = p.up_u;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = rbase + (r & 3) + 8 * (r >> 2);
          if (row < p.m && n < p.n_out) {
            const int oc = row / u;
            const int ph = row - oc * u;
            const int t = n * u + ph - p.up_pad;
            if (t >= 0 && t < p.t_out) {
              float v = acc[mi][ni][r];
              if (p.bias) v += p.bias[oc];
              store_std(o0, b, oc, t, v, t >= len_b);
            }
          }
        }
      } else {
        OutDesc o1{p.out1.y, p.out1.y_bstride, p.out1.y_cstride, p.out1.act, p.out1.res,
                   p.out1.res_bstride, p.out1.res_cstride, p.out1.res_scale,
                   p.out1.accumulate, p.out1.post_div};
        if (n < p.n_out) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = rbase + (r & 3) + 8 * (r >> 2);
            if (row < p.m) {
              float v = acc[mi][ni][r];
              if (p.bias) v += p.bias[row];
              if (cond) v += cond[row];
              if (row < p.split)
                store_std(o0, b, row, n, v, n >= len_b);
              else
                store_std(o1, b, row - p.split, n, v, n >= len_b);
            }
          }
        }
      }
    }
  }
}

template <int BM, int BN, int WM_, int WN_>
int launch_tile(const vits_conv1d_desc& d, int batch, hipStream_t s) {
  const int halo = (d.k - 1) * d.dil;
  const int xw_pad = (BN + halo + 3) & ~3;
  const size_t lds = sizeof(float) * ((size_t)d.kc * d.k * BM + (size_t)d.kc * xw_pad);
  if (lds > 160 * 1024) return VITS_E_UNSUP;
  dim3 grid((d.n_out + BN - 1) / BN, (d.m + BM - 1) / BM, batch);
  dim3 block(256);
  switch (d.epi) {
    case VITS_EPI_STORE:
      hipLaunchKernelGGL((conv1d_mfma_kernel<BM, BN, WM_, WN_, VITS_EPI_STORE>), grid, block, lds, s, d);
      break;
    case VITS_EPI_GATE:
      hipLaunchKernelGGL((conv1d_mfma_kernel<BM, BN, WM_, WN_, VITS_EPI_GATE>), grid, block, lds, s, d);
      break;
    case VITS_EPI_UPSAMPLE:
      hipLaunchKernelGGL((conv1d_mfma_kernel<BM, BN, WM_, WN_, VITS_EPI_UPSAMPLE>), grid, block, lds, s, d);
      break;
    default:
      return VITS_E_UNSUP;
  }
  return vits_launch_status();
}

int check_desc(const vits_conv1d_desc& d, int batch) {
  VITS_CHECK_ARG(d.x && d.w && d.out0.y);
  VITS_CHECK_ARG(batch > 0 && d.cin > 0 && d.m > 0 && d.k > 0 && d.dil > 0 && d.n_out > 0);
  VITS_CHECK_SHAPE(d.kc >= 2 && (d.kc % 2) == 0 && d.cin_pad % d.kc == 0 && d.cin_pad >= d.cin);
  VITS_CHECK_SHAPE(d.m_pad % 128 == 0 && d.m_pad >= d.m);
  VITS_CHECK_SHAPE(d.tin >= 0 && d.x_tstride >= 1);
  VITS_CHECK_SHAPE(d.x_tstride != 1 || d.x_cstride >= d.tin);
  if (d.epi == VITS_EPI_GATE) VITS_CHECK_SHAPE((d.m % 2) == 0);
  if (d.epi == VITS_EPI_UPSAMPLE) VITS_CHECK_SHAPE(d.up_u > 0 && d.m % d.up_u == 0 && d.t_out > 0);
  if (d.epi == VITS_EPI_STORE && d.split < d.m) VITS_CHECK_ARG(d.out1.y != nullptr);
  if ((reinterpret_cast<uintptr_t>(d.w) & 15) != 0) return VITS_E_SHAPE;
  return VITS_OK;
}

int conv1d_one(const vits_conv1d_desc& d, int batch, hipStream_t s) {
  int rc = check_desc(d, batch);
  if (rc) return rc;
  switch (d.tile) {
    case VITS_TILE_128x128:
      return launch_tile<128, 128, 2, 2>(d, batch, s);
    case VITS_TILE_64x256:
      return launch_tile<64, 256, 1, 4>(d, batch, s);
    case VITS_TILE_32x256:
      return launch_tile<32, 256, 1, 4>(d, batch, s);
    default:
      return VITS_E_UNSUP;
  }
}

}  // namespace

extern "C" int vits_conv1d_forward(const vits_conv1d_desc* d, int batch, void* stream) {
  if (!d) return VITS_E_ARG;
  return conv1d_one(*d, batch, as_stream(stream));
}

extern "C" int vits_conv1d_forward_seq(const vits_conv1d_desc* d, int n, int batch, void* stream) {
  if (!d || n < 0) return VITS_E_ARG;
  for (int i = 0; i < n; ++i) {
    int rc = conv1d_one(d[i], batch, as_stream(stream));
    if (rc) return rc;
  }
  return VITS_OK;
}
