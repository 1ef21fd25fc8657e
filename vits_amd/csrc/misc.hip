// misc.hip — small per-utterance / elementwise kernels around the conv stacks.
//
//   vits_linear_forward   per-utterance conditioning GEMV (all cond Linears
//                         of one forward stacked into one weight matrix):
//                         modules.py:109-110,139 (WN.cond_layer),
//                         modules.py:243-245,253 (ResBlock2.conds),
//                         attentions.py:143,152 (FFN2.cond),
//                         models.py:37-38,49-52 (DurationPredictor.cond1/2)
//   vits_expand_prior     attn-weighted prior expansion + reparameterised
//                         noise, models.py:569-571 (infer_p2)
//   vits_expand_durations durations -> lengths + expanded prior on the device
//                         (models.py:544-553, commons.py:143-155), the
//                         host sync of infer() removed
//   vits_conv_post_tanh   Generator tail, models.py:315-317
#include "common.h"

namespace {

// ---------------------------------------------------------------------------
// GEMV: one wave per output row n; the row of W (n_in floats) is read once
// with 16-byte loads and reused for every utterance in the batch.  g rows are
// L2-resident (batch x n_in floats).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void linear_rows_kernel(const float* __restrict__ g,
                                                          int64_t g_bstride,
                                                          const float* __restrict__ w,
                                                          const float* __restrict__ bias,
                                                          float* __restrict__ y, int64_t y_bstride,
                                                          int batch, int n_out, int n_in) {
  const int lane = threadIdx.x & 63;
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (n >= n_out) return;
  const float* wr = w + (int64_t)n * n_in;
  const float bv = bias ? bias[n] : 0.f;
  for (int b = 0; b < batch; ++b) {
    const float* gr = g + (int64_t)b * g_bstride;
    float s = 0.f;
    if ((n_in & 3) == 0) {
      for (int i = lane * 4; i < n_in; i += 256) {
        const float4 wv = *reinterpret_cast<const float4*>(wr + i);
        const float4 gv = *reinterpret_cast<const float4*>(gr + i);
        s += wv.x * gv.x + wv.y * gv.y + wv.z * gv.z + wv.w * gv.w;
      }
    } else {
      for (int i = lane; i < n_in; i += 64) s += wr[i] * gr[i];
    }
    s = wave_sum(s);
    if (lane == 0) y[(int64_t)b * y_bstride + n] = s + bv;
  }
}

// ---------------------------------------------------------------------------
// prior expansion.  Workgroup = (utterance b, 64 frames).  Each wave owns 16
// frames; for a frame it ballots the non-zero attention weights over t_x
// (one-hot in practice, but any weights are summed in x order, matching a
// sequential dot product) and accumulates m and s rows for all channels into
// an LDS tile that is then written out with the frame index contiguous.
// ---------------------------------------------------------------------------
constexpr int EP_T = 64;

__global__ __launch_bounds__(256) void expand_prior_kernel(const float* __restrict__ attn,
                                                           const float* __restrict__ m,
                                                           const float* __restrict__ s,
                                                           const float* __restrict__ noise,
                                                           float* __restrict__ z, int channels,
                                                           int t_y, int t_x, int exp_s,
                                                           float noise_scale) {
  extern __shared__ float tile[];  // [2][channels][EP_T+1]
  float* tm = tile;
  float* ts = tile + channels * (EP_T + 1);
  const int b = blockIdx.y;
  const int t0 = blockIdx.x * EP_T;
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const float* ab = attn + (int64_t)b * t_y * t_x;
  const float* mb = m + (int64_t)b * channels * t_x;
  const float* sb = s + (int64_t)b * channels * t_x;

  for (int tl = wid; tl < EP_T; tl += 4) {
    const int t = t0 + tl;
    // per-lane channel accumulators (channels <= 64*CPL)
    float am[4] = {0.f, 0.f, 0.f, 0.f};
    float as_[4] = {0.f, 0.f, 0.f, 0.f};
    if (t < t_y) {
      const float* ar = ab + (int64_t)t * t_x;
      for (int x0 = 0; x0 < t_x; x0 += 64) {
        const int x = x0 + lane;
        const float av = x < t_x ? ar[x] : 0.f;
        unsigned long long nz = __ballot(av != 0.f);
        while (nz) {
          const int bit = __ffsll((long long)nz) - 1;
          nz &= nz - 1;
          const float a = __shfl(av, bit, 64);
          const int xx = x0 + bit;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int c = lane + 64 * q;
            if (c < channels) {
              am[q] += a * mb[(int64_t)c * t_x + xx];
              as_[q] += a * sb[(int64_t)c * t_x + xx];
            }
          }
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = lane + 64 * q;
      if (c < channels) {
        tm[c * (EP_T + 1) + tl] = am[q];
        ts[c * (EP_T + 1) + tl] = as_[q];
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < channels * EP_T; i += 256) {
    const int c = i / EP_T;
    const int tl = i - c * EP_T;
    const int t = t0 + tl;
    if (t < t_y) {
      const int64_t o = ((int64_t)b * channels + c) * t_y + t;
      const float sv = ts[c * (EP_T + 1) + tl];
      z[o] = exp_s ? tm[c * (EP_T + 1) + tl] + noise[o] * expf(sv) * noise_scale
                   : tm[c * (EP_T + 1) + tl] + noise[o] * sv;
    }
  }
}

// ---------------------------------------------------------------------------
// durations -> lengths + expanded prior on the device (no host sync).
// models.py:544-553 / infer.py:169-176 / commons.py:143-155 compute
//   w = exp(logw) * rate; w_ceil = ceil(w); y_len = max(sum(w_ceil), 1)
//   (.item(): the host sync), path = infer_path(w_ceil), z = path-expanded
//   m + noise * path-expanded s (* noise_scale)
// here every frame of a static bucket t_y finds its token by binary search
// in the cumulative durations (frame t belongs to token x iff cum[x-1] <= t
// < cum[x], the one-hot of infer_path) and frames t >= y_len are zero; the
// per-stage lengths y_len * mult[i] (the masks of the flow / decoder convs)
// go to lens[i][b].  Workgroup = (64 frames, utterance); every workgroup
// rescans its utterance's durations (t_x <= 4096) in LDS.
// ---------------------------------------------------------------------------
constexpr int ED_T = 64;
constexpr int ED_MAX_TX = 4096;
constexpr int ED_MAX_STAGES = 8;
constexpr int ED_DRAWS = VITS_ED_DRAWS;  // raw generator words per utterance (mode 1)
struct EdStages {
  int32_t mult[ED_MAX_STAGES];
  int n;
};

__global__ __launch_bounds__(256) void expand_durations_kernel(
    const float* __restrict__ logw, int64_t logw_bstride, const int32_t* __restrict__ x_len,
    int t_x, float rate, int half_round, const float* __restrict__ m, const float* __restrict__ s,
    int64_t ms_bstride, int ms_cstride, const float* __restrict__ noise, int noise_mode,
    const int32_t* __restrict__ noise_start, int64_t noise_len, float noise_scale,
    float* __restrict__ z, int channels, int t_y, int batch, int32_t* __restrict__ lens,
    const EdStages st) {
  __shared__ int cum[ED_MAX_TX];
  __shared__ int part[256];
  __shared__ int xi[ED_T];
  const int b = blockIdx.y;
  const int tid = threadIdx.x;
  const int nx = x_len ? min(x_len[b], t_x) : t_x;
  // 1) integer durations of this thread's consecutive tokens, block scan
  const int per = (t_x + 255) / 256;
  const int xb0 = tid * per;
  int local = 0;
  for (int i = 0; i < per; ++i) {
    const int x = xb0 + i;
    if (x < t_x) {
      int d = 0;
      if (x < nx) {
        float w = expf(logw[(int64_t)b * logw_bstride + x]);
        if (half_round) w = (float)(_Float16)w;  // the fp16 model's torch.exp
        w = w * rate;
        if (half_round) w = (float)(_Float16)w;
        d = (int)ceilf(w);
      }
      local += d;
      cum[x] = local;  // inclusive within the thread for now
    }
  }
  part[tid] = local;
  __syncthreads();
  for (int o = 1; o < 256; o <<= 1) {
    const int v = tid >= o ? part[tid - o] : 0;
    __syncthreads();
    part[tid] += v;
    __syncthreads();
  }
  const int base = tid > 0 ? part[tid - 1] : 0;
  for (int i = 0; i < per; ++i) {
    const int x = xb0 + i;
    if (x < t_x) cum[x] += base;
  }
  __syncthreads();
  // y_len = clamp_min(sum(w_ceil), 1): the half model sums in fp16 (its
  // torch.sum result rounds to half: totals > 2048 frames round to even)
  int y_len = part[255];
  if (half_round) y_len = (int)(float)(_Float16)(float)y_len;
  y_len = max(y_len, 1);
  const int total = part[255];
  if (blockIdx.x == 0 && tid < st.n) lens[tid * batch + b] = y_len * st.mult[tid];
  // 2) token of each frame of this workgroup: first x with cum[x] > t
  const int t0 = blockIdx.x * ED_T;
  if (tid < ED_T) {
    const int t = t0 + tid;
    int r = -1;
    if (t < y_len && t < t_y && t < total) {  // (frames past the durations: no token)
      int lo = 0, hi = t_x - 1;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (cum[mid] > t) hi = mid; else lo = mid + 1;
      }
      r = lo;
    }
    xi[tid] = r;
  }
  __syncthreads();
  // 3) z[b][c][t] = m[c][x] + (noise(c, t) * s[c][x]) * noise_scale, 0 past y_len
  const float* mb = m + (int64_t)b * ms_bstride;
  const float* sb = s + (int64_t)b * ms_bstride;
  // mode 1: the slice start of infer.py:173, np.random.randint(noise_len -
  // C*y_len), drawn here where y_len is known, exactly as numpy's legacy
  // RandomState draws it: rng = high - 1; rng == 0 -> 0 without a draw;
  // else the first raw MT19937 word u of the pool with (u & mask) <= rng,
  // mask = the smallest 2^k - 1 >= rng (numpy's masked rejection for ranges
  // below 2^32).  The number of words consumed goes to lens[n_stage][b] so
  // the host re-advances its generator by exactly that many; -1 when the
  // slice does not fit (the reference's randint raises), -2 when every word
  // of the pool was rejected (probability < 2^-32: the host advances by the
  // whole pool and replays with the next words): z is then all zeros and no
  // noise element is read.
  int64_t nbase = 0;
  bool noise_ok = true;
  if (noise_mode) {
    const int64_t high = noise_len - (int64_t)channels * y_len;
    int used = -1;
    if (high >= 1 && high - 1 <= 0xFFFFFFFFll) {
      const uint32_t rng = (uint32_t)(high - 1);
      if (rng == 0) {
        used = 0;
      } else {
        used = -2;  // (until a word is accepted)
        uint32_t mask = rng;
        mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4;
        mask |= mask >> 8; mask |= mask >> 16;
        const uint32_t* pool = reinterpret_cast<const uint32_t*>(noise_start) +
                               (int64_t)b * ED_DRAWS;
        for (int i = 0; i < ED_DRAWS; ++i) {
          const uint32_t u = pool[i] & mask;
          if (u <= rng) {
            nbase = u;
            used = i + 1;
            break;
          }
        }
      }
    }
    noise_ok = used >= 0;
    if (blockIdx.x == 0 && tid == 0) lens[st.n * batch + b] = used;
  }
  for (int i = tid; i < channels * ED_T; i += 256) {
    const int c = i / ED_T;
    const int tl = i - c * ED_T;
    const int t = t0 + tl;
    if (t >= t_y) continue;
    const int x = xi[tl];
    float v = 0.f;
    if (x >= 0 && noise_ok) {
      // mode 0: noise [B][C][t_y]; mode 1: EmoVITS's buffer slice viewed as
      // [C][y_len] from element noise_start[b] (infer.py:172-175)
      const float n = noise_mode ? noise[nbase + (int64_t)c * y_len + t]
                                 : noise[((int64_t)b * channels + c) * t_y + t];
      v = mb[(int64_t)c * ms_cstride + x] + (n * sb[(int64_t)c * ms_cstride + x]) * noise_scale;
    }
    z[((int64_t)b * channels + c) * t_y + t] = v;
  }
}

// ---------------------------------------------------------------------------
// Generator tail: one thread per output sample; the input window of the
// workgroup ([channels][256 + k - 1]) is staged in LDS with the 0.01 leaky
// relu applied once per element.
// ---------------------------------------------------------------------------
constexpr int CP_T = 256;

// XT: the activation type of the last stage (float; __bf16 / _Float16 when
// the 16-bit model keeps its decoder activations 16-bit, engine.py ACT16)
template <typename XT>
__global__ __launch_bounds__(256) void conv_post_tanh_kernel(const XT* __restrict__ x,
                                                             int64_t x_bstride, int x_cstride,
                                                             const float* __restrict__ w,
                                                             float* __restrict__ y, int channels,
                                                             int t_len, int ksize) {
  extern __shared__ float sm[];  // [channels][CP_T + ksize - 1] then w
  const int W = CP_T + ksize - 1;
  float* xs = sm;
  float* wsm = sm + channels * W;
  const int b = blockIdx.y;
  const int t0 = blockIdx.x * CP_T;
  const int pad = (ksize - 1) / 2;
  const XT* xb = x + (int64_t)b * x_bstride;
  for (int i = threadIdx.x; i < channels * ksize; i += 256) wsm[i] = w[i];
  // 8 channels x 2 window columns per thread in flight at once (a load-use
  // chain per element serialised ~2 x channels global latencies: 240 us for
  // the B=16 decoder tail)
  constexpr int CG = 8;
  for (int c0 = 0; c0 < channels; c0 += CG) {
    float v[CG][2];
#pragma unroll
    for (int cc = 0; cc < CG; ++cc)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int t = threadIdx.x + 256 * h;
        const int tt = t0 - pad + t;
        const bool ok = c0 + cc < channels && t < W && tt >= 0 && tt < t_len;
        v[cc][h] = ok ? (float)xb[(int64_t)(c0 + cc) * x_cstride + tt] : 0.f;
      }
#pragma unroll
    for (int cc = 0; cc < CG; ++cc)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int t = threadIdx.x + 256 * h;
        if (c0 + cc < channels && t < W) {
          const float u = v[cc][h];
          xs[(c0 + cc) * W + t] = u < 0.f ? 0.01f * u : u;
        }
      }
  }
  __syncthreads();
  const int tl = threadIdx.x;
  const int t = t0 + tl;
  if (t >= t_len) return;
  float acc = 0.f;
  for (int c = 0; c < channels; ++c) {
    const float* xr = xs + c * W + tl;
    const float* wr = wsm + c * ksize;
    for (int j = 0; j < ksize; ++j) acc += wr[j] * xr[j];
  }
  y[(int64_t)b * t_len + t] = tanhf(acc);
}

// Aligned form (T % 4 == 0, 4-element-aligned rows, ksize <= 9): every
// thread issues all its 4-step block loads of the CPC-channel window at once
// (16 bytes fp32 / 8 bytes 16-bit per load) before the first is used - the
// grouped form above waits ~channels / 8 load round trips per workgroup (122
// us for the B=16 decoder tail, ~1.6 TB/s).  Window columns [t0 - 4, t0 +
// CP_T + 4): tap j of output t reads column t - t0 + 1 + j.
template <typename XT, int CPC>
__global__ __launch_bounds__(256) void conv_post_tanh_v4_kernel(const XT* __restrict__ x,
                                                                int64_t x_bstride, int x_cstride,
                                                                const float* __restrict__ w,
                                                                float* __restrict__ y, int t_len,
                                                                int ksize) {
  constexpr int W = CP_T + 8;         // window columns
  constexpr int NB = W / 4;           // 4-step blocks per channel row
  constexpr int NU = (CPC * NB + 255) / 256;
  typedef XT x4 __attribute__((ext_vector_type(4)));
  __shared__ float xs[CPC * W];
  __shared__ float wsm[CPC * 9];
  const int b = blockIdx.y;
  const int t0 = blockIdx.x * CP_T;
  const XT* xb = x + (int64_t)b * x_bstride;
  for (int i = threadIdx.x; i < CPC * ksize; i += 256) wsm[i] = w[i];
  x4 v[NU];
  bool ok[NU];
#pragma unroll
  for (int q = 0; q < NU; ++q) {
    const int u = threadIdx.x + 256 * q;
    const int c = u / NB;
    const int tt = t0 - 4 + 4 * (u - c * NB);
    ok[q] = u < CPC * NB && tt >= 0 && tt < t_len;  // a block is all in or all out
    v[q] = *reinterpret_cast<const x4*>(ok[q] ? xb + (int64_t)c * x_cstride + tt : xb);
  }
#pragma unroll
  for (int q = 0; q < NU; ++q) {
    const int u = threadIdx.x + 256 * q;
    if (u < CPC * NB) {
      const int c = u / NB;
      float4 f;
      float* fe = reinterpret_cast<float*>(&f);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float a = ok[q] ? (float)v[q][e] : 0.f;
        fe[e] = a < 0.f ? 0.01f * a : a;
      }
      *reinterpret_cast<float4*>(xs + c * W + 4 * (u - c * NB)) = f;
    }
  }
  __syncthreads();
  const int tl = threadIdx.x;
  const int t = t0 + tl;
  if (t >= t_len) return;
  const int off = 4 - (ksize - 1) / 2;  // window column of tap 0
  float acc = 0.f;
  for (int c = 0; c < CPC; ++c) {
    const float* xr = xs + c * W + tl + off;
    const float* wr = wsm + c * ksize;
    for (int j = 0; j < ksize; ++j) acc += wr[j] * xr[j];
  }
  y[(int64_t)b * t_len + t] = tanhf(acc);
}

}  // namespace

extern "C" int vits_linear_forward(const float* g, int64_t g_bstride, const float* w,
                                   const float* bias, float* y, int64_t y_bstride, int batch,
                                   int n_out, int n_in, void* stream) {
  VITS_CHECK_ARG(g && w && y && batch > 0 && n_out > 0 && n_in > 0);
  if ((n_in & 3) == 0)
    VITS_CHECK_SHAPE(((reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(g)) & 15) == 0 &&
                     (g_bstride & 3) == 0);
  dim3 grid((n_out + 3) / 4);
  hipLaunchKernelGGL(linear_rows_kernel, grid, dim3(256), 0, as_stream(stream), g, g_bstride, w,
                     bias, y, y_bstride, batch, n_out, n_in);
  return vits_launch_status();
}

extern "C" int vits_expand_prior(const float* attn, const float* m, const float* s,
                                 const float* noise, float* z, int batch, int channels, int t_y,
                                 int t_x, int exp_s, float noise_scale, void* stream) {
  VITS_CHECK_ARG(attn && m && s && noise && z && batch > 0 && channels > 0 && t_y > 0 && t_x > 0);
  VITS_CHECK_SHAPE(channels <= 256);
  const size_t lds = sizeof(float) * 2 * channels * (EP_T + 1);
  dim3 grid((t_y + EP_T - 1) / EP_T, batch);
  hipLaunchKernelGGL(expand_prior_kernel, grid, dim3(256), lds, as_stream(stream), attn, m, s,
                     noise, z, channels, t_y, t_x, exp_s, noise_scale);
  return vits_launch_status();
}

extern "C" int vits_expand_durations(const float* logw, int64_t logw_bstride,
                                     const int32_t* x_len, int t_x, float rate, int half_round,
                                     const float* m, const float* s, int64_t ms_bstride,
                                     int32_t ms_cstride, const float* noise, int noise_mode,
                                     const int32_t* noise_start, int64_t noise_len,
                                     float noise_scale, float* z,
                                     int batch, int channels, int t_y, int32_t* lens,
                                     const int32_t* stage_mult, int n_stage, void* stream) {
  VITS_CHECK_ARG(logw && m && s && noise && z && lens && batch > 0 && channels > 0 && t_y > 0 &&
                 t_x > 0);
  VITS_CHECK_ARG(n_stage >= 1 && n_stage <= ED_MAX_STAGES && (n_stage == 1 || stage_mult));
  VITS_CHECK_SHAPE(t_x <= ED_MAX_TX && ms_cstride >= t_x);
  VITS_CHECK_ARG(noise_mode == 0 || (noise_mode == 1 && noise_start));
  EdStages st;
  st.n = n_stage;
  for (int i = 0; i < ED_MAX_STAGES; ++i) st.mult[i] = i < n_stage ? (stage_mult ? stage_mult[i] : 1) : 0;
  dim3 grid((t_y + ED_T - 1) / ED_T, batch);
  hipLaunchKernelGGL(expand_durations_kernel, grid, dim3(256), 0, as_stream(stream), logw,
                     logw_bstride, x_len, t_x, rate, half_round, m, s, ms_bstride, ms_cstride,
                     noise, noise_mode, noise_start, noise_len, noise_scale, z, channels, t_y,
                     batch, lens, st);
  return vits_launch_status();
}

extern "C" int vits_conv_post_tanh(const float* x, int64_t x_bstride, int32_t x_cstride,
                                   const float* w, float* y, int batch, int channels, int t_len,
                                   int ksize, void* stream) {
  return vits_conv_post_tanh_lowp(x, x_bstride, x_cstride, w, y, batch, channels, t_len, ksize,
                                  VITS_WDT_F32, stream);
}

extern "C" int vits_conv_post_tanh_lowp(const void* x, int64_t x_bstride, int32_t x_cstride,
                                        const float* w, float* y, int batch, int channels,
                                        int t_len, int ksize, int xdtype, void* stream) {
  VITS_CHECK_ARG(x && w && y && batch > 0 && channels > 0 && t_len > 0 && ksize > 0);
  VITS_CHECK_ARG(xdtype == VITS_WDT_F32 || xdtype == VITS_WDT_BF16 || xdtype == VITS_WDT_F16);
  VITS_CHECK_SHAPE((ksize & 1) == 1 && ksize <= 257 && x_cstride >= t_len);
  const size_t lds = sizeof(float) * ((size_t)channels * (CP_T + ksize - 1) + channels * ksize);
  VITS_CHECK_SHAPE(lds <= 64 * 1024);
  dim3 grid((t_len + CP_T - 1) / CP_T, batch);
  hipStream_t s = as_stream(stream);
  const int esz = xdtype == VITS_WDT_F32 ? 4 : 2;
  if (channels == 32 && ksize <= 9 && (t_len & 3) == 0 && (x_cstride & 3) == 0 &&
      (x_bstride & 3) == 0 && (reinterpret_cast<uintptr_t>(x) & (4 * esz - 1)) == 0) {
    // the decoder tail (upsample_initial_channel / 2^4 = 32 channels, k = 7)
    if (xdtype == VITS_WDT_BF16)
      hipLaunchKernelGGL((conv_post_tanh_v4_kernel<__bf16, 32>), grid, dim3(256), 0, s,
                         static_cast<const __bf16*>(x), x_bstride, x_cstride, w, y, t_len, ksize);
    else if (xdtype == VITS_WDT_F16)
      hipLaunchKernelGGL((conv_post_tanh_v4_kernel<_Float16, 32>), grid, dim3(256), 0, s,
                         static_cast<const _Float16*>(x), x_bstride, x_cstride, w, y, t_len,
                         ksize);
    else
      hipLaunchKernelGGL((conv_post_tanh_v4_kernel<float, 32>), grid, dim3(256), 0, s,
                         static_cast<const float*>(x), x_bstride, x_cstride, w, y, t_len, ksize);
    return vits_launch_status();
  }
  if (xdtype == VITS_WDT_BF16)
    hipLaunchKernelGGL(conv_post_tanh_kernel<__bf16>, grid, dim3(256), lds, s,
                       static_cast<const __bf16*>(x), x_bstride, x_cstride, w, y, channels, t_len,
                       ksize);
  else if (xdtype == VITS_WDT_F16)
    hipLaunchKernelGGL(conv_post_tanh_kernel<_Float16>, grid, dim3(256), lds, s,
                       static_cast<const _Float16*>(x), x_bstride, x_cstride, w, y, channels,
                       t_len, ksize);
  else
    hipLaunchKernelGGL(conv_post_tanh_kernel<float>, grid, dim3(256), lds, s,
                       static_cast<const float*>(x), x_bstride, x_cstride, w, y, channels, t_len,
                       ksize);
  return vits_launch_status();
}
