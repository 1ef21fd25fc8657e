// stft.hip — STFT magnitude (+ adjoint) as LDS radix-2 Stockham FFTs.
//
// Replaces torch.stft + sqrt(re^2+im^2+eps) of
//   TorchSTFT.stft / STFTLoss.spec2mag   (modules.py:386-392, stft_loss.py:22-23),
//   spectrogram_torch                     (mel_processing.py:58-77, pad (n_fft-hop)/2,
//                                          center=False, eps 1e-6).
// Forward: one workgroup transforms FPB frames (FPB*n_fft <= 2048 points),
// entirely in LDS: reflect-padded, windowed frame -> complex n_fft-point
// Stockham FFT (natural-order output, ping-pong buffers) -> bins 0..n_fft/2.
// Backward: d mag / d(re,im) = (re,im)/mag; the adjoint of the real DFT is
// the real part of an inverse FFT of G = g_re + i g_im over the one-sided
// bins (upper bins 0), windowed into a per-frame workspace; a second kernel
// overlap-adds the frames per sample (gather: no atomics, deterministic) and
// folds the reflect padding back onto the signal.
#include "common.h"

namespace {

constexpr int FFT_MAX = 2048;  // complex points per workgroup

__device__ __forceinline__ int reflect_idx(int i, int L) {
  // torch reflect padding (no edge repeat); valid for |pad| < L
  if (i < 0) i = -i;
  if (i >= L) i = 2 * (L - 1) - i;
  return i;
}

// Twiddle table tw[m] = (cos, sin)(2 pi m / n), m < n/2, built once per
// workgroup (n/2 sincospif instead of one per butterfly and stage).
__device__ void fill_twiddles(float2* tw, int n) {
  for (int m = threadIdx.x; m < (n >> 1); m += blockDim.x) {
    float sn, cs;
    sincospif(2.0f * (float)m / (float)n, &sn, &cs);
    tw[m] = make_float2(cs, sn);
  }
}

// Stockham radix-2 over FPB independent transforms of size n laid out
// back to back in `a`; result ends in the returned buffer.  sign = -1
// forward (e^{-i}), +1 inverse (unnormalised).  Stage s twiddle of butterfly
// kk is e^{sign i pi kk / 2^s} = tw[kk << (log2n - 1 - s)] (sin negated for
// the forward transform).
__device__ float2* fft_lds(float2* a, float2* b, const float2* tw, int n, int log2n, int fpb,
                           float sign) {
  const int half = n >> 1;
  const int total = fpb * half;
  for (int s = 0; s < log2n; ++s) {
    const int ns = 1 << s;
    const int tsh = log2n - 1 - s;
    for (int i = threadIdx.x; i < total; i += blockDim.x) {
      const int f = i / half;
      const int j = i - f * half;
      const float2* src = a + f * n;
      float2* dst = b + f * n;
      const int kk = j & (ns - 1);
      const float2 v0 = src[j];
      float2 v1 = src[j + half];
      const float2 w = tw[kk << tsh];
      const float cs = w.x;
      const float sn = sign * w.y;
      const float tr = v1.x * cs - v1.y * sn;
      const float ti = v1.x * sn + v1.y * cs;
      const int d = ((j - kk) << 1) + kk;
      dst[d] = make_float2(v0.x + tr, v0.y + ti);
      dst[d + ns] = make_float2(v0.x - tr, v0.y - ti);
    }
    __syncthreads();
    float2* t = a;
    a = b;
    b = t;
  }
  return a;
}

__global__ __launch_bounds__(256) void stft_fwd_kernel(const float* __restrict__ x, int L,
                                                       const float* __restrict__ window, int n,
                                                       int log2n, int hop, int win, int pad,
                                                       int frames, int fpb, float eps,
                                                       float* __restrict__ mag,
                                                       float* __restrict__ re,
                                                       float* __restrict__ im) {
  extern __shared__ float2 sfft[];
  float2* a = sfft;
  float2* bbuf = sfft + fpb * n;
  float2* tw = bbuf + fpb * n;
  fill_twiddles(tw, n);
  const int b = blockIdx.y;
  const int f0 = blockIdx.x * fpb;
  const int woff = (n - win) / 2;
  const float* xb = x + (int64_t)b * L;
  for (int i = threadIdx.x; i < fpb * n; i += blockDim.x) {
    const int f = i / n;
    const int t = i - f * n;
    const int fr = f0 + f;
    float v = 0.f;
    const int wi = t - woff;
    if (fr < frames && wi >= 0 && wi < win) {
      const int src = reflect_idx(fr * hop + t - pad, L);
      v = xb[src] * window[wi];
    }
    a[i] = make_float2(v, 0.f);
  }
  __syncthreads();
  const float2* out = fft_lds(a, bbuf, tw, n, log2n, fpb, -1.f);
  const int nb = n / 2 + 1;
  for (int i = threadIdx.x; i < fpb * nb; i += blockDim.x) {
    const int k = i / fpb;
    const int f = i - k * fpb;
    const int fr = f0 + f;
    if (fr >= frames) continue;
    const float2 c = out[f * n + k];
    const int64_t o = ((int64_t)b * nb + k) * frames + fr;
    mag[o] = sqrtf(c.x * c.x + c.y * c.y + eps);
    if (re) re[o] = c.x;
    if (im) im[o] = c.y;
  }
}

__global__ __launch_bounds__(256) void stft_bwd_frames_kernel(
    const float* __restrict__ gmag, const float* __restrict__ mag, const float* __restrict__ re,
    const float* __restrict__ im, const float* __restrict__ window, int n, int log2n, int win,
    int frames, int fpb, float* __restrict__ dframes) {
  extern __shared__ float2 sfft[];
  float2* a = sfft;
  float2* bbuf = sfft + fpb * n;
  float2* tw = bbuf + fpb * n;
  fill_twiddles(tw, n);
  const int b = blockIdx.y;
  const int f0 = blockIdx.x * fpb;
  const int nb = n / 2 + 1;
  const int woff = (n - win) / 2;
  for (int i = threadIdx.x; i < fpb * n; i += blockDim.x) {
    const int k = i / fpb;  // bin-major so reads along frames are contiguous
    const int f = i - k * fpb;
    const int fr = f0 + f;
    float2 g = make_float2(0.f, 0.f);
    if (k < nb && fr < frames) {
      const int64_t o = ((int64_t)b * nb + k) * frames + fr;
      const float s = gmag[o] / mag[o];
      g = make_float2(s * re[o], s * im[o]);
    }
    a[f * n + k] = g;
  }
  __syncthreads();
  const float2* out = fft_lds(a, bbuf, tw, n, log2n, fpb, +1.f);
  for (int i = threadIdx.x; i < fpb * n; i += blockDim.x) {
    const int f = i / n;
    const int t = i - f * n;
    const int fr = f0 + f;
    if (fr >= frames) continue;
    const int wi = t - woff;
    const float w = (wi >= 0 && wi < win) ? window[wi] : 0.f;
    dframes[((int64_t)b * frames + fr) * n + t] = out[f * n + t].x * w;
  }
}

// overlap-add of frame gradients per padded sample, then reflect fold.
__device__ __forceinline__ float padded_grad(const float* df, int i, int n, int hop, int frames) {
  // frames f with f*hop <= i < f*hop + n
  int fhi = i / hop;
  if (fhi >= frames) fhi = frames - 1;
  float s = 0.f;
  for (int f = fhi; f >= 0; --f) {
    const int t = i - f * hop;
    if (t >= n) break;
    s += df[(int64_t)f * n + t];
  }
  return s;
}

__global__ __launch_bounds__(256) void stft_bwd_fold_kernel(const float* __restrict__ dframes, int L,
                                                            int n, int hop, int pad, int frames,
                                                            float* __restrict__ gx) {
  const int b = blockIdx.y;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= L) return;
  const float* df = dframes + (int64_t)b * frames * n;
  const int P = L + 2 * pad;
  float g = 0.f;
  // centre copy: padded index j + pad
  g += padded_grad(df, j + pad, n, hop, frames);
  // left reflection: padded i < pad maps to j = pad - i  (j in [1, pad])
  if (j >= 1 && j <= pad) g += padded_grad(df, pad - j, n, hop, frames);
  // right reflection: padded i >= pad + L maps to j = 2(L-1) - (i - pad)
  {
    const int i = 2 * (L - 1) - j + pad;
    if (i >= pad + L && i < P) g += padded_grad(df, i, n, hop, frames);
  }
  gx[(int64_t)b * L + j] = g;
}

int ilog2(int n) {
  int l = 0;
  while ((1 << l) < n) ++l;
  return (1 << l) == n ? l : -1;
}

}  // namespace

extern "C" int64_t vits_stft_workspace(int batch, int length, int n_fft, int hop, int pad) {
  if (batch <= 0 || n_fft <= 0 || hop <= 0) return 0;
  const int frames = (length + 2 * pad - n_fft) / hop + 1;
  if (frames <= 0) return 0;
  return (int64_t)batch * frames * n_fft;
}

extern "C" int vits_stft_mag_forward(const float* x, int batch, int length, const float* window,
                                     int n_fft, int hop, int win, int pad, float eps, float* mag,
                                     float* re, float* im, void* stream) {
  VITS_CHECK_ARG(x && window && mag && batch > 0 && length > 0 && hop > 0 && win > 0);
  const int log2n = ilog2(n_fft);
  VITS_CHECK_SHAPE(log2n >= 1 && n_fft <= FFT_MAX && win <= n_fft && pad >= 0 && pad < length);
  const int frames = (length + 2 * pad - n_fft) / hop + 1;
  VITS_CHECK_SHAPE(frames > 0);
  const int fpb = n_fft >= 1024 ? 1 : 1024 / n_fft;
  const size_t lds = sizeof(float2) * (2 * fpb * n_fft + n_fft / 2);
  dim3 grid((frames + fpb - 1) / fpb, batch);
  hipLaunchKernelGGL(stft_fwd_kernel, grid, dim3(256), lds, as_stream(stream), x, length, window,
                     n_fft, log2n, hop, win, pad, frames, fpb, eps, mag, re, im);
  return vits_launch_status();
}

extern "C" int vits_stft_mag_backward(const float* grad_mag, const float* mag, const float* re,
                                      const float* im, const float* window, int batch, int length,
                                      int n_fft, int hop, int win, int pad, float* grad_x,
                                      float* workspace, int64_t workspace_floats, void* stream) {
  VITS_CHECK_ARG(grad_mag && mag && re && im && window && grad_x && workspace);
  VITS_CHECK_ARG(batch > 0 && length > 0 && hop > 0 && win > 0);
  const int log2n = ilog2(n_fft);
  VITS_CHECK_SHAPE(log2n >= 1 && n_fft <= FFT_MAX && win <= n_fft && pad >= 0 && pad < length);
  const int frames = (length + 2 * pad - n_fft) / hop + 1;
  VITS_CHECK_SHAPE(frames > 0);
  if (workspace_floats < vits_stft_workspace(batch, length, n_fft, hop, pad)) return VITS_E_ARG;
  const int fpb = n_fft >= 1024 ? 1 : 1024 / n_fft;
  const size_t lds = sizeof(float2) * (2 * fpb * n_fft + n_fft / 2);
  hipStream_t s = as_stream(stream);
  dim3 grid((frames + fpb - 1) / fpb, batch);
  hipLaunchKernelGGL(stft_bwd_frames_kernel, grid, dim3(256), lds, s, grad_mag, mag, re, im,
                     window, n_fft, log2n, win, frames, fpb, workspace);
  int rc = vits_launch_status();
  if (rc) return rc;
  dim3 g2((length + 255) / 256, batch);
  hipLaunchKernelGGL(stft_bwd_fold_kernel, g2, dim3(256), 0, s, workspace, length, n_fft, hop, pad,
                     frames, grad_x);
  return vits_launch_status();
}
