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
#include <stdlib.h>

#include "common.h"

namespace {

constexpr int FFT_MAX = 2048;  // complex points per workgroup
constexpr int STFT_WG = 256;   // threads per workgroup (every launch below)
constexpr int STFT_PER = FFT_MAX / STFT_WG;  // staged elements per thread

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

// Compile-time twiddle table: (cos, sin)(2 pi m / FFT_MAX), m < FFT_MAX / 2,
// from double-precision Taylor series rounded to float (no per-workgroup
// sincos fill, no LDS for twiddles).  Size-n transforms read it with stride
// FFT_MAX / n.
struct TwTable {
  float c[FFT_MAX / 2];
  float s[FFT_MAX / 2];
};
constexpr double kPi = 3.14159265358979323846264338327950288;
constexpr double taylor_sin(double x) {
  double term = x, sum = x;
  for (int k = 1; k < 24; ++k) {
    term *= -x * x / ((2.0 * k) * (2.0 * k + 1.0));
    sum += term;
  }
  return sum;
}
constexpr double taylor_cos(double x) {
  double term = 1.0, sum = 1.0;
  for (int k = 1; k < 24; ++k) {
    term *= -x * x / ((2.0 * k - 1.0) * (2.0 * k));
    sum += term;
  }
  return sum;
}
constexpr TwTable make_tw() {
  TwTable t{};
  for (int m = 0; m < FFT_MAX / 2; ++m) {
    // reduce to [0, pi/2]: theta in [0, pi)
    const double th = 2.0 * kPi * m / FFT_MAX;
    const bool hi = th > kPi / 2;
    const double r = hi ? kPi - th : th;
    t.c[m] = (float)(hi ? -taylor_cos(r) : taylor_cos(r));
    t.s[m] = (float)taylor_sin(r);
  }
  return t;
}
__constant__ TwTable g_tw = make_tw();

// the workgroup's n/2 twiddles of size n, copied from the constant table
// into LDS (coalesced reads; divergent constant-table reads per butterfly
// measured slower: 182 -> 231 us)
__device__ void load_twiddles(float2* tw, int n) {
  const int stride = FFT_MAX / n;
  for (int m = threadIdx.x; m < (n >> 1); m += blockDim.x)
    tw[m] = make_float2(g_tw.c[m * stride], g_tw.s[m * stride]);
}

// Twiddle e^{sign 2 pi i m / n} for 0 <= m < n (e^{i(t + pi)} = -e^{i t}).
__device__ __forceinline__ float2 twiddle(const float2* tw, int m, int n, float sign) {
  const int half = n >> 1;
  float2 w = tw[m < half ? m : m - half];
  if (m >= half) w = make_float2(-w.x, -w.y);
  return make_float2(w.x, sign * w.y);
}

__device__ __forceinline__ float2 cmul(float2 a, float2 w) {
  return make_float2(a.x * w.x - a.y * w.y, a.x * w.y + a.y * w.x);
}

// Mixed radix-4 Stockham (one radix-2 stage first when log2 n is odd): the
// same autosort formulation as fft_lds with half the stages / barriers /
// LDS round trips.  Stage with span Ns and radix R, item j < n/R:
//   v[r] = src[j + r n/R] * e^{sign 2 pi i (j mod Ns) r / (Ns R)}
//   DFT_R(v) -> dst[(j / Ns) Ns R + (j mod Ns) + r Ns]
__device__ float2* fft_lds4(float2* a, float2* b, const float2* tw, int n, int log2n, int fpb,
                            float sign) {
  int ns = 1;
  if (log2n & 1) {  // radix-2 stage, Ns = 1: no twiddles
    const int half = n >> 1;
    for (int i = threadIdx.x; i < fpb * half; i += blockDim.x) {
      const int f = i / half;
      const int j = i - f * half;
      const float2 v0 = a[f * n + j], v1 = a[f * n + j + half];
      b[f * n + 2 * j] = make_float2(v0.x + v1.x, v0.y + v1.y);
      b[f * n + 2 * j + 1] = make_float2(v0.x - v1.x, v0.y - v1.y);
    }
    __syncthreads();
    float2* t = a;
    a = b;
    b = t;
    ns = 2;
  }
  const int q = n >> 2;
  for (; ns < n; ns <<= 2) {
    const int tstep = n / (ns * 4);  // table index per unit of (j mod Ns) r
    for (int i = threadIdx.x; i < fpb * q; i += blockDim.x) {
      const int f = i / q;
      const int j = i - f * q;
      const float2* src = a + f * n;
      float2* dst = b + f * n;
      const int k = j & (ns - 1);
      float2 v0 = src[j], v1 = src[j + q], v2 = src[j + 2 * q], v3 = src[j + 3 * q];
      if (ns > 1) {
        v1 = cmul(v1, twiddle(tw, k * tstep, n, sign));
        v2 = cmul(v2, twiddle(tw, 2 * k * tstep, n, sign));
        v3 = cmul(v3, twiddle(tw, 3 * k * tstep, n, sign));
      }
      const float2 t0 = make_float2(v0.x + v2.x, v0.y + v2.y);
      const float2 t1 = make_float2(v0.x - v2.x, v0.y - v2.y);
      const float2 t2 = make_float2(v1.x + v3.x, v1.y + v3.y);
      const float2 d13 = make_float2(v1.x - v3.x, v1.y - v3.y);
      // t3 = (sign i) (v1 - v3)
      const float2 t3 = sign < 0.f ? make_float2(d13.y, -d13.x) : make_float2(-d13.y, d13.x);
      const int o = ((j - k) << 2) + k;
      dst[o] = make_float2(t0.x + t2.x, t0.y + t2.y);
      dst[o + ns] = make_float2(t1.x + t3.x, t1.y + t3.y);
      dst[o + 2 * ns] = make_float2(t0.x - t2.x, t0.y - t2.y);
      dst[o + 3 * ns] = make_float2(t1.x - t3.x, t1.y - t3.y);
    }
    __syncthreads();
    float2* t = a;
    a = b;
    b = t;
  }
  return a;
}

// One transform job (a signal batch at one resolution), device side.
struct StftJobD {
  const float* x;       // forward input [B][L]
  const float* window;  // [win]
  const float* gmag;    // backward: d loss / d mag
  float* mag;           // [B][n/2+1][frames]
  float* re;
  float* im;
  float* dframes;       // backward workspace [B][frames][n]
  float* gx;            // backward output [B][L]
  int L, n, log2n, hop, win, pad, frames, fpb, batch;
  float eps;
  int fmajor;  // mag / re / im / grad_mag as [B][frames][n/2+1] (else [B][n/2+1][frames])
};

// forward: frames f0 .. f0+fpb-1 of utterance b (radix-4 Stockham, fft_lds4;
// fft_lds is the radix-2 reference formulation it replaced)
__device__ void stft_fwd_block(const StftJobD& J, int fblk, int b, float2* sfft) {
  const int n = J.n, fpb = J.fpb;
  float2* a = sfft;
  float2* bbuf = sfft + fpb * n;
  float2* tw = bbuf + fpb * n;
  load_twiddles(tw, n);
  const int f0 = fblk * fpb;
  const int woff = (n - J.win) / 2;
  const float* xb = J.x + (int64_t)b * J.L;
  // every element's loads issued before the first LDS store (a per-element
  // load-use chain serialised up to 8 global latencies per workgroup)
  float xv[STFT_PER], wv[STFT_PER];
#pragma unroll
  for (int q = 0; q < STFT_PER; ++q) {
    const int i = threadIdx.x + q * STFT_WG;
    const int f = i / n;
    const int t = i - f * n;
    const int fr = f0 + f;
    const int wi = t - woff;
    const bool ok = i < fpb * n && fr < J.frames && wi >= 0 && wi < J.win;
    const int src = ok ? reflect_idx(fr * J.hop + t - J.pad, J.L) : 0;
    xv[q] = ok ? xb[src] : 0.f;
    wv[q] = ok ? J.window[wi] : 0.f;
  }
#pragma unroll
  for (int q = 0; q < STFT_PER; ++q) {
    const int i = threadIdx.x + q * STFT_WG;
    if (i < fpb * n) a[i] = make_float2(xv[q] * wv[q], 0.f);
  }
  __syncthreads();
  const float2* out = fft_lds4(a, bbuf, tw, n, J.log2n, fpb, -1.f);
  const int nb = n / 2 + 1;
  if (J.fmajor) {
    // frame-major: the workgroup's fpb frames are one contiguous run of
    // fpb * nb outputs - every store instruction writes whole lines
    const int nf = min(fpb, J.frames - f0);
    const int64_t base = ((int64_t)b * J.frames + f0) * nb;
    for (int i = threadIdx.x; i < nf * nb; i += blockDim.x) {
      const int f = i / nb;
      const float2 c = out[f * n + (i - f * nb)];
      J.mag[base + i] = sqrtf(c.x * c.x + c.y * c.y + J.eps);
      if (J.re) J.re[base + i] = c.x;
      if (J.im) J.im[base + i] = c.y;
    }
    return;
  }
  for (int i = threadIdx.x; i < fpb * nb; i += blockDim.x) {
    const int k = i / fpb;
    const int f = i - k * fpb;
    const int fr = f0 + f;
    if (fr >= J.frames) continue;
    const float2 c = out[f * n + k];
    const int64_t o = ((int64_t)b * nb + k) * J.frames + fr;
    J.mag[o] = sqrtf(c.x * c.x + c.y * c.y + J.eps);
    if (J.re) J.re[o] = c.x;
    if (J.im) J.im[o] = c.y;
  }
}

// backward, per frame: d mag / d(re, im) = (re, im) / mag, adjoint real DFT
// = real part of the inverse FFT of the one-sided spectrum, windowed
__device__ void stft_bwd_frames_block(const StftJobD& J, int fblk, int b, float2* sfft) {
  const int n = J.n, fpb = J.fpb;
  float2* a = sfft;
  float2* bbuf = sfft + fpb * n;
  float2* tw = bbuf + fpb * n;
  load_twiddles(tw, n);
  const int f0 = fblk * fpb;
  const int nb = n / 2 + 1;
  const int woff = (n - J.win) / 2;
  float gm[STFT_PER], mg[STFT_PER], rr[STFT_PER], ii[STFT_PER];
#pragma unroll
  for (int q = 0; q < STFT_PER; ++q) {
    const int i = threadIdx.x + q * STFT_WG;
    // element (bin k, frame f) of this thread: ordered so the reads run along
    // the contiguous axis of the layout (frames, or bins when frame-major)
    int k, f;
    if (J.fmajor) {
      f = i / n;
      k = i - f * n;
    } else {
      k = i / fpb;
      f = i - k * fpb;
    }
    const int fr = f0 + f;
    const bool ok = i < fpb * n && k < nb && fr < J.frames;
    const int64_t o = !ok ? 0
                      : J.fmajor ? ((int64_t)b * J.frames + fr) * nb + k
                                 : ((int64_t)b * nb + k) * J.frames + fr;
    gm[q] = ok ? J.gmag[o] : 0.f;
    mg[q] = ok ? J.mag[o] : 1.f;
    rr[q] = ok ? J.re[o] : 0.f;
    ii[q] = ok ? J.im[o] : 0.f;
  }
#pragma unroll
  for (int q = 0; q < STFT_PER; ++q) {
    const int i = threadIdx.x + q * STFT_WG;
    if (i < fpb * n) {
      int k, f;
      if (J.fmajor) {
        f = i / n;
        k = i - f * n;
      } else {
        k = i / fpb;
        f = i - k * fpb;
      }
      const float sc = gm[q] / mg[q];
      a[f * n + k] = make_float2(sc * rr[q], sc * ii[q]);
    }
  }
  __syncthreads();
  const float2* out = fft_lds4(a, bbuf, tw, n, J.log2n, fpb, +1.f);
  for (int i = threadIdx.x; i < fpb * n; i += blockDim.x) {
    const int f = i / n;
    const int t = i - f * n;
    const int fr = f0 + f;
    if (fr >= J.frames) continue;
    const int wi = t - woff;
    const float w = (wi >= 0 && wi < J.win) ? J.window[wi] : 0.f;
    J.dframes[((int64_t)b * J.frames + fr) * n + t] = out[f * n + t].x * w;
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

__device__ void stft_bwd_fold_block(const StftJobD& J, int jblk, int b) {
  const int j = jblk * blockDim.x + threadIdx.x;
  const int L = J.L, n = J.n, hop = J.hop, pad = J.pad, frames = J.frames;
  if (j >= L) return;
  const float* df = J.dframes + (int64_t)b * frames * n;
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
  J.gx[(int64_t)b * L + j] = g;
}

// ---------------------------------------------------------------------------
// Forward, two-pass register FFT (n = N1 * N2, the four-step factorisation):
//   pass 1, item (frame f, column t2):  Y[k1] = DFT_N1 over t1 of
//           x[N2 t1 + t2] (loaded windowed + reflect-padded straight from
//           global memory into registers), times W_n^{t2 k1} -> LDS
//   pass 2, item (frame f, row k1):     X[k1 + N1 k2] = DFT_N2 over t2 of the
//           LDS column, |X| (and re / im) of the one-sided bins -> global
// Each point crosses LDS once (one write, one read, one barrier) instead of
// once per radix-4 stage, and the DFTs run unrolled in registers with
// compile-time twiddles; F frames per workgroup (F n = 4096 points).
// LDS planes are [F][N2][N1 + 1] floats (re, im): odd row stride, no bank
// conflicts on the column writes / row reads.
// ---------------------------------------------------------------------------
constexpr TwTable kTwC = make_tw();  // compile-time copy for the register DFTs

constexpr int brev_c(int i, int logn) {
  int r = 0;
  for (int b = 0; b < logn; ++b) r |= ((i >> b) & 1) << (logn - 1 - b);
  return r;
}
constexpr int ilog2_c(int n) { return n <= 1 ? 0 : 1 + ilog2_c(n >> 1); }

// forward DFT (e^{-i}) of N <= 64 points held in registers, natural order in
// and out: bit-reversed renaming, then radix-2 decimation in time; every
// index and twiddle is a compile-time constant after unrolling
template <int N>
__device__ __forceinline__ void dft_reg(float (&xr)[N], float (&xi)[N]) {
  constexpr int LN = ilog2_c(N);
  float ar[N], ai[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    ar[brev_c(i, LN)] = xr[i];
    ai[brev_c(i, LN)] = xi[i];
  }
#pragma unroll
  for (int m = 2; m <= N; m <<= 1) {
#pragma unroll
    for (int k = 0; k < N; k += m) {
#pragma unroll
      for (int j = 0; j < m / 2; ++j) {
        const int p = k + j, q = k + j + m / 2;
        float vr, vi;
        if (j == 0) {
          vr = ar[q];
          vi = ai[q];
        } else if (4 * j == m) {  // W = -i
          vr = ai[q];
          vi = -ar[q];
        } else {
          const float c = kTwC.c[j * (FFT_MAX / m)];
          const float sn = -kTwC.s[j * (FFT_MAX / m)];
          vr = ar[q] * c - ai[q] * sn;
          vi = ar[q] * sn + ai[q] * c;
        }
        const float ur = ar[p], ui = ai[p];
        ar[p] = ur + vr;
        ai[p] = ui + vi;
        ar[q] = ur - vr;
        ai[q] = ui - vi;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < N; ++i) {
    xr[i] = ar[i];
    xi[i] = ai[i];
  }
}

// SP2: pass 2 as two half-size DFTs per row (radix-2 decimation in
// frequency: even bins = DFT_{N2/2}(y[t] + y[t + N2/2]), odd bins =
// DFT_{N2/2}((y[t] - y[t + N2/2]) W_N2^t)), one per thread - keeps n = 2048
// (N2 = 64) at the register footprint of a 32-point DFT
template <int N1, int N2, int F, bool SP2 = false>
__device__ void stft_fwd2_block(const StftJobD& J, int fblk, int b, float* sm) {
  constexpr int n = N1 * N2;
  constexpr int YS = N1 + 1;
  static_assert(F * N2 <= STFT_WG, "one pass-1 item per thread (the staging aliases Y)");
  float* const twc = sm;  // W_n^m = cos - i sin (2 pi m / n), m < n
  float* const tws = sm + n;
  float* const yre = sm + 2 * n;
  float* const yim = yre + F * N2 * YS;
  // the workgroup's signal segment (its F frames overlap by n - hop) and the
  // zero-extended window, staged once with coalesced loads (reflect padding
  // applied here); aliased by Y after every thread holds its column
  float* const xs = sm + 2 * n;
  const int f0 = fblk * F;
  const int seg0 = f0 * J.hop - J.pad;
  const int seglen = (F - 1) * J.hop + n;
  float* const ws = xs + seglen;
  const int woff = (n - J.win) / 2;
  const float* xb = J.x + (int64_t)b * J.L;
  // staging in groups of UNR elements per thread whose loads are all issued
  // (from clamped addresses, zeroed after) before the first LDS write: a
  // conditional load per element is a branch with its own wait, one memory
  // round trip per element
  constexpr int UNR = 8;
  for (int m0 = threadIdx.x; m0 < n; m0 += STFT_WG * UNR) {
    float c[UNR], sn[UNR], wv[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int m = m0 + u * STFT_WG;
      const int mm = m < n ? m : 0;
      const int h = mm < n / 2 ? mm : mm - n / 2;
      const int wi = mm - woff;
      c[u] = g_tw.c[h * (FFT_MAX / n)];
      sn[u] = g_tw.s[h * (FFT_MAX / n)];
      wv[u] = J.window[(wi >= 0 && wi < J.win) ? wi : 0];
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int m = m0 + u * STFT_WG;
      if (m < n) {
        const int wi = m - woff;
        twc[m] = m < n / 2 ? c[u] : -c[u];
        tws[m] = m < n / 2 ? sn[u] : -sn[u];
        ws[m] = (wi >= 0 && wi < J.win) ? wv[u] : 0.f;
      }
    }
  }
  for (int i0 = threadIdx.x; i0 < seglen; i0 += STFT_WG * UNR) {
    float v[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int i = i0 + u * STFT_WG;
      const int t = seg0 + i;
      const bool ok = i < seglen && t >= -J.pad && t < J.L + J.pad;
      v[u] = xb[ok ? reflect_idx(t, J.L) : 0];
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int i = i0 + u * STFT_WG;
      const int t = seg0 + i;
      if (i < seglen) xs[i] = (t >= -J.pad && t < J.L + J.pad) ? v[u] : 0.f;
    }
  }
  __syncthreads();
  const int it = threadIdx.x;
  const bool act1 = it < F * N2;
  const int f = it / N2;
  const int t2 = it - f * N2;
  float xr[N1], xi[N1];
  if (act1) {
    const bool live = f0 + f < J.frames;
#pragma unroll
    for (int t1 = 0; t1 < N1; ++t1) {
      const int t = N2 * t1 + t2;
      xr[t1] = live ? xs[f * J.hop + t] * ws[t] : 0.f;
      xi[t1] = 0.f;
    }
  }
  __syncthreads();  // Y overwrites the staged segment
  if (act1) {
    dft_reg<N1>(xr, xi);
    float* const ro = yre + (f * N2 + t2) * YS;
    float* const io = yim + (f * N2 + t2) * YS;
    ro[0] = xr[0];
    io[0] = xi[0];
#pragma unroll
    for (int k1 = 1; k1 < N1; ++k1) {
      const int m = t2 * k1;  // < n
      const float c = twc[m], sn = -tws[m];
      ro[k1] = xr[k1] * c - xi[k1] * sn;
      io[k1] = xr[k1] * sn + xi[k1] * c;
    }
  }
  __syncthreads();
  const int nb = n / 2 + 1;
  if constexpr (SP2) {
    constexpr int H = N2 / 2;
    for (int it = threadIdx.x; it < 2 * F * N1; it += STFT_WG) {
      const int par = it & 1;  // neighbouring lanes: even / odd bins of one row
      const int r = it >> 1;
      int f, k1;
      if (J.fmajor) {
        f = r / N1;
        k1 = r - f * N1;
      } else {
        k1 = r / F;
        f = r - k1 * F;
      }
      const int fr = f0 + f;
      float xr[H], xi[H];
#pragma unroll
      for (int t = 0; t < H; ++t) {
        const float ar = yre[(f * N2 + t) * YS + k1], ai = yim[(f * N2 + t) * YS + k1];
        const float br = yre[(f * N2 + t + H) * YS + k1], bi = yim[(f * N2 + t + H) * YS + k1];
        if (par == 0) {
          xr[t] = ar + br;
          xi[t] = ai + bi;
        } else {
          const float dr = ar - br, di = ai - bi;
          if (t == 0) {
            xr[t] = dr;
            xi[t] = di;
          } else {
            const float c = kTwC.c[t * (FFT_MAX / N2)], sn = -kTwC.s[t * (FFT_MAX / N2)];
            xr[t] = dr * c - di * sn;
            xi[t] = dr * sn + di * c;
          }
        }
      }
      dft_reg<H>(xr, xi);
      if (fr >= J.frames) continue;
#pragma unroll
      for (int q = 0; q <= H / 2; ++q) {
        const int k = k1 + N1 * (2 * q + par);
        if (k < nb) {
          const int64_t o = J.fmajor ? ((int64_t)b * J.frames + fr) * nb + k
                                     : ((int64_t)b * nb + k) * J.frames + fr;
          J.mag[o] = sqrtf(xr[q] * xr[q] + xi[q] * xi[q] + J.eps);
          if (J.re) J.re[o] = xr[q];
          if (J.im) J.im[o] = xi[q];
        }
      }
    }
    return;
  }
  for (int it = threadIdx.x; it < F * N1; it += STFT_WG) {
    int f, k1;
    if (J.fmajor) {
      f = it / N1;
      k1 = it - f * N1;
    } else {
      k1 = it / F;
      f = it - k1 * F;
    }
    const int fr = f0 + f;
    float xr[N2], xi[N2];
#pragma unroll
    for (int t2 = 0; t2 < N2; ++t2) {
      xr[t2] = yre[(f * N2 + t2) * YS + k1];
      xi[t2] = yim[(f * N2 + t2) * YS + k1];
    }
    dft_reg<N2>(xr, xi);
    if (fr >= J.frames) continue;
#pragma unroll
    for (int k2 = 0; k2 <= N2 / 2; ++k2) {
      const int k = k1 + N1 * k2;
      if (k < nb) {
        const int64_t o = J.fmajor ? ((int64_t)b * J.frames + fr) * nb + k
                                   : ((int64_t)b * nb + k) * J.frames + fr;
        J.mag[o] = sqrtf(xr[k2] * xr[k2] + xi[k2] * xi[k2] + J.eps);
        if (J.re) J.re[o] = xr[k2];
        if (J.im) J.im[o] = xi[k2];
      }
    }
  }
}

// (N1, N2, F) per size; 0 frames = size not covered (radix-4 Stockham path)
__host__ __device__ constexpr int fwd2_frames(int n) {
  return n == 128 ? 32 : n == 256 ? 16 : n == 512 ? 8 : n == 1024 ? 4 : n == 2048 ? 2 : 0;
}
size_t fwd2_lds(int n, int hop) {
  const int n1 = n == 128 ? 16 : n == 256 ? 16 : n == 512 ? 16 : 32;
  const int F = fwd2_frames(n);
  const int y = 2 * F * (n / n1) * (n1 + 1);  // Y planes
  const int st = (F - 1) * hop + 2 * n;         // staged segment + window (aliased by Y)
  return sizeof(float) * (2 * n + (y > st ? y : st));
}
__device__ void stft_fwd2_any(const StftJobD& J, int fblk, int b, float* sm) {
  switch (J.n) {
    case 128: stft_fwd2_block<16, 8, 32>(J, fblk, b, sm); break;
    case 256: stft_fwd2_block<16, 16, 16>(J, fblk, b, sm); break;
    case 512: stft_fwd2_block<16, 32, 8>(J, fblk, b, sm); break;
    case 1024: stft_fwd2_block<32, 32, 4>(J, fblk, b, sm); break;
    case 2048: stft_fwd2_block<32, 64, 2, true>(J, fblk, b, sm); break;
    default: break;
  }
}

// ---- launch-level: one job (grid.y = utterance) or up to MAX_JOBS jobs in
// one launch (grid.x runs over every job's blocks; a block finds its job in
// the prefix table), so the ten transforms of an MR-STFT loss fill the chip
// as one launch instead of ten small ones
constexpr int STFT_MAX_JOBS = 16;
struct StftJobs {
  StftJobD job[STFT_MAX_JOBS];
  int end[STFT_MAX_JOBS];  // exclusive prefix of blocks per job
  int per_b[STFT_MAX_JOBS];  // blocks per utterance
  int njobs;
};

__device__ __forceinline__ int find_job(const StftJobs& J, int blk) {
  int j = 0;
  while (j + 1 < J.njobs && blk >= J.end[j]) ++j;
  return j;
}

__global__ __launch_bounds__(256) void stft_fwd_kernel(const StftJobD J) {
  extern __shared__ float2 sfft[];
  stft_fwd_block(J, blockIdx.x, blockIdx.y, sfft);
}

__global__ __launch_bounds__(256) void stft_fwd_multi_kernel(const StftJobs J) {
  extern __shared__ float2 sfft[];
  const int j = find_job(J, blockIdx.x);
  const int local = blockIdx.x - (j ? J.end[j - 1] : 0);
  const int b = local / J.per_b[j];
  stft_fwd_block(J.job[j], local - b * J.per_b[j], b, sfft);
}

__global__ __launch_bounds__(256) void stft_fwd2_kernel(const StftJobD J) {
  extern __shared__ float sm2[];
  stft_fwd2_any(J, blockIdx.x, blockIdx.y, sm2);
}

__global__ __launch_bounds__(256) void stft_fwd2_multi_kernel(const StftJobs J) {
  extern __shared__ float sm2[];
  const int j = find_job(J, blockIdx.x);
  const int local = blockIdx.x - (j ? J.end[j - 1] : 0);
  const int b = local / J.per_b[j];
  stft_fwd2_any(J.job[j], local - b * J.per_b[j], b, sm2);
}

__global__ __launch_bounds__(256) void stft_bwd_frames_kernel(const StftJobD J) {
  extern __shared__ float2 sfft[];
  stft_bwd_frames_block(J, blockIdx.x, blockIdx.y, sfft);
}

__global__ __launch_bounds__(256) void stft_bwd_frames_multi_kernel(const StftJobs J) {
  extern __shared__ float2 sfft[];
  const int j = find_job(J, blockIdx.x);
  const int local = blockIdx.x - (j ? J.end[j - 1] : 0);
  const int b = local / J.per_b[j];
  stft_bwd_frames_block(J.job[j], local - b * J.per_b[j], b, sfft);
}

__global__ __launch_bounds__(256) void stft_bwd_fold_kernel(const StftJobD J) {
  stft_bwd_fold_block(J, blockIdx.x, blockIdx.y);
}

__global__ __launch_bounds__(256) void stft_bwd_fold_multi_kernel(const StftJobs J) {
  const int j = find_job(J, blockIdx.x);
  const int local = blockIdx.x - (j ? J.end[j - 1] : 0);
  const int b = local / J.per_b[j];
  stft_bwd_fold_block(J.job[j], local - b * J.per_b[j], b);
}

int ilog2(int n) {
  int l = 0;
  while ((1 << l) < n) ++l;
  return (1 << l) == n ? l : -1;
}

// host: fill one device job from the C-ABI arguments; 0 or a VITS_E code
int make_job(StftJobD& J, const float* x, int batch, int length, const float* window, int n_fft,
             int hop, int win, int pad, float eps) {
  VITS_CHECK_ARG(window && batch > 0 && length > 0 && hop > 0 && win > 0);
  const int log2n = ilog2(n_fft);
  VITS_CHECK_SHAPE(log2n >= 1 && n_fft <= FFT_MAX && win <= n_fft && pad >= 0 && pad < length);
  const int frames = (length + 2 * pad - n_fft) / hop + 1;
  VITS_CHECK_SHAPE(frames > 0);
  J = StftJobD{};
  J.x = x;
  J.window = window;
  J.L = length;
  J.n = n_fft;
  J.log2n = log2n;
  J.hop = hop;
  J.win = win;
  J.pad = pad;
  J.frames = frames;
  J.fpb = n_fft >= 1024 ? 1 : 1024 / n_fft;
  J.batch = batch;
  J.eps = eps;
  return VITS_OK;
}

size_t job_lds(const StftJobD& J) { return sizeof(float2) * (2 * J.fpb * J.n + J.n / 2); }
int job_fblocks(const StftJobD& J) { return (J.frames + J.fpb - 1) / J.fpb; }

// forward kind: the two-pass register FFT for n = 128 .. 2048, the radix-4
// Stockham LDS FFT for other sizes
bool use_fwd2(int n, int hop) {
  return fwd2_frames(n) > 0 && hop <= n && fwd2_lds(n, hop) <= 64 * 1024;
}
int fwd2_fblocks(const StftJobD& J) {
  const int f = fwd2_frames(J.n);
  return (J.frames + f - 1) / f;
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
  VITS_CHECK_ARG(x && mag);
  StftJobD J;
  int rc = make_job(J, x, batch, length, window, n_fft, hop, win, pad, eps);
  if (rc) return rc;
  J.mag = mag;
  J.re = re;
  J.im = im;
  if (use_fwd2(n_fft, hop)) {
    hipLaunchKernelGGL(stft_fwd2_kernel, dim3(fwd2_fblocks(J), batch), dim3(256), fwd2_lds(n_fft, hop),
                       as_stream(stream), J);
    return vits_launch_status();
  }
  dim3 grid(job_fblocks(J), batch);
  hipLaunchKernelGGL(stft_fwd_kernel, grid, dim3(256), job_lds(J), as_stream(stream), J);
  return vits_launch_status();
}

extern "C" int vits_stft_mag_backward(const float* grad_mag, const float* mag, const float* re,
                                      const float* im, const float* window, int batch, int length,
                                      int n_fft, int hop, int win, int pad, float* grad_x,
                                      float* workspace, int64_t workspace_floats, void* stream) {
  VITS_CHECK_ARG(grad_mag && mag && re && im && grad_x && workspace);
  StftJobD J;
  int rc = make_job(J, nullptr, batch, length, window, n_fft, hop, win, pad, 0.f);
  if (rc) return rc;
  if (workspace_floats < vits_stft_workspace(batch, length, n_fft, hop, pad)) return VITS_E_ARG;
  J.gmag = grad_mag;
  J.mag = const_cast<float*>(mag);
  J.re = const_cast<float*>(re);
  J.im = const_cast<float*>(im);
  J.dframes = workspace;
  J.gx = grad_x;
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(stft_bwd_frames_kernel, dim3(job_fblocks(J), batch), dim3(256), job_lds(J), s,
                     J);
  rc = vits_launch_status();
  if (rc) return rc;
  hipLaunchKernelGGL(stft_bwd_fold_kernel, dim3((length + 255) / 256, batch), dim3(256), 0, s, J);
  return vits_launch_status();
}

extern "C" int vits_stft_mag_forward_multi(const vits_stft_job* jobs, int njobs, void* stream) {
  VITS_CHECK_ARG(jobs && njobs > 0 && njobs <= STFT_MAX_JOBS);
  // two launches at most: the sizes the two-pass kernel covers, the rest on
  // the Stockham kernel (each launch walks its own job table)
  StftJobs M[2] = {};
  size_t lds[2] = {0, 0};
  int blocks[2] = {0, 0};
  for (int i = 0; i < njobs; ++i) {
    const vits_stft_job& q = jobs[i];
    VITS_CHECK_ARG(q.x && q.mag);
    const int kind = use_fwd2(q.n_fft, q.hop) ? 0 : 1;
    StftJobs& S = M[kind];
    const int j = S.njobs++;
    int rc = make_job(S.job[j], q.x, q.batch, q.length, q.window, q.n_fft, q.hop, q.win, q.pad,
                      q.eps);
    if (rc) return rc;
    S.job[j].mag = q.mag;
    S.job[j].re = q.re;
    S.job[j].im = q.im;
    S.job[j].fmajor = q.layout;
    S.per_b[j] = kind == 0 ? fwd2_fblocks(S.job[j]) : job_fblocks(S.job[j]);
    blocks[kind] += S.per_b[j] * q.batch;
    S.end[j] = blocks[kind];
    const size_t l = kind == 0 ? fwd2_lds(q.n_fft, q.hop) : job_lds(S.job[j]);
    lds[kind] = l > lds[kind] ? l : lds[kind];
  }
  hipStream_t s = as_stream(stream);
  if (M[0].njobs) {
    hipLaunchKernelGGL(stft_fwd2_multi_kernel, dim3(blocks[0]), dim3(256), lds[0], s, M[0]);
    int rc = vits_launch_status();
    if (rc) return rc;
  }
  if (M[1].njobs)
    hipLaunchKernelGGL(stft_fwd_multi_kernel, dim3(blocks[1]), dim3(256), lds[1], s, M[1]);
  return vits_launch_status();
}

extern "C" int64_t vits_stft_workspace_multi(const vits_stft_job* jobs, int njobs) {
  if (!jobs || njobs <= 0) return 0;
  int64_t tot = 0;
  for (int i = 0; i < njobs; ++i)
    tot += vits_stft_workspace(jobs[i].batch, jobs[i].length, jobs[i].n_fft, jobs[i].hop,
                               jobs[i].pad);
  return tot;
}

extern "C" int vits_stft_mag_backward_multi(const vits_stft_job* jobs, int njobs,
                                            float* workspace, int64_t workspace_floats,
                                            void* stream) {
  VITS_CHECK_ARG(jobs && njobs > 0 && njobs <= STFT_MAX_JOBS && workspace);
  if (workspace_floats < vits_stft_workspace_multi(jobs, njobs)) return VITS_E_ARG;
  StftJobs M{}, F{};
  M.njobs = F.njobs = njobs;
  size_t lds = 0;
  int blocks = 0, fblocks = 0;
  int64_t woff = 0;
  for (int i = 0; i < njobs; ++i) {
    const vits_stft_job& q = jobs[i];
    VITS_CHECK_ARG(q.grad_mag && q.mag && q.re && q.im && q.grad_x);
    int rc = make_job(M.job[i], nullptr, q.batch, q.length, q.window, q.n_fft, q.hop, q.win,
                      q.pad, 0.f);
    if (rc) return rc;
    StftJobD& J = M.job[i];
    J.gmag = q.grad_mag;
    J.mag = q.mag;
    J.re = q.re;
    J.im = q.im;
    J.dframes = workspace + woff;
    J.gx = q.grad_x;
    J.fmajor = q.layout;
    woff += vits_stft_workspace(q.batch, q.length, q.n_fft, q.hop, q.pad);
    F.job[i] = J;
    M.per_b[i] = job_fblocks(J);
    blocks += M.per_b[i] * q.batch;
    M.end[i] = blocks;
    F.per_b[i] = (q.length + 255) / 256;
    fblocks += F.per_b[i] * q.batch;
    F.end[i] = fblocks;
    lds = job_lds(J) > lds ? job_lds(J) : lds;
  }
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(stft_bwd_frames_multi_kernel, dim3(blocks), dim3(256), lds, s, M);
  int rc = vits_launch_status();
  if (rc) return rc;
  hipLaunchKernelGGL(stft_bwd_fold_multi_kernel, dim3(fblocks), dim3(256), 0, s, F);
  return vits_launch_status();
}
