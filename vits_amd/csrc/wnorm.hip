// wnorm.hip — the weight reparametrisations of the train_stft step as a few
// launches for the whole network instead of ~10 small torch ops per layer.
//
// * Weight normalisation (legacy torch.nn.utils.weight_norm, dim 0: every
//   generator conv / upsampler / conditioning Linear, modules.py:58-109,
//   models.py:233): w = v * (g / ||v_row||), one wave per row of dim 0 over
//   every layer of a launch (up to VITS_WNORM_MAX layers travel in the
//   kernel arguments), and its backward
//     dg = <dw, v_row> / n ,  dv = (g / n) * (dw - v * <dw, v_row> / n^2)
//   (torch's weight_norm_fwd/bwd_first_dim kernels, same formulas).
// * Spectral normalisation (torch.nn.utils.spectral_norm, dim 0, one power
//   iteration per forward in training, mrd.py's discriminators): one
//   workgroup per layer runs
//     v = normalize(W^T u) ; u = normalize(W v) ; sigma = u . (W v) ;
//     W_sn = W / sigma
//   and the backward of W / sigma(W) with sigma = u . mv(W, v) (u, v
//   constants):  dW = dW_sn / sigma + (-<dW_sn, W> / sigma^2) u v^T.
//   emu16: the reference runs the hook inside its fp16 autocast region, where
//   mv is an fp16 op (operands rounded to fp16, result rounded to fp16, fp32
//   accumulation) and dot / normalize promote back to fp32; emu16 = 1
//   reproduces those rounding points, including the fp16 outer product of
//   mv's backward.
#include "common.h"

namespace {

struct WnList {
  vits_wnorm_layer t[VITS_WNORM_MAX];
  int32_t rowstart[VITS_WNORM_MAX + 1];  // global row of each layer's row 0
  int32_t n;
};

__device__ __forceinline__ int wn_layer_of(const WnList& L, int gr) {
  int lo = 0, hi = L.n - 1;  // largest l with rowstart[l] <= gr
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (L.rowstart[mid] <= gr)
      lo = mid;
    else
      hi = mid - 1;
  }
  return lo;
}

__global__ __launch_bounds__(256) void wnorm_fwd_kernel(const WnList L, float* __restrict__ norms) {
  const int gr = (int)blockIdx.x * 4 + ((int)threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (gr >= L.rowstart[L.n]) return;
  const int l = wn_layer_of(L, gr);
  const vits_wnorm_layer& T = L.t[l];
  const int r = gr - L.rowstart[l];
  const int64_t base = (int64_t)r * T.cols;
  const float* v = T.v + base;
  float ss = 0.f;
  for (int c = lane; c < T.cols; c += 64) ss += v[c] * v[c];
  const float nrm = sqrtf(wave_sum(ss));
  const float s = T.g[r] / nrm;
  float* w = T.w + base;
  for (int c = lane; c < T.cols; c += 64) w[c] = v[c] * s;
  if (lane == 0) norms[gr] = nrm;
}

__global__ __launch_bounds__(256) void wnorm_bwd_kernel(const WnList L,
                                                        const float* __restrict__ norms) {
  const int gr = (int)blockIdx.x * 4 + ((int)threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (gr >= L.rowstart[L.n]) return;
  const int l = wn_layer_of(L, gr);
  const vits_wnorm_layer& T = L.t[l];
  const int r = gr - L.rowstart[l];
  const int64_t base = (int64_t)r * T.cols;
  const float* v = T.v + base;
  const float* dw = T.dw + base;
  float dot = 0.f;
  for (int c = lane; c < T.cols; c += 64) dot += dw[c] * v[c];
  dot = wave_sum(dot);
  const float nrm = norms[gr];
  const float rn = 1.0f / nrm;
  const float gn = T.g[r] * rn;
  const float k = dot * rn * rn;
  float* dv = T.dv + base;
  for (int c = lane; c < T.cols; c += 64) dv[c] = gn * (dw[c] - v[c] * k);
  if (lane == 0) T.dg[r] = dot * rn;
}

// ---- spectral norm -------------------------------------------------------
struct SnList {
  vits_snorm_layer t[VITS_SNORM_MAX];
};

__device__ __forceinline__ float h16(float x, bool emu) {
  return emu ? (float)(_Float16)x : x;
}

// sum over the 256 threads of a workgroup (red: 4 floats of LDS scratch)
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

__global__ __launch_bounds__(256) void snorm_fwd_kernel(const SnList L, int training, int emu16) {
  const vits_snorm_layer& T = L.t[blockIdx.x];
  const bool emu = emu16 != 0;
  const int rows = T.rows, cols = T.cols;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  extern __shared__ float sm[];
  float* su = sm;            // u  [rows]
  float* st = su + rows;     // mv(W, v) [rows]
  float* sv = st + rows;     // v  [cols]
  float* red = sv + cols;    // 4
  const float* W = T.w;
  if (training) {
    for (int r = tid; r < rows; r += 256) su[r] = h16(T.u[r], emu);
    __syncthreads();
    // v = normalize(W^T u)
    float ss = 0.f;
    for (int c = tid; c < cols; c += 256) {
      float acc = 0.f;
      for (int r = 0; r < rows; ++r) acc += h16(W[(int64_t)r * cols + c], emu) * su[r];
      acc = h16(acc, emu);
      sv[c] = acc;
      ss += acc * acc;
    }
    const float dv = fmaxf(sqrtf(block_sum(ss, red)), T.eps);
    for (int c = tid; c < cols; c += 256) {
      const float x = sv[c] / dv;
      T.v[c] = x;
      sv[c] = x;
    }
  } else {
    for (int c = tid; c < cols; c += 256) sv[c] = T.v[c];
  }
  __syncthreads();
  // t = mv(W, v): one wave per row
  for (int r = wid; r < rows; r += 4) {
    const float* wr = W + (int64_t)r * cols;
    float acc = 0.f;
    for (int c = lane; c < cols; c += 64) acc += h16(wr[c], emu) * h16(sv[c], emu);
    acc = wave_sum(acc);
    if (lane == 0) st[r] = h16(acc, emu);
  }
  __syncthreads();
  if (training) {
    // u = normalize(t)
    float ss = 0.f;
    for (int r = tid; r < rows; r += 256) ss += st[r] * st[r];
    const float du = fmaxf(sqrtf(block_sum(ss, red)), T.eps);
    for (int r = tid; r < rows; r += 256) {
      const float x = st[r] / du;
      T.u[r] = x;
      su[r] = x;
    }
  } else {
    for (int r = tid; r < rows; r += 256) su[r] = T.u[r];
  }
  __syncthreads();
  // sigma = dot(u, mv(W, v)) (fp32: dot promotes)
  float sg = 0.f;
  for (int r = tid; r < rows; r += 256) sg += su[r] * st[r];
  const float sigma = block_sum(sg, red);
  // saved for the backward: sigma, u, v of this call
  if (tid == 0) T.saved[0] = sigma;
  for (int r = tid; r < rows; r += 256) T.saved[1 + r] = su[r];
  for (int c = tid; c < cols; c += 256) T.saved[1 + rows + c] = sv[c];
  const int64_t n = (int64_t)rows * cols;
  for (int64_t i = tid; i < n; i += 256) T.w_sn[i] = W[i] / sigma;
}

__global__ __launch_bounds__(256) void snorm_bwd_kernel(const SnList L, int emu16) {
  const vits_snorm_layer& T = L.t[blockIdx.x];
  const bool emu = emu16 != 0;
  const int rows = T.rows, cols = T.cols;
  const int tid = threadIdx.x;
  __shared__ float red[4];
  const float sigma = T.saved[0];
  const float* u = T.saved + 1;
  const float* v = u + rows;
  const int64_t n = (int64_t)rows * cols;
  float s = 0.f;
  for (int64_t i = tid; i < n; i += 256) s += T.dw_sn[i] * T.w[i];
  // div backward for the divisor: sum(-g * W / sigma^2)
  const float gs = -block_sum(s, red) / (sigma * sigma);
  for (int r = 0; r < rows; ++r) {
    // dot backward (fp32) -> fp16 mv output gradient under emu16
    const float gt = h16(gs * u[r], emu);
    const float* gr = T.dw_sn + (int64_t)r * cols;
    float* out = T.dw + (int64_t)r * cols;
    for (int c = tid; c < cols; c += 256)
      out[c] = gr[c] / sigma + h16(gt * h16(v[c], emu), emu);
  }
}

}  // namespace

extern "C" int vits_weight_norm_forward(const vits_wnorm_layer* layers, int n, float* norms,
                                        void* stream) {
  VITS_CHECK_ARG(layers && norms && n >= 0);
  int row0 = 0;
  for (int base = 0; base < n; base += VITS_WNORM_MAX) {
    const int cnt = n - base < VITS_WNORM_MAX ? n - base : VITS_WNORM_MAX;
    WnList L;
    L.n = cnt;
    int rows = 0;
    for (int i = 0; i < cnt; ++i) {
      L.t[i] = layers[base + i];
      VITS_CHECK_ARG(L.t[i].v && L.t[i].g && L.t[i].w && L.t[i].rows > 0 && L.t[i].cols > 0);
      L.rowstart[i] = rows;
      rows += L.t[i].rows;
    }
    L.rowstart[cnt] = rows;
    hipLaunchKernelGGL(wnorm_fwd_kernel, dim3((rows + 3) / 4), dim3(256), 0, as_stream(stream), L,
                       norms + row0);
    const int rc = vits_launch_status();
    if (rc) return rc;
    row0 += rows;
  }
  return VITS_OK;
}

extern "C" int vits_weight_norm_backward(const vits_wnorm_layer* layers, int n, const float* norms,
                                         void* stream) {
  VITS_CHECK_ARG(layers && norms && n >= 0);
  int row0 = 0;
  for (int base = 0; base < n; base += VITS_WNORM_MAX) {
    const int cnt = n - base < VITS_WNORM_MAX ? n - base : VITS_WNORM_MAX;
    WnList L;
    L.n = cnt;
    int rows = 0;
    for (int i = 0; i < cnt; ++i) {
      L.t[i] = layers[base + i];
      VITS_CHECK_ARG(L.t[i].v && L.t[i].g && L.t[i].dw && L.t[i].dv && L.t[i].dg &&
                     L.t[i].rows > 0 && L.t[i].cols > 0);
      L.rowstart[i] = rows;
      rows += L.t[i].rows;
    }
    L.rowstart[cnt] = rows;
    hipLaunchKernelGGL(wnorm_bwd_kernel, dim3((rows + 3) / 4), dim3(256), 0, as_stream(stream), L,
                       norms + row0);
    const int rc = vits_launch_status();
    if (rc) return rc;
    row0 += rows;
  }
  return VITS_OK;
}

static size_t snorm_lds(const vits_snorm_layer& t) {
  return sizeof(float) * ((size_t)2 * t.rows + t.cols + 4);
}

extern "C" int vits_spectral_norm_supported(int rows, int cols) {
  vits_snorm_layer t{};
  t.rows = rows;
  t.cols = cols;
  return rows > 0 && cols > 0 && snorm_lds(t) <= VITS_SNORM_MAX_LDS ? 1 : 0;
}

extern "C" int vits_spectral_norm_forward(const vits_snorm_layer* layers, int n, int training,
                                          int emu16, void* stream) {
  VITS_CHECK_ARG(layers && n >= 0);
  for (int base = 0; base < n; base += VITS_SNORM_MAX) {
    const int cnt = n - base < VITS_SNORM_MAX ? n - base : VITS_SNORM_MAX;
    SnList L;
    size_t lds = 0;
    for (int i = 0; i < cnt; ++i) {
      L.t[i] = layers[base + i];
      const vits_snorm_layer& t = L.t[i];
      VITS_CHECK_ARG(t.w && t.u && t.v && t.w_sn && t.saved);
      if (!vits_spectral_norm_supported(t.rows, t.cols)) return VITS_E_UNSUP;
      if (snorm_lds(t) > lds) lds = snorm_lds(t);
    }
    hipLaunchKernelGGL(snorm_fwd_kernel, dim3(cnt), dim3(256), lds, as_stream(stream), L,
                       training, emu16);
    const int rc = vits_launch_status();
    if (rc) return rc;
  }
  return VITS_OK;
}

extern "C" int vits_spectral_norm_backward(const vits_snorm_layer* layers, int n, int emu16,
                                           void* stream) {
  VITS_CHECK_ARG(layers && n >= 0);
  for (int base = 0; base < n; base += VITS_SNORM_MAX) {
    const int cnt = n - base < VITS_SNORM_MAX ? n - base : VITS_SNORM_MAX;
    SnList L;
    for (int i = 0; i < cnt; ++i) {
      L.t[i] = layers[base + i];
      const vits_snorm_layer& t = L.t[i];
      VITS_CHECK_ARG(t.w && t.dw_sn && t.dw && t.saved && t.rows > 0 && t.cols > 0);
    }
    hipLaunchKernelGGL(snorm_bwd_kernel, dim3(cnt), dim3(256), 0, as_stream(stream), L, emu16);
    const int rc = vits_launch_status();
    if (rc) return rc;
  }
  return VITS_OK;
}
