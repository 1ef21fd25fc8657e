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
//   iteration per forward in training, mrd.py's discriminators):
//     v = normalize(W^T u) ; u = normalize(W v) ; sigma = u . (W v) ;
//     W_sn = W / sigma
//   as five grid-wide phases over all layers, and the backward of
//   W / sigma(W) with sigma = u . mv(W, v) (u, v constants):
//     dW = dW_sn / sigma + (-<dW_sn, W> / sigma^2) u v^T.
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
// Phases (one launch each, all layers of a list together; the per-layer
// block ranges of a launch are prefix sums in the arguments):
//   F1 (training)  t1 = W^T u           grid: layers x 64-column blocks
//   F2             v = normalize(t1)    one workgroup per layer
//   F3             t2 = W v             grid: layers x 4-row blocks (wave/row)
//   F4             u = normalize(t2), sigma = u . t2
//   F5             W_sn = W / sigma     grid: layers x element chunks
// t1 / t2 live in the v / u slots of `saved`.  The backward: B1 partial
// sums of <dW_sn, W> per chunk, B2 dW per chunk (every workgroup sums its
// layer's partials in the same order: deterministic).
struct SnGrid {
  vits_snorm_layer t[VITS_SNORM_MAX];
  int32_t bstart[VITS_SNORM_MAX + 1];
  int32_t n;
};
constexpr int SN_CHUNK = 4096;  // elements per workgroup in F5 / B1 / B2

// W_sn / dW_sn element of logical index i ([rows][cols] row-major): the same
// fp32 layout, or (cl_channels = C > 0) an fp16 [O][kh][kw][C] channels-last
// image of a Conv2d weight [O][C][kh][kw] (cols = C * kh * kw) - what the
// reference's autocast MIOpen conv gets after casting W / sigma
__device__ __forceinline__ int64_t sn_cl_index(int64_t i, int cols, int C) {
  const int64_t o = i / cols;
  const int rem = (int)(i - o * cols);
  const int hw = cols / C;
  const int c = rem / hw;
  const int p = rem - c * hw;
  return o * cols + (int64_t)p * C + c;
}

__device__ __forceinline__ int sn_layer_of(const SnGrid& G, int b) {
  int lo = 0, hi = G.n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (G.bstart[mid] <= b)
      lo = mid;
    else
      hi = mid - 1;
  }
  return lo;
}

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

// F1: t1[c] = h(sum_r h(W[r][c]) h(u[r])) for 64 columns; the 4 waves take
// rows r = w (mod 4), lane = column, then reduce through LDS
__global__ __launch_bounds__(256) void snorm_t1_kernel(const SnGrid G, int emu16) {
  const int b = blockIdx.x;
  const int l = sn_layer_of(G, b);
  const vits_snorm_layer& T = G.t[l];
  const bool emu = emu16 != 0;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int c = (b - G.bstart[l]) * 64 + lane;
  __shared__ float part[4][64];
  float acc = 0.f;
  if (c < T.cols) {
    const float* W = T.w + c;
    int r = wid;
    for (; r + 12 < T.rows; r += 16) {  // 4 independent loads in flight
      const float a0 = W[(int64_t)r * T.cols], a1 = W[(int64_t)(r + 4) * T.cols];
      const float a2 = W[(int64_t)(r + 8) * T.cols], a3 = W[(int64_t)(r + 12) * T.cols];
      acc += h16(a0, emu) * h16(T.u[r], emu);
      acc += h16(a1, emu) * h16(T.u[r + 4], emu);
      acc += h16(a2, emu) * h16(T.u[r + 8], emu);
      acc += h16(a3, emu) * h16(T.u[r + 12], emu);
    }
    for (; r < T.rows; r += 4) acc += h16(W[(int64_t)r * T.cols], emu) * h16(T.u[r], emu);
  }
  part[wid][lane] = acc;
  __syncthreads();
  if (wid == 0 && c < T.cols) {
    const float t = part[0][lane] + part[1][lane] + part[2][lane] + part[3][lane];
    T.saved[1 + T.rows + c] = h16(t, emu);
  }
}

// F2: v = t1 / max(||t1||, eps) (training) or v = the stored v (eval)
__global__ __launch_bounds__(256) void snorm_v_kernel(const SnGrid G, int training) {
  const vits_snorm_layer& T = G.t[blockIdx.x];
  float* sv = T.saved + 1 + T.rows;
  __shared__ float red[4];
  if (!training) {
    for (int c = threadIdx.x; c < T.cols; c += 256) sv[c] = T.v[c];
    return;
  }
  float ss = 0.f;
  for (int c = threadIdx.x; c < T.cols; c += 256) ss += sv[c] * sv[c];
  const float d = fmaxf(sqrtf(block_sum(ss, red)), T.eps);
  for (int c = threadIdx.x; c < T.cols; c += 256) {
    const float x = sv[c] / d;
    sv[c] = x;
    T.v[c] = x;
  }
}

// F3: t2[r] = h(sum_c h(W[r][c]) h(v[c])), one wave per row
__global__ __launch_bounds__(256) void snorm_t2_kernel(const SnGrid G, int emu16) {
  const int b = blockIdx.x;
  const int l = sn_layer_of(G, b);
  const vits_snorm_layer& T = G.t[l];
  const bool emu = emu16 != 0;
  const int lane = threadIdx.x & 63;
  const int r = (b - G.bstart[l]) * 4 + (threadIdx.x >> 6);
  if (r >= T.rows) return;
  const float* wr = T.w + (int64_t)r * T.cols;
  const float* sv = T.saved + 1 + T.rows;
  float acc = 0.f;
  for (int c = lane; c < T.cols; c += 64) acc += h16(wr[c], emu) * h16(sv[c], emu);
  acc = wave_sum(acc);
  if (lane == 0) T.saved[1 + r] = h16(acc, emu);
}

// F4: u = t2 / max(||t2||, eps) (training) or the stored u (eval);
// sigma = dot(u, t2) in fp32 (torch.dot promotes under autocast)
__global__ __launch_bounds__(256) void snorm_u_kernel(const SnGrid G, int training) {
  const vits_snorm_layer& T = G.t[blockIdx.x];
  float* su = T.saved + 1;
  __shared__ float red[4];
  float d = 1.f;
  if (training) {
    float ss = 0.f;
    for (int r = threadIdx.x; r < T.rows; r += 256) ss += su[r] * su[r];
    d = fmaxf(sqrtf(block_sum(ss, red)), T.eps);
  }
  float sg = 0.f;
  for (int r = threadIdx.x; r < T.rows; r += 256) {
    const float t2 = su[r];
    const float u = training ? t2 / d : T.u[r];
    sg += u * t2;
    su[r] = u;
    if (training) T.u[r] = u;
  }
  const float sigma = block_sum(sg, red);
  if (threadIdx.x == 0) T.saved[0] = sigma;
}

// F5: W_sn = W / sigma
__global__ __launch_bounds__(256) void snorm_out_kernel(const SnGrid G) {
  const int b = blockIdx.x;
  const int l = sn_layer_of(G, b);
  const vits_snorm_layer& T = G.t[l];
  const float sigma = T.saved[0];
  const int64_t n = (int64_t)T.rows * T.cols;
  const int64_t i0 = (int64_t)(b - G.bstart[l]) * SN_CHUNK;
  for (int64_t i = i0 + threadIdx.x; i < i0 + SN_CHUNK && i < n; i += 256)
    if (T.cl_channels > 0)
      reinterpret_cast<_Float16*>(T.w_sn)[sn_cl_index(i, T.cols, T.cl_channels)] =
          (_Float16)(T.w[i] / sigma);
    else
      T.w_sn[i] = T.w[i] / sigma;
}

__device__ __forceinline__ float sn_dw(const vits_snorm_layer& T, int64_t i) {
  if (T.cl_channels > 0)
    return (float)reinterpret_cast<const _Float16*>(T.dw_sn)[sn_cl_index(i, T.cols, T.cl_channels)];
  return T.dw_sn[i];
}

// B1: partial[chunk] = sum over the chunk of dW_sn * W
__global__ __launch_bounds__(256) void snorm_bwd_dot_kernel(const SnGrid G, float* __restrict__ part) {
  const int b = blockIdx.x;
  const int l = sn_layer_of(G, b);
  const vits_snorm_layer& T = G.t[l];
  const int64_t n = (int64_t)T.rows * T.cols;
  const int64_t i0 = (int64_t)(b - G.bstart[l]) * SN_CHUNK;
  __shared__ float red[4];
  float s = 0.f;
  for (int64_t i = i0 + threadIdx.x; i < i0 + SN_CHUNK && i < n; i += 256) s += sn_dw(T, i) * T.w[i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) part[b] = s;
}

// B2: dW = dW_sn / sigma + h(h(gs u[r]) h(v[c])),  gs = -<dW_sn, W> / sigma^2
__global__ __launch_bounds__(256) void snorm_bwd_kernel(const SnGrid G, const float* __restrict__ part,
                                                        int emu16) {
  const int b = blockIdx.x;
  const int l = sn_layer_of(G, b);
  const vits_snorm_layer& T = G.t[l];
  const bool emu = emu16 != 0;
  __shared__ float red[4];
  float s = 0.f;
  for (int q = G.bstart[l] + (int)threadIdx.x; q < G.bstart[l + 1]; q += 256) s += part[q];
  const float sigma = T.saved[0];
  const float gs = -block_sum(s, red) / (sigma * sigma);
  const float* u = T.saved + 1;
  const float* v = u + T.rows;
  const int64_t n = (int64_t)T.rows * T.cols;
  const int64_t i0 = (int64_t)(b - G.bstart[l]) * SN_CHUNK;
  for (int64_t i = i0 + threadIdx.x; i < i0 + SN_CHUNK && i < n; i += 256) {
    const int r = (int)(i / T.cols);
    const int c = (int)(i - (int64_t)r * T.cols);
    T.dw[i] = sn_dw(T, i) / sigma + h16(h16(gs * u[r], emu) * h16(v[c], emu), emu);
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

// block ranges of a list of layers: per-layer block count f(layer)
template <typename F>
static int sn_fill(SnGrid& G, const vits_snorm_layer* layers, int cnt, F blocks) {
  G.n = cnt;
  int tot = 0;
  for (int i = 0; i < cnt; ++i) {
    G.t[i] = layers[i];
    G.bstart[i] = tot;
    tot += blocks(layers[i]);
  }
  G.bstart[cnt] = tot;
  return tot;
}

static int sn_chunks(const vits_snorm_layer& t) {
  return (int)(((int64_t)t.rows * t.cols + SN_CHUNK - 1) / SN_CHUNK);
}

extern "C" int vits_spectral_norm_supported(int rows, int cols) {
  return rows > 0 && cols > 0 && (int64_t)rows * cols < (1LL << 31) ? 1 : 0;
}

extern "C" int vits_spectral_norm_forward(const vits_snorm_layer* layers, int n, int training,
                                          int emu16, void* stream) {
  VITS_CHECK_ARG(layers && n >= 0);
  hipStream_t s = as_stream(stream);
  for (int base = 0; base < n; base += VITS_SNORM_MAX) {
    const int cnt = n - base < VITS_SNORM_MAX ? n - base : VITS_SNORM_MAX;
    const vits_snorm_layer* ls = layers + base;
    for (int i = 0; i < cnt; ++i) {
      VITS_CHECK_ARG(ls[i].w && ls[i].u && ls[i].v && ls[i].w_sn && ls[i].saved);
      VITS_CHECK_ARG(ls[i].cl_channels >= 0 &&
                     (ls[i].cl_channels == 0 || ls[i].cols % ls[i].cl_channels == 0));
      if (!vits_spectral_norm_supported(ls[i].rows, ls[i].cols)) return VITS_E_UNSUP;
    }
    SnGrid G;
    int rc;
    if (training) {
      const int nb = sn_fill(G, ls, cnt, [](const vits_snorm_layer& t) { return (t.cols + 63) / 64; });
      hipLaunchKernelGGL(snorm_t1_kernel, dim3(nb), dim3(256), 0, s, G, emu16);
      if ((rc = vits_launch_status())) return rc;
    }
    sn_fill(G, ls, cnt, [](const vits_snorm_layer&) { return 1; });
    hipLaunchKernelGGL(snorm_v_kernel, dim3(cnt), dim3(256), 0, s, G, training);
    if ((rc = vits_launch_status())) return rc;
    int nb = sn_fill(G, ls, cnt, [](const vits_snorm_layer& t) { return (t.rows + 3) / 4; });
    hipLaunchKernelGGL(snorm_t2_kernel, dim3(nb), dim3(256), 0, s, G, emu16);
    if ((rc = vits_launch_status())) return rc;
    sn_fill(G, ls, cnt, [](const vits_snorm_layer&) { return 1; });
    hipLaunchKernelGGL(snorm_u_kernel, dim3(cnt), dim3(256), 0, s, G, training);
    if ((rc = vits_launch_status())) return rc;
    nb = sn_fill(G, ls, cnt, sn_chunks);
    hipLaunchKernelGGL(snorm_out_kernel, dim3(nb), dim3(256), 0, s, G);
    if ((rc = vits_launch_status())) return rc;
  }
  return VITS_OK;
}

extern "C" int64_t vits_spectral_norm_workspace(const vits_snorm_layer* layers, int n) {
  if (!layers || n < 0) return -1;
  int64_t tot = 0;
  for (int i = 0; i < n; ++i) tot += sn_chunks(layers[i]);
  return tot;
}

extern "C" int vits_spectral_norm_backward(const vits_snorm_layer* layers, int n, int emu16,
                                           float* workspace, int64_t ws_floats, void* stream) {
  VITS_CHECK_ARG(layers && n >= 0 && workspace);
  VITS_CHECK_ARG(ws_floats >= vits_spectral_norm_workspace(layers, n));
  hipStream_t s = as_stream(stream);
  float* part = workspace;
  for (int base = 0; base < n; base += VITS_SNORM_MAX) {
    const int cnt = n - base < VITS_SNORM_MAX ? n - base : VITS_SNORM_MAX;
    const vits_snorm_layer* ls = layers + base;
    for (int i = 0; i < cnt; ++i)
      VITS_CHECK_ARG(ls[i].w && ls[i].dw_sn && ls[i].dw && ls[i].saved && ls[i].rows > 0 &&
                     ls[i].cols > 0 && ls[i].cl_channels >= 0 &&
                     (ls[i].cl_channels == 0 || ls[i].cols % ls[i].cl_channels == 0));
    SnGrid G;
    const int nb = sn_fill(G, ls, cnt, sn_chunks);
    hipLaunchKernelGGL(snorm_bwd_dot_kernel, dim3(nb), dim3(256), 0, s, G, part);
    int rc = vits_launch_status();
    if (rc) return rc;
    hipLaunchKernelGGL(snorm_bwd_kernel, dim3(nb), dim3(256), 0, s, G, part, emu16);
    if ((rc = vits_launch_status())) return rc;
    part += nb;
  }
  return VITS_OK;
}
