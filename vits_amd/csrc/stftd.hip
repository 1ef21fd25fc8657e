// stftd.hip — the element-wise glue around the STFT discriminators' 2-D
// convs in the fp16-autocast training step (mrd.py:94-156: Conv2d ->
// LeakyReLU(0.2) -> Conv2d ... ; train_stft.py:196-214).
//
// The layers after the first run on MIOpen's channels-last (NHWC) solvers;
// the first layer runs on the HIP training conv over frequency rows joined
// along time (discriminators.conv2d_freq: [B][C][F_out * L], row f's T
// outputs at columns f*L + p1 .. f*L + p1 + T).  Two kernel pairs replace
// what torch launches around those convs:
//
//  join_to_cl (forward): out[b][f][t][c] = lrelu(y[b][c][f*L + p1 + t]) -
//    the slice of the joined rows, the NCHW -> NHWC copy and the LeakyReLU
//    in one pass (torch: a transposing copy + leaky_relu);
//  join_to_cl (backward): dy[b][c][j] = lrelu'(out) * g[b][f][t][c] at the
//    row's output columns, 0 at its pad columns - the joined-row gradient
//    the conv's backward reads (torch: leaky_relu_backward + the slice
//    gradient's zero fill + a transposing copy);
//  bias_lrelu (forward): out = lrelu(y + b) on an NHWC tensor - MIOpen's
//    conv then runs without bias;
//  bias_lrelu (backward): dy = lrelu'(out) * g and db[c] = sum of dy over
//    (b, h, w) in one pass (torch: leaky_relu_backward + the conv bias
//    gradient's reduction and memsets).  db is summed in fp32 per workgroup,
//    the workgroup partials added in workgroup order by a one-workgroup
//    launch (deterministic), and rounded through fp16 as the reference's
//    fp16 bias gradient is (autocast casts the bias to fp16 for the conv).
//
// Arithmetic: every value is rounded to the 16-bit type where torch's
// autocast ops round it (conv output, + bias, leaky_relu; slope * x in fp32).
#include <type_traits>

#include "common.h"

namespace {

__device__ __forceinline__ float lrelu_f(float v, float slope) {
  return v < 0.f ? v * slope : v;
}

// ---- join_to_cl ----------------------------------------------------------
// grid (ceil(NT / 64), B), 256 threads; a workgroup moves 64 consecutive
// output rows n = f*T + t of one utterance through an LDS tile [C][64 + 2].
constexpr int JT = 64;
constexpr int JP = JT + 2;

template <typename E>
__global__ __launch_bounds__(256) void join_to_cl_fwd_kernel(
    const E* __restrict__ y, E* __restrict__ out, int C, int F_out, int L, int p1, int T,
    float slope) {
  extern __shared__ char smem_raw[];
  E* tile = reinterpret_cast<E*>(smem_raw);  // [C][JP]
  const int NT = F_out * T;
  const int n0 = blockIdx.x * JT;
  const int b = blockIdx.y;
  const int tid = threadIdx.x;
  const int64_t FL = (int64_t)F_out * L;
  {
    const int tx = tid & 63;
    const int n = n0 + tx;
    const bool ok = n < NT;
    const int f = ok ? n / T : 0;
    const int64_t col = (int64_t)f * L + p1 + (n - f * T);
    const E* yb = y + (int64_t)b * C * FL + col;
    for (int c = tid >> 6; c < C; c += 4) tile[c * JP + tx] = ok ? yb[(int64_t)c * FL] : (E)0.f;
  }
  __syncthreads();
  const int CG = C >> 3;  // 8-channel groups per row
  typedef E e8 __attribute__((ext_vector_type(8)));
  for (int e = tid; e < JT * CG; e += 256) {
    const int r = e / CG;
    const int cg = e - r * CG;
    const int n = n0 + r;
    if (n >= NT) continue;
    e8 v;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (E)lrelu_f((float)tile[(8 * cg + i) * JP + r], slope);
    *reinterpret_cast<e8*>(out + ((int64_t)b * NT + n) * C + 8 * cg) = v;
  }
}

// grid (ceil(F_out * L / 64), B): a workgroup writes 64 consecutive joined
// columns j of dy for every channel.
template <typename E>
__global__ __launch_bounds__(256) void join_to_cl_bwd_kernel(
    const E* __restrict__ g, const E* __restrict__ out, E* __restrict__ dy, int C, int F_out,
    int L, int p1, int T, float slope) {
  extern __shared__ char smem_raw[];
  E* tile = reinterpret_cast<E*>(smem_raw);  // [C][JP]
  const int NT = F_out * T;
  const int FL = F_out * L;
  const int j0 = blockIdx.x * JT;
  const int b = blockIdx.y;
  const int tid = threadIdx.x;
  const int CG = C >> 3;
  typedef E e8 __attribute__((ext_vector_type(8)));
  for (int e = tid; e < JT * CG; e += 256) {
    const int r = e / CG;
    const int cg = e - r * CG;
    const int j = j0 + r;
    const int f = j / L;
    const int t = j - f * L - p1;
    e8 v;
    if (j < FL && t >= 0 && t < T) {
      const int64_t off = ((int64_t)b * NT + f * T + t) * C + 8 * cg;
      const e8 gv = *reinterpret_cast<const e8*>(g + off);
      const e8 ov = *reinterpret_cast<const e8*>(out + off);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float gg = (float)gv[i];
        v[i] = (E)((float)ov[i] > 0.f ? gg : gg * slope);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = (E)0.f;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) tile[(8 * cg + i) * JP + r] = v[i];
  }
  __syncthreads();
  const int tx = tid & 63;
  const int j = j0 + tx;
  if (j < FL) {
    E* db = dy + (int64_t)b * C * FL + j;
    for (int c = tid >> 6; c < C; c += 4) db[(int64_t)c * FL] = tile[c * JP + tx];
  }
}

// ---- bias_lrelu ----------------------------------------------------------
// NHWC rows of C channels; a thread owns one 8-channel group of a row.
template <typename E>
__global__ __launch_bounds__(256) void bias_lrelu_fwd_kernel(
    const E* __restrict__ y, const float* __restrict__ bias, E* __restrict__ out, int C,
    int64_t n8, float slope) {
  typedef E e8 __attribute__((ext_vector_type(8)));
  const int CG = C >> 3;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n8;
       e += (int64_t)gridDim.x * 256) {
    const int cg = (int)(e % CG);
    const e8 v = reinterpret_cast<const e8*>(y)[e];
    e8 o;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      // conv output (fp16) + the fp16-cast bias, rounded; then the activation
      const float s = (float)(E)((float)v[i] + (float)(E)bias[8 * cg + i]);
      o[i] = (E)lrelu_f(s, slope);
    }
    reinterpret_cast<e8*>(out)[e] = o;
  }
}

// Column sums of a [nrows][C] fp32 block (nrows <= 16 * 256 / C * 8 ...):
// thread (w0, c4) adds rows w0, w0 + P4, ... of column quad c4 (coalesced
// across the workgroup), then the P4 row sums of each channel are added in
// order in LDS.  Fixed order: deterministic.  Returns via dst[c] (c < C).
__device__ void column_sums(const float* src, int nrows, int C, float* red, float* dst,
                            bool round16_f16, bool round16_bf16) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  f4* red4 = reinterpret_cast<f4*>(red);
  const int tid = threadIdx.x;
  const int C4 = C >> 2;
  const int P4 = 256 / C4;
  const int c4 = tid % C4;
  const int w0 = tid / C4;
  f4 s4 = {0.f, 0.f, 0.f, 0.f};
  const f4* p4 = reinterpret_cast<const f4*>(src);
#pragma unroll 4
  for (int w = w0; w < nrows; w += P4) s4 += p4[(int64_t)w * C4 + c4];
  __syncthreads();
  red4[tid] = s4;
  __syncthreads();
  for (int c = tid; c < C; c += 256) {
    const int q = c >> 2, i = c & 3;
    float s = 0.f;
    for (int p = 0; p < P4; ++p) s += red4[p * C4 + q][i];
    if (round16_f16) s = (float)(_Float16)s;
    if (round16_bf16) s = (float)(__bf16)s;
    dst[c] = s;
  }
}

// grid NB workgroups: workgroup w writes dy for its rows and their column
// sums to partial[w][C] (fp32); bias_lrelu_db_kernel then adds the NB
// partials in workgroup order (deterministic).  (A last-workgroup ticket in
// this kernel needs device-scope fences, i.e. an L2 write-back per
// workgroup on gfx950: measured 23-61 us per launch against ~8 us.)
template <typename E>
__global__ __launch_bounds__(256) void bias_lrelu_bwd_kernel(
    const E* __restrict__ g, const E* __restrict__ out, E* __restrict__ dy,
    float* __restrict__ partial, int C, int64_t rows, float slope) {
  typedef E e8 __attribute__((ext_vector_type(8)));
  __shared__ float red[256 * 8];
  const int tid = threadIdx.x;
  const int CG = C >> 3;            // divides 256 (host check)
  const int RPI = 256 / CG;         // rows per workgroup iteration
  const int cg = tid % CG;
  const int rl = tid / CG;
  const int nb = gridDim.x;
  float acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = 0.f;
  const int64_t per = (rows + nb - 1) / nb;
  const int64_t r0 = (int64_t)blockIdx.x * per;
  const int64_t r1 = r0 + per < rows ? r0 + per : rows;
  for (int64_t r = r0 + rl; r < r1; r += 2 * RPI) {
    e8 gv[2], ov[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int64_t rr = r + u * RPI;
      if (rr < r1) {
        gv[u] = *reinterpret_cast<const e8*>(g + rr * C + 8 * cg);
        ov[u] = *reinterpret_cast<const e8*>(out + rr * C + 8 * cg);
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int64_t rr = r + u * RPI;
      if (rr < r1) {
        e8 d;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float gg = (float)gv[u][i];
          d[i] = (E)((float)ov[u][i] > 0.f ? gg : gg * slope);
          acc[i] += (float)d[i];
        }
        *reinterpret_cast<e8*>(dy + rr * C + 8 * cg) = d;
      }
    }
  }
  if (!partial) return;  // (data gradient only: no bias gradient wanted)
#pragma unroll
  for (int i = 0; i < 8; ++i) red[tid * 8 + i] = acc[i];
  __syncthreads();
  // channel c = 8 cg + i: sum over the RPI threads of group cg
  for (int c = tid; c < C; c += 256) {
    const int gq = c >> 3, i = c & 7;
    float s = 0.f;
    for (int q = 0; q < RPI; ++q) s += red[(q * CG + gq) * 8 + i];
    partial[(int64_t)blockIdx.x * C + c] = s;
  }
}

// one workgroup: db[c] = fp16-rounded sum over w of partial[w][c], in order
template <typename E>
__global__ __launch_bounds__(256) void bias_lrelu_db_kernel(const float* __restrict__ partial,
                                                            float* __restrict__ db, int C,
                                                            int nb) {
  __shared__ float red[256 * 4];
  column_sums(partial, nb, C, red, db, std::is_same<E, _Float16>::value,
              !std::is_same<E, _Float16>::value);
}

int grid_for(int64_t n) {
  const int64_t want = (n + 255) / 256;
  return (int)(want < 4096 ? want : 4096);
}

}  // namespace

extern "C" int vits_stftd_join_to_cl_forward(const void* y, void* out, int batch, int C,
                                             int F_out, int L, int p1, int T, float slope,
                                             int wdtype, void* stream) {
  VITS_CHECK_ARG(y && out && batch > 0 && C > 0 && C % 8 == 0 && C <= 512 && F_out > 0);
  VITS_CHECK_ARG(T > 0 && p1 >= 0 && L >= T + p1);
  VITS_CHECK_ARG(wdtype == VITS_WDT_F16 || wdtype == VITS_WDT_BF16);
  const dim3 grid((F_out * T + JT - 1) / JT, batch);
  const size_t lds = (size_t)C * JP * 2;
  hipStream_t s = as_stream(stream);
  if (wdtype == VITS_WDT_F16)
    hipLaunchKernelGGL(join_to_cl_fwd_kernel<_Float16>, grid, dim3(256), lds, s,
                       (const _Float16*)y, (_Float16*)out, C, F_out, L, p1, T, slope);
  else
    hipLaunchKernelGGL(join_to_cl_fwd_kernel<__bf16>, grid, dim3(256), lds, s,
                       (const __bf16*)y, (__bf16*)out, C, F_out, L, p1, T, slope);
  return vits_launch_status();
}

extern "C" int vits_stftd_join_to_cl_backward(const void* g, const void* out, void* dy, int batch,
                                              int C, int F_out, int L, int p1, int T,
                                              float slope, int wdtype, void* stream) {
  VITS_CHECK_ARG(g && out && dy && batch > 0 && C > 0 && C % 8 == 0 && C <= 512 && F_out > 0);
  VITS_CHECK_ARG(T > 0 && p1 >= 0 && L >= T + p1);
  VITS_CHECK_ARG(wdtype == VITS_WDT_F16 || wdtype == VITS_WDT_BF16);
  const dim3 grid((F_out * L + JT - 1) / JT, batch);
  const size_t lds = (size_t)C * JP * 2;
  hipStream_t s = as_stream(stream);
  if (wdtype == VITS_WDT_F16)
    hipLaunchKernelGGL(join_to_cl_bwd_kernel<_Float16>, grid, dim3(256), lds, s,
                       (const _Float16*)g, (const _Float16*)out, (_Float16*)dy, C, F_out, L, p1,
                       T, slope);
  else
    hipLaunchKernelGGL(join_to_cl_bwd_kernel<__bf16>, grid, dim3(256), lds, s,
                       (const __bf16*)g, (const __bf16*)out, (__bf16*)dy, C, F_out, L, p1, T,
                       slope);
  return vits_launch_status();
}

extern "C" int vits_bias_lrelu_forward(const void* y, const float* bias, void* out, int64_t rows,
                                       int C, float slope, int wdtype, void* stream) {
  VITS_CHECK_ARG(y && bias && out && rows > 0 && C > 0 && C % 8 == 0);
  VITS_CHECK_ARG(wdtype == VITS_WDT_F16 || wdtype == VITS_WDT_BF16);
  const int64_t n8 = rows * (C / 8);
  hipStream_t s = as_stream(stream);
  if (wdtype == VITS_WDT_F16)
    hipLaunchKernelGGL(bias_lrelu_fwd_kernel<_Float16>, dim3(grid_for(n8)), dim3(256), 0, s,
                       (const _Float16*)y, bias, (_Float16*)out, C, n8, slope);
  else
    hipLaunchKernelGGL(bias_lrelu_fwd_kernel<__bf16>, dim3(grid_for(n8)), dim3(256), 0, s,
                       (const __bf16*)y, bias, (__bf16*)out, C, n8, slope);
  return vits_launch_status();
}

extern "C" int vits_bias_lrelu_workspace(int64_t rows, int C) {
  // the backward's workgroups (each reduces >= 64 rows, at most 512) times
  // C: floats of their partial sums
  if (rows <= 0 || C <= 0) return 0;
  int64_t nb = (rows + 63) / 64;
  if (nb > 512) nb = 512;
  return (int)(nb * C);
}

extern "C" int vits_bias_lrelu_backward(const void* g, const void* out, void* dy, float* db,
                                        float* workspace, int ws_floats, int64_t rows, int C,
                                        float slope, int wdtype, void* stream) {
  VITS_CHECK_ARG(g && out && dy && rows > 0 && C > 0 && (!db || workspace));
  VITS_CHECK_ARG(C % 8 == 0 && 256 % (C / 8) == 0 && C <= 512);
  VITS_CHECK_ARG(wdtype == VITS_WDT_F16 || wdtype == VITS_WDT_BF16);
  const int need = vits_bias_lrelu_workspace(rows, C);
  VITS_CHECK_ARG(!db || ws_floats >= need);
  const int nb = need / C;
  if (!db) workspace = nullptr;  // db NULL: the data gradient only, one launch
  hipStream_t s = as_stream(stream);
  if (wdtype == VITS_WDT_F16) {
    hipLaunchKernelGGL(bias_lrelu_bwd_kernel<_Float16>, dim3(nb), dim3(256), 0, s,
                       (const _Float16*)g, (const _Float16*)out, (_Float16*)dy, workspace, C,
                       rows, slope);
    if (db)
      hipLaunchKernelGGL(bias_lrelu_db_kernel<_Float16>, dim3(1), dim3(256), 0, s, workspace, db,
                         C, nb);
  } else {
    hipLaunchKernelGGL(bias_lrelu_bwd_kernel<__bf16>, dim3(nb), dim3(256), 0, s,
                       (const __bf16*)g, (const __bf16*)out, (__bf16*)dy, workspace, C, rows,
                       slope);
    if (db)
      hipLaunchKernelGGL(bias_lrelu_db_kernel<__bf16>, dim3(1), dim3(256), 0, s, workspace, db,
                         C, nb);
  }
  return vits_launch_status();
}
