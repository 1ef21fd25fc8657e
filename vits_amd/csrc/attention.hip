// attention.hip — scaled-dot-product attention of attentions.MultiHeadAttention
// (attentions.py:85-100) on gfx950 fp32 MFMA, flash-style (online softmax).
//
// q/k/v arrive channel-major [B][H*D][T] straight from the 1x1 projection
// convs (attentions.py:79-81), so no transpose is ever materialised:
//   S^T[key][query] = K[key][:] . Q[query][:]       (v_mfma_f32_32x32x2_f32)
// with the key on the accumulator ROW and the query on the lane: the softmax
// over keys is then an in-register reduction plus one xor-32 shuffle per
// query, and the accumulator registers are directly the B operand of
//   O^T[d][query] += V^T[d][key] . P^T[key][query]
// (k-step r of that product takes key (r&3)+8(r>>2)+4*(lane>>5), which is
// exactly the row register r holds in each half-wave).
//
// One wave = one (utterance, head, 32-query tile).  Mask semantics follow
// attentions.py:94-95: scores.masked_fill(mask == 0, -1e4) with
// mask = x_mask[q] * x_mask[k]; keys beyond T (tile padding) are excluded
// (-inf), so a fully-masked query row averages all T keys exactly like the
// reference softmax over the padded row.
#include "common.h"

namespace {

constexpr int AT_Q = 32;
constexpr int AT_K = 32;

template <int D>
__global__ __launch_bounds__(64) void attn_fwd_kernel(const float* __restrict__ q,
                                                      const float* __restrict__ k,
                                                      const float* __restrict__ v,
                                                      float* __restrict__ out, int H, int T,
                                                      int64_t bstride, int64_t out_bstride,
                                                      const int32_t* __restrict__ lengths) {
  static_assert(D % 16 == 0, "head dim multiple of 16");
  constexpr int KS = D / 2;          // k-steps of the QK product
  constexpr int DT = (D + 31) / 32;  // d tiles of the PV product (last one partial for D%32)
  const int lane = threadIdx.x;
  const int l32 = lane & 31;
  const int lhi = lane >> 5;
  const int q0 = blockIdx.x * AT_Q;
  const int h = blockIdx.y;
  const int b = blockIdx.z;
  const int len = lengths ? lengths[b] : T;
  const int64_t hoff = (int64_t)b * bstride + (int64_t)h * D * T;
  const float* qb = q + hoff;
  const float* kb = k + hoff;
  const float* vb = v + hoff;
  const float scale_div = sqrtf((float)D);

  // Q^T fragment (B operand): lane holds Q[query q0+l32][d = 2s + lhi] / sqrt(D)
  const int qi = q0 + l32;
  const bool qvalid = qi < T;
  float qf[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) qf[s] = qvalid ? qb[(int64_t)(2 * s + lhi) * T + qi] / scale_div : 0.f;
  const bool qmasked = qi >= len;

  f32x16 o[DT];
#pragma unroll
  for (int t = 0; t < DT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[t][r] = 0.f;
  float m_run = -INFINITY;
  float l_run = 0.f;

  for (int k0 = 0; k0 < T; k0 += AT_K) {
    // S^T tile: rows = keys k0 + row, cols = queries
    f32x16 s;
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] = 0.f;
    const int kr = k0 + l32;  // A operand row (key) of this lane
    const bool kvalid = kr < T;
#pragma unroll
    for (int st = 0; st < KS; ++st) {
      const float a = kvalid ? kb[(int64_t)(2 * st + lhi) * T + kr] : 0.f;
      s = __builtin_amdgcn_mfma_f32_32x32x2f32(a, qf[st], s, 0, 0, 0);
    }
    // mask + online softmax over the key rows of this lane's query column
    float mloc = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = k0 + (r & 3) + 8 * (r >> 2) + 4 * lhi;
      float sv = s[r];
      if (key >= T)
        sv = -INFINITY;
      else if (qmasked || key >= len)
        sv = -1e4f;
      s[r] = sv;
      mloc = fmaxf(mloc, sv);
    }
    mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
    const float m_new = fmaxf(m_run, mloc);
    const float alpha = (m_run == -INFINITY) ? 0.f : expf(m_run - m_new);
    float psum = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float p = (s[r] == -INFINITY) ? 0.f : expf(s[r] - m_new);
      s[r] = p;
      psum += p;
    }
    psum += __shfl_xor(psum, 32, 64);
    l_run = l_run * alpha + psum;
    m_run = m_new;
#pragma unroll
    for (int t = 0; t < DT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[t][r] *= alpha;
    // O^T[d][query] += V^T[d][key] P^T[key][query]
#pragma unroll
    for (int t = 0; t < DT; ++t) {
      const bool dvalid = (D % 32 == 0) || (t * 32 + l32 < D);
      const float* vr = vb + (int64_t)(t * 32 + l32) * T + k0 + 4 * lhi;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int kk = (r & 3) + 8 * (r >> 2);
        const float a = (dvalid && k0 + kk + 4 * lhi < T) ? vr[kk] : 0.f;
        o[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, s[r], o[t], 0, 0, 0);
      }
    }
  }
  // epilogue: O^T rows = d, cols = query (this lane)
  if (!qvalid) return;
  const float inv = 1.0f / l_run;
  float* ob = out + (int64_t)b * out_bstride + (int64_t)h * D * T;
#pragma unroll
  for (int t = 0; t < DT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int d = t * 32 + (r & 3) + 8 * (r >> 2) + 4 * lhi;
      if (D % 32 == 0 || d < D) ob[(int64_t)d * T + qi] = o[t][r] * inv;
    }
}

}  // namespace

extern "C" int vits_attention_forward(const float* q, const float* k, const float* v, float* out,
                                      int batch, int heads, int head_dim, int t_len,
                                      int64_t bstride, int64_t out_bstride,
                                      const int32_t* lengths, void* stream) {
  VITS_CHECK_ARG(q && k && v && out && batch > 0 && heads > 0 && t_len > 0);
  VITS_CHECK_SHAPE(bstride >= (int64_t)heads * head_dim * t_len);
  VITS_CHECK_SHAPE(out_bstride >= (int64_t)heads * head_dim * t_len);
  dim3 grid((t_len + AT_Q - 1) / AT_Q, heads, batch);
  hipStream_t s = as_stream(stream);
  switch (head_dim) {
#define VITS_ATTN_CASE(D)                                                                      \
    case D:                                                                                    \
      hipLaunchKernelGGL(attn_fwd_kernel<D>, grid, dim3(64), 0, s, q, k, v, out, heads, t_len, \
                         bstride, out_bstride, lengths);                                       \
      break;
    VITS_ATTN_CASE(16)
    VITS_ATTN_CASE(32)
    VITS_ATTN_CASE(48)
#undef VITS_ATTN_CASE
    case 64:
      hipLaunchKernelGGL(attn_fwd_kernel<64>, grid, dim3(64), 0, s, q, k, v, out, heads, t_len,
                         bstride, out_bstride, lengths);
      break;
    case 128:
      hipLaunchKernelGGL(attn_fwd_kernel<128>, grid, dim3(64), 0, s, q, k, v, out, heads, t_len,
                         bstride, out_bstride, lengths);
      break;
    case 96:
      hipLaunchKernelGGL(attn_fwd_kernel<96>, grid, dim3(64), 0, s, q, k, v, out, heads, t_len,
                         bstride, out_bstride, lengths);
      break;
    default:
      return VITS_E_UNSUP;
  }
  return vits_launch_status();
}
