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

// ---------------------------------------------------------------------------
// Training attention (attentions.py:85-100 under autograd, p_dropout > 0):
// forward + backward, fp32 MFMA on fp16 / fp32 q, k, v (the 1x1 projection
// convs' outputs), flash-style: the forward keeps only O and the per-query
// log-sum-exp; the backward recomputes P.  Dropout: keep[b][h][q][key]
// (uint8, drawn by the caller) scales the probabilities that multiply V by
// keep * keep_scale (keep_scale = 1 / (1 - p)), as nn.Dropout does to
// p_attn; the softmax normaliser itself is dropout-free.  With
//   S = Q K^T / sqrt(D) (masked_fill(mask == 0, -1e4)), P = softmax(S),
//   Pd = P o M (M = keep * keep_scale), O = Pd V,
// the gradients are dV = Pd^T dO, dP = (dO V^T) o M,
//   dS = P o (dP - delta), delta_q = sum_d dO[q][d] O[q][d]
// (= rowsum(P o dP)), dS = 0 where the mask filled the score,
//   dQ = dS K / sqrt(D), dK = dS^T Q / sqrt(D).
// Kernel A (one wave per 32-query tile): delta, dQ - the accumulator holds
// S^T[key][query] as in attn_fwd_kernel (keys on registers, queries on
// lanes).  Kernel B (one wave per 32-key tile): dK, dV - the accumulator
// holds S[query][key] (queries on registers, keys on lanes), so P / dS are
// directly the B operand of the products that sum over queries.
// ---------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ float ldf(const T* p, int64_t i) {
  return (float)p[i];
}

template <int D, typename T>
__global__ __launch_bounds__(64) void attn_train_fwd_kernel(
    const T* __restrict__ q, const T* __restrict__ k, const T* __restrict__ v,
    const uint8_t* __restrict__ keep, float keep_scale, T* __restrict__ out,
    float* __restrict__ lse, int H, int Tn, const int32_t* __restrict__ lengths) {
  constexpr int KS = D / 2;
  constexpr int DT = D / 32;
  const int lane = threadIdx.x;
  const int l32 = lane & 31;
  const int lhi = lane >> 5;
  const int q0 = blockIdx.x * AT_Q;
  const int h = blockIdx.y;
  const int b = blockIdx.z;
  const int len = lengths ? lengths[b] : Tn;
  const int64_t hoff = ((int64_t)b * H + h) * D * Tn;
  const T* qb = q + hoff;
  const T* kb = k + hoff;
  const T* vb = v + hoff;
  const float rs = 1.0f / sqrtf((float)D);
  const int qi = q0 + l32;
  const bool qvalid = qi < Tn;
  const bool qmasked = qi >= len;
  const uint8_t* kp = keep ? keep + (((int64_t)b * H + h) * Tn + (qvalid ? qi : 0)) * Tn : nullptr;
  float qf[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) qf[s] = qvalid ? ldf(qb, (int64_t)(2 * s + lhi) * Tn + qi) * rs : 0.f;
  f32x16 o[DT];
#pragma unroll
  for (int t = 0; t < DT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[t][r] = 0.f;
  float m_run = -INFINITY, l_run = 0.f;
  for (int k0 = 0; k0 < Tn; k0 += AT_K) {
    f32x16 s;
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] = 0.f;
    const int kr = k0 + l32;
    const bool kvalid = kr < Tn;
#pragma unroll
    for (int st = 0; st < KS; ++st) {
      const float a = kvalid ? ldf(kb, (int64_t)(2 * st + lhi) * Tn + kr) : 0.f;
      s = __builtin_amdgcn_mfma_f32_32x32x2f32(a, qf[st], s, 0, 0, 0);
    }
    float mloc = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = k0 + (r & 3) + 8 * (r >> 2) + 4 * lhi;
      float sv = s[r];
      if (key >= Tn)
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
      const int key = k0 + (r & 3) + 8 * (r >> 2) + 4 * lhi;
      float p = (s[r] == -INFINITY) ? 0.f : expf(s[r] - m_new);
      psum += p;
      if (kp && key < Tn) p *= kp[key] ? keep_scale : 0.f;
      s[r] = p;
    }
    psum += __shfl_xor(psum, 32, 64);
    l_run = l_run * alpha + psum;
    m_run = m_new;
#pragma unroll
    for (int t = 0; t < DT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[t][r] *= alpha;
#pragma unroll
    for (int t = 0; t < DT; ++t) {
      const T* vr = vb + (int64_t)(t * 32 + l32) * Tn + k0 + 4 * lhi;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int kk = (r & 3) + 8 * (r >> 2);
        const float a = (k0 + kk + 4 * lhi < Tn) ? (float)vr[kk] : 0.f;
        o[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, s[r], o[t], 0, 0, 0);
      }
    }
  }
  if (!qvalid) return;
  const float inv = 1.0f / l_run;
  T* ob = out + hoff;
#pragma unroll
  for (int t = 0; t < DT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int d = t * 32 + (r & 3) + 8 * (r >> 2) + 4 * lhi;
      ob[(int64_t)d * Tn + qi] = (T)(o[t][r] * inv);
    }
  // (m, 1/l) per query, not m + log(l): a fully masked row has m = -1e4 and
  // -1e4 + log(l) is not representable closely enough in fp32 (ulp ~1e-3)
  if (lhi == 0) {
    const int64_t e = ((int64_t)b * H + h) * Tn + qi;
    lse[2 * e] = m_run;
    lse[2 * e + 1] = inv;
  }
}

// kernel A: delta and dQ, one wave per (b, h, 32 queries)
template <int D, typename T>
__global__ __launch_bounds__(64) void attn_train_bwd_dq_kernel(
    const T* __restrict__ q, const T* __restrict__ k, const T* __restrict__ v,
    const T* __restrict__ o, const T* __restrict__ dout, const uint8_t* __restrict__ keep,
    float keep_scale, const float* __restrict__ lse, float* __restrict__ delta,
    T* __restrict__ dq, int H, int Tn, const int32_t* __restrict__ lengths) {
  constexpr int KS = D / 2;
  constexpr int DT = D / 32;
  const int lane = threadIdx.x;
  const int l32 = lane & 31;
  const int lhi = lane >> 5;
  const int q0 = blockIdx.x * AT_Q;
  const int h = blockIdx.y;
  const int b = blockIdx.z;
  const int len = lengths ? lengths[b] : Tn;
  const int64_t hoff = ((int64_t)b * H + h) * D * Tn;
  const int64_t roff = ((int64_t)b * H + h) * Tn;
  const T* qb = q + hoff;
  const T* kb = k + hoff;
  const T* vb = v + hoff;
  const float rs = 1.0f / sqrtf((float)D);
  const int qi = q0 + l32;
  const bool qvalid = qi < Tn;
  const int qc = qvalid ? qi : 0;
  const bool qmasked = qi >= len;
  const uint8_t* kp = keep ? keep + (roff + qc) * Tn : nullptr;
  float qf[KS], df[KS];
  float dl = 0.f;
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int64_t e = (int64_t)(2 * s + lhi) * Tn + qc;
    qf[s] = qvalid ? ldf(qb, e) * rs : 0.f;
    const float g = qvalid ? ldf(dout + hoff, e) : 0.f;
    df[s] = g;
    dl += qvalid ? g * ldf(o + hoff, e) : 0.f;
  }
  dl += __shfl_xor(dl, 32, 64);
  if (qvalid && lhi == 0) delta[roff + qi] = dl;
  const float mq = qvalid ? lse[2 * (roff + qi)] : 0.f;
  const float iq = qvalid ? lse[2 * (roff + qi) + 1] : 0.f;
  f32x16 acc[DT];
#pragma unroll
  for (int t = 0; t < DT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  for (int k0 = 0; k0 < Tn; k0 += AT_K) {
    f32x16 s, dp;
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] = dp[r] = 0.f;
    const int kr = k0 + l32;
    const bool kvalid = kr < Tn;
#pragma unroll
    for (int st = 0; st < KS; ++st) {
      const int64_t e = (int64_t)(2 * st + lhi) * Tn + kr;
      const float a = kvalid ? ldf(kb, e) : 0.f;
      const float c = kvalid ? ldf(vb, e) : 0.f;
      s = __builtin_amdgcn_mfma_f32_32x32x2f32(a, qf[st], s, 0, 0, 0);
      dp = __builtin_amdgcn_mfma_f32_32x32x2f32(c, df[st], dp, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = k0 + (r & 3) + 8 * (r >> 2) + 4 * lhi;
      float ds = 0.f;
      if (key < Tn && qvalid) {
        const bool filled = qmasked || key >= len;
        const float p = expf((filled ? -1e4f : s[r]) - mq) * iq;
        const float m = kp ? (kp[key] ? keep_scale : 0.f) : 1.f;
        ds = filled ? 0.f : p * (dp[r] * m - dl);
      }
      s[r] = ds;
    }
    // dQ^T[d][q] += K^T[d][key] dS^T[key][q]
#pragma unroll
    for (int t = 0; t < DT; ++t) {
      const T* kr2 = kb + (int64_t)(t * 32 + l32) * Tn + k0 + 4 * lhi;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int kk = (r & 3) + 8 * (r >> 2);
        const float a = (k0 + kk + 4 * lhi < Tn) ? (float)kr2[kk] : 0.f;
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, s[r], acc[t], 0, 0, 0);
      }
    }
  }
  if (!qvalid) return;
  T* db = dq + hoff;
#pragma unroll
  for (int t = 0; t < DT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int d = t * 32 + (r & 3) + 8 * (r >> 2) + 4 * lhi;
      db[(int64_t)d * Tn + qi] = (T)(acc[t][r] * rs);
    }
}

// kernel B: dK and dV, one wave per (b, h, 32 keys); delta from kernel A
template <int D, typename T>
__global__ __launch_bounds__(64) void attn_train_bwd_dkv_kernel(
    const T* __restrict__ q, const T* __restrict__ k, const T* __restrict__ v,
    const T* __restrict__ dout, const uint8_t* __restrict__ keep, float keep_scale,
    const float* __restrict__ lse, const float* __restrict__ delta, T* __restrict__ dk,
    T* __restrict__ dv, int H, int Tn, const int32_t* __restrict__ lengths) {
  constexpr int KS = D / 2;
  constexpr int DT = D / 32;
  const int lane = threadIdx.x;
  const int l32 = lane & 31;
  const int lhi = lane >> 5;
  const int k0 = blockIdx.x * AT_K;
  const int h = blockIdx.y;
  const int b = blockIdx.z;
  const int len = lengths ? lengths[b] : Tn;
  const int64_t hoff = ((int64_t)b * H + h) * D * Tn;
  const int64_t roff = ((int64_t)b * H + h) * Tn;
  const T* qb = q + hoff;
  const T* kb = k + hoff;
  const T* vb = v + hoff;
  const T* gb = dout + hoff;
  const float rs = 1.0f / sqrtf((float)D);
  const int ki = k0 + l32;  // this lane's key (B operand column)
  const bool kvalid = ki < Tn;
  const int kc = kvalid ? ki : 0;
  float kf[KS], vf[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int64_t e = (int64_t)(2 * s + lhi) * Tn + kc;
    kf[s] = kvalid ? ldf(kb, e) * rs : 0.f;
    vf[s] = kvalid ? ldf(vb, e) : 0.f;
  }
  f32x16 adk[DT], adv[DT];
#pragma unroll
  for (int t = 0; t < DT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) adk[t][r] = adv[t][r] = 0.f;
  for (int q0 = 0; q0 < Tn; q0 += AT_Q) {
    f32x16 s, dp;
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] = dp[r] = 0.f;
    const int qr = q0 + l32;  // A operand row (query) of this lane
    const bool qrv = qr < Tn;
#pragma unroll
    for (int st = 0; st < KS; ++st) {
      const int64_t e = (int64_t)(2 * st + lhi) * Tn + qr;
      const float a = qrv ? ldf(qb, e) : 0.f;
      const float c = qrv ? ldf(gb, e) : 0.f;
      s = __builtin_amdgcn_mfma_f32_32x32x2f32(a, kf[st], s, 0, 0, 0);
      dp = __builtin_amdgcn_mfma_f32_32x32x2f32(c, vf[st], dp, 0, 0, 0);
    }
    f32x16 pd;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int qq = q0 + (r & 3) + 8 * (r >> 2) + 4 * lhi;
      float ds = 0.f, pv = 0.f;
      if (qq < Tn && kvalid) {
        const bool filled = qq >= len || ki >= len;
        const float p = expf((filled ? -1e4f : s[r]) - lse[2 * (roff + qq)]) *
                        lse[2 * (roff + qq) + 1];
        const float m = keep ? (keep[(roff + qq) * Tn + ki] ? keep_scale : 0.f) : 1.f;
        pv = p * m;
        ds = filled ? 0.f : p * (dp[r] * m - delta[roff + qq]);
      }
      pd[r] = pv;
      s[r] = ds;
    }
    // dV^T[d][key] += dO^T[d][q] Pd[q][key]; dK^T[d][key] += Q^T[d][q] dS[q][key]
#pragma unroll
    for (int t = 0; t < DT; ++t) {
      const int64_t rowo = (int64_t)(t * 32 + l32) * Tn + q0 + 4 * lhi;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int kk = (r & 3) + 8 * (r >> 2);
        const bool ok = q0 + kk + 4 * lhi < Tn;
        const float go = ok ? (float)gb[rowo + kk] : 0.f;
        const float qa = ok ? (float)qb[rowo + kk] : 0.f;
        adv[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(go, pd[r], adv[t], 0, 0, 0);
        adk[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(qa, s[r], adk[t], 0, 0, 0);
      }
    }
  }
  if (!kvalid) return;
#pragma unroll
  for (int t = 0; t < DT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int d = t * 32 + (r & 3) + 8 * (r >> 2) + 4 * lhi;
      dk[hoff + (int64_t)d * Tn + ki] = (T)(adk[t][r] * rs);
      dv[hoff + (int64_t)d * Tn + ki] = (T)adv[t][r];
    }
}

template <int D, typename T>
int attn_train_fwd_launch(const void* q, const void* k, const void* v, const uint8_t* keep,
                          float keep_scale, void* out, float* lse, int B, int H, int Tn,
                          const int32_t* lengths, hipStream_t s) {
  dim3 grid((Tn + AT_Q - 1) / AT_Q, H, B);
  hipLaunchKernelGGL((attn_train_fwd_kernel<D, T>), grid, dim3(64), 0, s,
                     static_cast<const T*>(q), static_cast<const T*>(k), static_cast<const T*>(v),
                     keep, keep_scale, static_cast<T*>(out), lse, H, Tn, lengths);
  return vits_launch_status();
}

template <int D, typename T>
int attn_train_bwd_launch(const void* q, const void* k, const void* v, const void* o,
                          const void* dout, const uint8_t* keep, float keep_scale,
                          const float* lse, float* delta, void* dq, void* dk, void* dv, int B,
                          int H, int Tn, const int32_t* lengths, hipStream_t s) {
  dim3 grid((Tn + AT_Q - 1) / AT_Q, H, B);
  hipLaunchKernelGGL((attn_train_bwd_dq_kernel<D, T>), grid, dim3(64), 0, s,
                     static_cast<const T*>(q), static_cast<const T*>(k), static_cast<const T*>(v),
                     static_cast<const T*>(o), static_cast<const T*>(dout), keep, keep_scale, lse,
                     delta, static_cast<T*>(dq), H, Tn, lengths);
  int rc = vits_launch_status();
  if (rc) return rc;
  hipLaunchKernelGGL((attn_train_bwd_dkv_kernel<D, T>), grid, dim3(64), 0, s,
                     static_cast<const T*>(q), static_cast<const T*>(k), static_cast<const T*>(v),
                     static_cast<const T*>(dout), keep, keep_scale, lse, delta,
                     static_cast<T*>(dk), static_cast<T*>(dv), H, Tn, lengths);
  return vits_launch_status();
}

}  // namespace

extern "C" int vits_attention_train_forward(const void* q, const void* k, const void* v,
                                            const uint8_t* keep, float keep_scale, void* out,
                                            float* lse, int batch, int heads, int head_dim,
                                            int t_len, const int32_t* lengths, int dtype,
                                            void* stream) {
  VITS_CHECK_ARG(q && k && v && out && lse && batch > 0 && heads > 0 && t_len > 0);
  VITS_CHECK_ARG(dtype == VITS_WDT_F32 || dtype == VITS_WDT_F16);
  hipStream_t s = as_stream(stream);
#define VITS_ATT_T(D)                                                                              if (head_dim == D)                                                                                 return dtype == VITS_WDT_F16                                                                                ? attn_train_fwd_launch<D, _Float16>(q, k, v, keep, keep_scale, out, lse, batch,                                                      heads, t_len, lengths, s)                                   : attn_train_fwd_launch<D, float>(q, k, v, keep, keep_scale, out, lse, batch,                                                      heads, t_len, lengths, s);
  VITS_ATT_T(32)
  VITS_ATT_T(64)
  VITS_ATT_T(96)
  VITS_ATT_T(128)
#undef VITS_ATT_T
  return VITS_E_UNSUP;
}

extern "C" int vits_attention_train_backward(const void* q, const void* k, const void* v,
                                             const void* out, const void* dout,
                                             const uint8_t* keep, float keep_scale,
                                             const float* lse, float* delta, void* dq, void* dk,
                                             void* dv, int batch, int heads, int head_dim,
                                             int t_len, const int32_t* lengths, int dtype,
                                             void* stream) {
  VITS_CHECK_ARG(q && k && v && out && dout && lse && delta && dq && dk && dv);
  VITS_CHECK_ARG(batch > 0 && heads > 0 && t_len > 0);
  VITS_CHECK_ARG(dtype == VITS_WDT_F32 || dtype == VITS_WDT_F16);
  hipStream_t s = as_stream(stream);
#define VITS_ATT_T(D)                                                                              if (head_dim == D)                                                                                 return dtype == VITS_WDT_F16                                                                                ? attn_train_bwd_launch<D, _Float16>(q, k, v, out, dout, keep, keep_scale, lse,                                                       delta, dq, dk, dv, batch, heads, t_len,                                                          lengths, s)                                                 : attn_train_bwd_launch<D, float>(q, k, v, out, dout, keep, keep_scale, lse,                                                       delta, dq, dk, dv, batch, heads, t_len,                                                          lengths, s);
  VITS_ATT_T(32)
  VITS_ATT_T(64)
  VITS_ATT_T(96)
  VITS_ATT_T(128)
#undef VITS_ATT_T
  return VITS_E_UNSUP;
}

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
