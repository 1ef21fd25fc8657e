// resblock.hip — one ResBlock2 dilation pair of the HiFi-GAN Generator as
// ONE kernel (fp32 MFMA, v_mfma_f32_32x32x2_f32):
//
//   y = x + c2( tanh(a + sa) * sigmoid(b + sb) ) ,   (a | b) = c1(lrelu(x, 0.1))
//
// (modules.py:250-260: c1 = Conv1d(C, C', k, dil d), c2 = Conv1d(C'/2, C, k,
// dil 1), sa/sb = the per-utterance cond Linear; here C' = C).
//
// The unfused path runs c1 (gate epilogue) -> gated [B][C/2][T] in HBM -> c2
// (residual epilogue): per pair it moves x, g, g, x (residual), y through
// HBM.  Fused, one workgroup owns an output time tile of BN = NG - (k-1)
// columns and all C channels:
//   phase 1: the c1 GEMM (rows = the C' gate-interleaved outputs, NG columns
//            = the tile plus c2's (k-1)/2 halo each side), gate epilogue
//            written to LDS as G[C/2][NG] - zero outside [0, T), which is
//            c2's own zero padding (the halo columns are recomputed by the
//            neighbouring tile, never exchanged);
//   phase 2: the c2 GEMM reading its B operand straight from G (tap j =
//            column shift j), residual / mean epilogue to HBM.
// HBM traffic per pair: x (with halo) in, y out; the residual re-read hits
// the L2 lines phase 1 just staged.
//
// Staging as in conv1d_impl.h: weight chunks [kc][k][C] by LDS-DMA, the x
// window by 16-byte register loads (leaky-relu + zero padding applied on the
// way into LDS), double-buffered, one barrier per K-chunk.  Every launch
// holds up to 3 independent pairs (the three resblock branches of a stage).
#include "common.h"

namespace {

typedef __attribute__((address_space(3))) void* lds_void_t;
typedef float f32x4v __attribute__((ext_vector_type(4)));

constexpr int RB_GROUP = 3;
constexpr int RB_XFLOATS = 4096;  // x window floats per stage (16 per thread)
struct RbGroup {
  vits_resblock_pair_desc d[RB_GROUP];
  int n;
  int batch;
};

__device__ __forceinline__ float rb_sigmoid(float x) {
  return __builtin_amdgcn_rcpf(1.0f + __expf(-x));
}
__device__ __forceinline__ float rb_tanh(float x) {
  return 2.0f * __builtin_amdgcn_rcpf(1.0f + __expf(-2.0f * x)) - 1.0f;
}

// LDS floats of one stage / of the whole kernel (host and device agree)
__host__ __device__ inline int rb_xrs_max(int NG, int k, int dil) {
  return 4 * ((NG + (k - 1) * dil + 3 + 3) >> 2);
}
__host__ __device__ inline int rb_stage_floats(int M, int NG, const vits_resblock_pair_desc& d) {
  const int s1 = d.kc1 * d.k * M + d.kc1 * rb_xrs_max(NG, d.k, d.dil);
  const int s2 = d.kc2 * d.k * M;
  return s1 > s2 ? s1 : s2;
}
__host__ __device__ inline int rb_gs(int NG) { return NG + 12; }
__host__ __device__ inline int rb_lds_floats(int M, int NG, const vits_resblock_pair_desc& d) {
  // erow (2M) + G (M/2 rows) + 2 stages + tail pad (the pipelined LDS reads
  // run one k-step past a chunk)
  return 2 * M + (M / 2) * rb_gs(NG) + 2 * rb_stage_floats(M, NG, d) + 2 * d.k * M +
         2 * rb_xrs_max(NG, d.k, d.dil) + 64;
}

template <int M, int NG, int WAVES_M, int WAVES_N>
__global__ __launch_bounds__(256, 2) void resblock_pair_kernel(const RbGroup G) {
  constexpr int WM = M / WAVES_M;
  constexpr int WN = NG / WAVES_N;
  constexpr int TM = WM / 32;
  constexpr int TN = WN / 32;
  constexpr int H = M / 2;
  constexpr int GS = NG + 12;
  constexpr int NU = RB_XFLOATS / 1024;  // 16-byte staging units per thread
  static_assert(WAVES_M * WAVES_N == 4 && TM >= 1 && TN >= 1, "4 waves, 32x32 sub-tiles");

  const int gi = (int)blockIdx.z / G.batch;
  const vits_resblock_pair_desc& p = G.d[gi];
  const int b = (int)blockIdx.z - gi * G.batch;
  const int k = p.k;
  const int dil = p.dil;
  const int T = p.t_len;
  // valid length of this utterance (masked decoder of the bucketed infer):
  // the gated tensor is zero past it (c2's zero padding at the utterance
  // end) and the outputs there are 0, as the conv kernel's lengths mask
  const int L = p.lengths ? min(T, (int)p.lengths[b]) : T;
  const int p1 = (k - 1) * dil / 2;
  const int p2 = (k - 1) / 2;
  const int BN = NG - 2 * p2;
  const int n0 = blockIdx.x * BN;
  if (n0 >= T) return;
  if (p.lengths && p.len_skip > 0 && n0 >= L + p.len_skip) return;  // bucketed infer

  extern __shared__ float smem[];
  float* const erow = smem;                 // [2M]: phase-1 / phase-2 row constants
  float* const gl = smem + 2 * M;           // G [H][GS]
  float* const stage0 = gl + H * GS;
  const int SS = rb_stage_floats(M, NG, p);
  float* const stage1 = stage0 + SS;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = (wid / WAVES_N) * WM;
  const int wn = (wid % WAVES_N) * WN;
  const int l32 = lane & 31;
  const int lhi = lane >> 5;

  // row constants: c1 bias + cond in the gate-interleaved row order, c2 bias
  const float* cond = p.cond ? p.cond + (int64_t)b * p.cond_bstride : nullptr;
  for (int r = tid; r < 2 * M; r += 256) {
    float e = 0.f;
    if (r < M) {
      const int idx = (r & 1) ? H + (r >> 1) : (r >> 1);
      if (p.b1) e = p.b1[idx];
      if (cond) e += cond[idx];
    } else if (p.b2) {
      e = p.b2[r - M];
    }
    erow[r] = e;
  }

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // ---------------- phase 1: c1 over NG columns starting at n0 - p2 -------
  const int kc1 = p.kc1;
  const int xw = NG + (k - 1) * dil;
  const int tw0 = n0 - p2 - p1;           // first window column's time
  const int xstart = tw0 & ~3;            // floor to a 16-byte block
  const int xsh = tw0 - xstart;
  const int nb = (xw + xsh + 3) >> 2;
  const int xrs = 4 * nb;
  const int wsz1 = kc1 * k * M;
  const float* xb = p.x + (int64_t)b * p.x_bstride;
  const float slope = p.in_slope;
  const int nunits = kc1 * nb;
  f32x4v xreg[NU];
  int xrow[NU], xoff[NU];
#pragma unroll
  for (int q = 0; q < NU; ++q) {
    const int u = tid + q * 256;
    const int r = u / nb;
    const int tt = xstart + 4 * (u - r * nb);
    const bool ok = u < nunits && tt >= 0 && tt < T;
    xrow[q] = ok ? r : (1 << 24);
    xoff[q] = ok ? r * p.x_cstride + tt : 0;
  }
  auto wdma = [&](const float* w, int m_pad, int c0, int wsz, float* st) {
    const float* src = w + (int64_t)c0 * k * m_pad;
    const int pieces = (wsz + 255) >> 8;
    for (int q = wid; q < pieces; q += 4) {
      const int e = q * 256 + lane * 4;
      if (e < wsz) {
        const int r = e / M;
        const int col = e - r * M;
        __builtin_amdgcn_global_load_lds(src + (int64_t)r * m_pad + col,
                                         (lds_void_t)(st + q * 256), 16, 0, 0);
      }
    }
  };
  auto gload = [&](int c0) {
    const float* base = xb + (int64_t)c0 * p.x_cstride;
    const int lim = p.channels - c0;
#pragma unroll
    for (int q = 0; q < NU; ++q) {
      if (q * 256 < nunits) {
        const float* src = xrow[q] < lim ? base + xoff[q] : xb;
        xreg[q] = *reinterpret_cast<const f32x4v*>(src);
      }
    }
  };
  auto lstore = [&](float* st, int c0) {
    float* xs = st + wsz1;
    const int lim = p.channels - c0;
#pragma unroll
    for (int q = 0; q < NU; ++q) {
      if (q * 256 < nunits) {
        const int u = tid + q * 256;
        if (u < nunits) {
          const bool ok = xrow[q] < lim;
          f32x4v v = xreg[q];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float t = v[e] < 0.f ? v[e] * slope : v[e];
            v[e] = ok ? t : 0.f;
          }
          const int r = u / nb;
          *reinterpret_cast<f32x4v*>(xs + r * xrs + 4 * (u - r * nb)) = v;
        }
      }
    }
  };
  // one K-chunk of MFMAs: A rows (2cp + lhi)*k + j of the chunk's weights,
  // B row 2cp + lhi of `xs` (row stride rs) shifted by j*ts
  auto mma_chunk = [&](const float* ws, const float* xs, int rs, int ts, int half) {
    const float* wa = ws + lhi * k * M + wm + l32;
    const float* xa = xs + lhi * rs + wn + l32;
    const int sa = 2 * k * M;
    const int sb = 2 * rs;
    const int steps = k * half;
    int j = 0, cp = 0;
    const float* pa = wa;
    const float* pb = xa;
    auto advance = [&]() {
      ++cp;
      pa += sa;
      pb += sb;
      if (cp == half) {
        cp = 0;
        ++j;
        pa = wa + j * M;
        pb = xa + j * ts;
      }
    };
    float a0[TM], b0[TN], a1[TM], b1[TN];
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) a0[mi] = pa[mi * 32];
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) b0[ni] = pb[ni * 32];
    advance();
    int s = 0;
    for (; s + 2 <= steps; s += 2) {
#pragma unroll
      for (int mi = 0; mi < TM; ++mi) a1[mi] = pa[mi * 32];
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) b1[ni] = pb[ni * 32];
      advance();
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int mi = 0; mi < TM; ++mi)
#pragma unroll
        for (int ni = 0; ni < TN; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[mi], b0[ni], acc[mi][ni], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
#pragma unroll
      for (int mi = 0; mi < TM; ++mi) a0[mi] = pa[mi * 32];
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) b0[ni] = pb[ni * 32];
      advance();
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int mi = 0; mi < TM; ++mi)
#pragma unroll
        for (int ni = 0; ni < TN; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[mi], b1[ni], acc[mi][ni], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    if (s < steps) {
#pragma unroll
      for (int mi = 0; mi < TM; ++mi)
#pragma unroll
        for (int ni = 0; ni < TN; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[mi], b0[ni], acc[mi][ni], 0, 0, 0);
    }
  };

  const int nch1 = p.channels / kc1;
  const int kc2 = p.kc2;
  const int nch2 = H / kc2;
  const int wsz2 = kc2 * k * M;
  wdma(p.w1, p.m_pad1, 0, wsz1, stage0);
  gload(0);
  lstore(stage0, 0);
  __syncthreads();
  for (int ch = 0; ch < nch1; ++ch) {
    float* cur = (ch & 1) ? stage1 : stage0;
    float* nxt = (ch & 1) ? stage0 : stage1;
    const bool more = ch + 1 < nch1;
    if (more) {
      wdma(p.w1, p.m_pad1, (ch + 1) * kc1, wsz1, nxt);
      gload((ch + 1) * kc1);
    } else {
      // phase 2's first weight chunk, under the last phase-1 MFMAs
      wdma(p.w2, p.m_pad2, 0, wsz2, nxt);
    }
    mma_chunk(cur, cur + wsz1 + xsh, xrs, dil, kc1 >> 1);
    if (more) lstore(nxt, (ch + 1) * kc1);
    __syncthreads();
  }

  // gate epilogue -> G (zero outside [0, T): c2's zero padding)
#pragma unroll
  for (int mi = 0; mi < TM; ++mi) {
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) {
      const int col = wn + ni * 32 + l32;
      const int t = n0 - p2 + col;
      const bool in = t >= 0 && t < L;
      const int rloc = wm + mi * 32 + 4 * lhi;
#pragma unroll
      for (int r = 0; r < 16; r += 2) {
        const int row = rloc + (r & 3) + 8 * (r >> 2);
        const float va = acc[mi][ni][r] + erow[row];
        const float vb = acc[mi][ni][r + 1] + erow[row + 1];
        const float v = rb_tanh(va) * rb_sigmoid(vb);
        gl[(row >> 1) * GS + col] = in ? v : 0.f;
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][ni][r] = 0.f;
    }
  }
  for (int i = tid; i < H * (GS - NG); i += 256) {
    const int r = i / (GS - NG);
    gl[r * GS + NG + (i - r * (GS - NG))] = 0.f;
  }
  __syncthreads();

  // ---------------- phase 2: c2 from G -------------------------------------
  int st = nch1;  // stage index of W2 chunk 0
  for (int ch = 0; ch < nch2; ++ch, ++st) {
    float* cur = (st & 1) ? stage1 : stage0;
    float* nxt = (st & 1) ? stage0 : stage1;
    if (ch + 1 < nch2) wdma(p.w2, p.m_pad2, (ch + 1) * kc2, wsz2, nxt);
    mma_chunk(cur, gl + ch * kc2 * GS, GS, 1, kc2 >> 1);
    __syncthreads();
  }

  // residual (+ branch mean) epilogue
  float* yb = p.y + (int64_t)b * p.y_bstride;
  const float* rb = xb;
#pragma unroll
  for (int mi = 0; mi < TM; ++mi) {
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) {
      const int col = wn + ni * 32 + l32;
      const int t = n0 + col;
      if (col < BN && t < T) {
        const int rloc = wm + mi * 32 + 4 * lhi;
        float v[16], rv[16];
#pragma unroll
        for (int r = 0; r < 16; ++r)
          rv[r] = rb[(int64_t)(rloc + (r & 3) + 8 * (r >> 2)) * p.x_cstride + t];
#pragma unroll
        for (int r = 0; r < 16; ++r)
          v[r] = rv[r] + (acc[mi][ni][r] + erow[M + rloc + (r & 3) + 8 * (r >> 2)]);
        if (p.accumulate) {
          float yo[16];
#pragma unroll
          for (int r = 0; r < 16; ++r)
            yo[r] = yb[(int64_t)(rloc + (r & 3) + 8 * (r >> 2)) * p.y_cstride + t];
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] = yo[r] + v[r];
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float o = v[r];
          if (p.post_div != 1.0f) o = o / p.post_div;
          if (t >= L) o = 0.f;
          yb[(int64_t)(rloc + (r & 3) + 8 * (r >> 2)) * p.y_cstride + t] = o;
        }
      }
    }
  }
}

template <int M, int NG, int WM_, int WN_>
int rb_launch(const RbGroup& g, hipStream_t s) {
  int lds = 0, gx = 0;
  for (int i = 0; i < g.n; ++i) {
    const vits_resblock_pair_desc& d = g.d[i];
    const int BN = NG - (d.k - 1);
    if (BN < 32) return VITS_E_UNSUP;
    if (d.kc1 * rb_xrs_max(NG, d.k, d.dil) > RB_XFLOATS) return VITS_E_UNSUP;
    const int l = 4 * rb_lds_floats(M, NG, d);
    if (l > lds) lds = l;
    const int x = (d.t_len + BN - 1) / BN;
    if (x > gx) gx = x;
  }
  if (lds > 160 * 1024) return VITS_E_UNSUP;
  hipLaunchKernelGGL((resblock_pair_kernel<M, NG, WM_, WN_>), dim3(gx, 1, g.n * g.batch),
                     dim3(256), lds, s, g);
  return vits_launch_status();
}

int rb_check(const vits_resblock_pair_desc& d) {
  VITS_CHECK_ARG(d.x && d.w1 && d.w2 && d.y);
  // other workgroups still read x (halos, residual): never write in place
  VITS_CHECK_ARG(reinterpret_cast<const void*>(d.y) != reinterpret_cast<const void*>(d.x));
  VITS_CHECK_SHAPE(d.channels == 32 || d.channels == 64);
  VITS_CHECK_SHAPE(d.k >= 1 && (d.k & 1) == 1 && d.dil >= 1 && d.t_len > 0);
  VITS_CHECK_SHAPE(d.kc1 >= 2 && (d.kc1 & 1) == 0 && d.channels % d.kc1 == 0);
  VITS_CHECK_SHAPE(d.kc2 >= 2 && (d.kc2 & 1) == 0 && (d.channels / 2) % d.kc2 == 0);
  VITS_CHECK_SHAPE(d.m_pad1 >= d.channels && d.m_pad2 >= d.channels);
  VITS_CHECK_SHAPE(d.cin_pad1 >= d.channels && d.cin_pad2 >= d.channels / 2);
  // 16-byte x staging: time-contiguous rows, T % 4 == 0, aligned
  VITS_CHECK_SHAPE((d.t_len & 3) == 0 && (d.x_cstride & 3) == 0 && (d.x_bstride & 3) == 0 &&
                   d.x_cstride >= d.t_len && (reinterpret_cast<uintptr_t>(d.x) & 15) == 0);
  VITS_CHECK_SHAPE((reinterpret_cast<uintptr_t>(d.w1) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(d.w2) & 15) == 0 && (d.m_pad1 & 3) == 0 &&
                   (d.m_pad2 & 3) == 0);
  return VITS_OK;
}

}  // namespace

extern "C" int vits_resblock_pair_forward(const vits_resblock_pair_desc* d, int n, int batch,
                                          void* stream) {
  if (!d || n < 1 || n > RB_GROUP || batch < 1) return VITS_E_ARG;
  RbGroup g;
  g.n = n;
  g.batch = batch;
  for (int i = 0; i < n; ++i) {
    int rc = rb_check(d[i]);
    if (rc) return rc;
    if (d[i].channels != d[0].channels) return VITS_E_SHAPE;
    g.d[i] = d[i];
  }
  hipStream_t s = as_stream(stream);
  switch (d[0].channels) {
    case 32:
      return count_ok(rb_launch<32, 256, 1, 4>(g, s), VITS_CNT_RESBLOCK);
    case 64:
      return count_ok(rb_launch<64, 256, 1, 4>(g, s), VITS_CNT_RESBLOCK);
    default:
      return VITS_E_UNSUP;
  }
}

extern "C" int vits_resblock_pair_kc(int channels, int k, int dil, int* kc1, int* kc2) {
  // K-chunks: the largest even divisors (c1: of C, c2: of C/2) within the
  // x-window register budget that keep the workgroup's LDS at <= 80 KiB
  // (two workgroups per CU); kc1 first (its chunks carry the x window)
  if (!kc1 || !kc2 || channels < 2 || k < 1 || dil < 1) return VITS_E_ARG;
  const int NG = 256;
  vits_resblock_pair_desc d{};
  d.k = k;
  d.dil = dil;
  int best1 = 0, best2 = 0;
  for (int c1 = 2; c1 <= 16; c1 += 2) {
    if (channels % c1 || c1 * rb_xrs_max(NG, k, dil) > RB_XFLOATS) continue;
    for (int c2 = 2; c2 <= 16; c2 += 2) {
      if ((channels / 2) % c2) continue;
      d.kc1 = c1;
      d.kc2 = c2;
      if (4 * rb_lds_floats(channels, NG, d) > 80 * 1024) continue;
      if (c1 > best1 || (c1 == best1 && c2 > best2)) {
        best1 = c1;
        best2 = c2;
      }
    }
  }
  if (!best1 || !best2) return VITS_E_UNSUP;
  *kc1 = best1;
  *kc2 = best2;
  return VITS_OK;
}
