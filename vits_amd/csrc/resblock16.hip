// resblock16.hip — one ResBlock2 dilation pair of a 16-bit (bf16 / fp16)
// Generator as ONE kernel, 16-bit MFMAs (v_mfma_f32_32x32x16_{bf16,f16}),
// fp32 accumulation, 16-bit activations in HBM:
//
//   y = x + c2( tanh(a + sa) * sigmoid(b + sb) ) ,   (a | b) = c1(lrelu(x, slope))
//
// (modules.py:250-260: c1 = Conv1d(C, C, k, dil d), c2 = Conv1d(C/2, C, k),
// sa / sb = the utterance's cond Linear; models.py:306-318 averages the
// branches: the last pair of each branch accumulates into the stage output).
//
// The two-conv path writes the gated tensor to HBM and reads it back, plus
// the residual: for the 32- / 64-channel stages of a long-form utterance
// (T = 240,000 / 480,000 samples) that traffic and the two launches' short K
// loops (K = C * k and C/2 * k) dominate.  Here one workgroup owns a time
// tile of BN = NG - (k - 1) outputs and all C channels:
//   staging: the whole c1 input window (C channels x NG + (k-1) dil columns,
//            lrelu applied, zero outside [0, T)) goes to LDS once, as
//            [t][C + 8] 16-bit rows (one 16-byte B fragment per lane: 8
//            channels of one column), 4 channels x 4 steps per unit, the
//            transpose done in registers (conv1d_impl.h's T4 staging);
//   phase 1: the c1 GEMM over NG columns (the tile plus c2's (k-1)/2 halo
//            each side), A fragments (gate-interleaved rows) from the packed
//            16-bit image in global memory / L2, one k-step ahead; the gate
//            epilogue writes G[t][C/2 + 8] (16-bit, zero outside [0, L):
//            c2's own zero padding at the utterance ends);
//   phase 2: the c2 GEMM straight from G (tap j = column shift j), residual
//            (x re-read: L2-resident) + bias (+ running branch mean) epilogue
//            to HBM.
// Halo columns are recomputed by the neighbouring tile, never exchanged.
// Every launch holds up to 3 independent pairs (the branches of a stage).
// Weight images: vits_conv1d_desc's 16-bit layout [cin_pad/16][k][2][m_pad][8]
// (ops.to_lowp), c1's rows gate-interleaved (row 2q = a_q, 2q+1 = b_q).
#include <type_traits>

#include "common.h"

namespace {

constexpr int R16_GROUP = 3;
// phase-1 columns per tile: 256 for C = 32 / 64 (4 waves x 64 columns),
// 128 for C = 128 (2 x 2 waves of 64 rows x 64 columns: the 128-channel
// window and gated tile fit two workgroups per CU)
__host__ __device__ constexpr int r16_ng(int C) { return C == 128 ? 128 : 256; }
struct R16Group {
  vits_resblock_pair_desc d[R16_GROUP];
  int n;
  int batch;
  // mean: ONE output, the mean of the n members' pair outputs (the last
  // pairs of a stage's branches, models.py:311-313): each workgroup runs
  // every member on its time tile (tile width bn, common to the members)
  // and keeps the running sum in registers; d[0] names the output
  int mean;
  int bn;
};

__device__ __forceinline__ float r16_sigmoid(float x) {
  return __builtin_amdgcn_rcpf(1.0f + __expf(-x));
}
__device__ __forceinline__ float r16_tanh(float x) {
  return 2.0f * __builtin_amdgcn_rcpf(1.0f + __expf(-2.0f * x)) - 1.0f;
}

// LDS geometry (host and device agree): window columns (4-aligned), row
// pitches in elements, bytes of the whole workgroup
__host__ __device__ inline int r16_xcols(int NG, int k, int dil) {
  // NG + (k-1) dil window columns + up to 3 of alignment shift, 4-blocks
  return ((NG + (k - 1) * dil + 3 + 3) >> 2) << 2;
}
// the gated tile G overlays the c1 window (dead after phase 1; one barrier
// between): 50 KB instead of 71 KB at C = 128, k = 11 - three workgroups per
// CU instead of two on the 64- and 128-channel stages (C5 trace: this kernel
// family 4.95 -> 4.82 ms per step, profiles/r05_r16al_*)
__host__ __device__ inline int r16_lds_bytes(int C, int k, int dil) {
  const int xp = C + 8, gp = C / 2 + 8, NG = r16_ng(C);
  const int xsz = r16_xcols(NG, k, dil) * xp, gsz = (NG + 16) * gp;
  return 2 * (xsz > gsz ? xsz : gsz) + 4 * 2 * C + 64;
}

template <int C, typename T, bool MEAN>
__global__ __launch_bounds__(256, MEAN ? 2 : 3) void resblock16_kernel(
    const R16Group G) {
  constexpr int H = C / 2;
  constexpr int NG = r16_ng(C);
  constexpr int WAVES_M = C == 128 ? 2 : 1;
  constexpr int WAVES_N = 4 / WAVES_M;
  constexpr int TM = C / 32 / WAVES_M;  // 32-row MFMA tiles of c1 / c2 per wave
  constexpr int TN = 2;                 // 64 columns per wave
  static_assert(NG == 64 * WAVES_N, "tile columns");
  constexpr int XP = C + 8;        // window row pitch (16-bit elements)
  constexpr int GP = H + 8;        // gated row pitch
  constexpr int S1 = C / 16;       // 16-channel slabs of c1's K
  constexpr int S2 = H / 16;       // ... of c2's K
  typedef T t8 __attribute__((ext_vector_type(8)));
  typedef T t4 __attribute__((ext_vector_type(4)));
  static_assert(C == 32 || C == 64 || C == 128, "32- / 64- / 128-channel stages");

  const int gsel = MEAN ? 0 : (int)blockIdx.z / G.batch;
  const int b = (int)blockIdx.z - gsel * G.batch;
  const vits_resblock_pair_desc& p0 = G.d[gsel];
  const int Tn = p0.t_len;
  const int L = p0.lengths ? min(Tn, (int)p0.lengths[b]) : Tn;
  const int BN = MEAN ? G.bn : NG - (p0.k - 1);
  const int n0 = blockIdx.x * BN;
  if (n0 >= Tn) return;
  if (p0.lengths && p0.len_skip > 0 && n0 >= L + p0.len_skip) return;

  extern __shared__ float smem[];
  float* const erow = smem;                                   // [2C] row constants
  T* const xs = reinterpret_cast<T*>(smem + 2 * C + 16);      // [xcols][XP]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wn = (wid % WAVES_N) * 64;   // wave's column offset
  const int wm = (wid / WAVES_N) * (C / WAVES_M);  // wave's row offset
  const int l32 = lane & 31;
  const int lhi = lane >> 5;

  f32x16 acc[TM][TN];
  f32x16 ysum[MEAN ? TM : 1][MEAN ? TN : 1];  // (MEAN: the running branch sum)
  if constexpr (MEAN) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) ysum[i][j][r] = 0.f;
  }

  const int nmem = MEAN ? G.n : 1;
  for (int mem = 0; mem < nmem; ++mem) {
  const vits_resblock_pair_desc& p = G.d[gsel + mem];
  const int k = p.k;
  const int dil = p.dil;
  const int p1 = (k - 1) * dil / 2;
  const int p2 = (k - 1) / 2;
  const int xcols = r16_xcols(NG, k, dil);
  T* const gs = xs;  // [NG + 16][GP], over the dead c1 window
  if (mem > 0) __syncthreads();  // the previous member's reads of LDS are done

  // row constants: c1 bias + cond (gate-interleaved order), c2 bias
  const float* cond = p.cond ? p.cond + (int64_t)b * p.cond_bstride : nullptr;
  for (int r = tid; r < 2 * C; r += 256) {
    float e = 0.f;
    if (r < C) {
      const int idx = (r & 1) ? H + (r >> 1) : (r >> 1);
      if (p.b1) e = p.b1[idx];
      if (cond) e += cond[idx];
    } else if (p.b2) {
      e = p.b2[r - C];
    }
    erow[r] = e;
  }

  // ---- the c1 window -> LDS (lrelu, zero padding), 4 ch x 4 steps per unit
  const T* xb = reinterpret_cast<const T*>(p.x) + (int64_t)b * p.x_bstride;
  const int tw0 = n0 - p2 - p1;          // time of window column 0 (before the shift)
  const int xstart = tw0 & ~3;           // 8-byte aligned block start
  const int xsh = tw0 - xstart;          // window column c sits at LDS column c + xsh
  const int nb = xcols >> 2;             // 4-step blocks
  const float slope = p.in_slope;
  {
    // unit u -> (channel quad cq, 4-step block tb), quads fastest (distinct
    // LDS banks for the 8-byte writes).  Every unit's four 8-byte loads are
    // issued before any is consumed (NU units per thread in registers): a
    // load -> convert -> store loop waits one memory round trip per unit.
    constexpr int NU = ((C / 4) * ((NG + 96 + 6) / 4) + 255) / 256;
    const int nunits = (C / 4) * nb;
    // (loads are unconditional - out-of-range units read the utterance's
    // first block and are zeroed below - so no branch splits the batch)
    t4 v[NU][4];
    bool okq[NU];
#pragma unroll
    for (int q = 0; q < NU; ++q) {
      const int u = tid + 256 * q;
      const int cq = u % (C / 4);
      const int tt = xstart + 4 * (u / (C / 4));
      okq[q] = u < nunits && tt >= 0 && tt < Tn;  // T % 4 == 0: a block is all in or out
      const int64_t off = okq[q] ? (int64_t)(4 * cq) * p.x_cstride + tt : 0;
      const int64_t cs = okq[q] ? p.x_cstride : 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[q][i] = *reinterpret_cast<const t4*>(xb + off + i * cs);
    }
#pragma unroll
    for (int q = 0; q < NU; ++q) {
      const int u = tid + 256 * q;
      if (u < nunits) {
        const int cq = u % (C / 4);
        const int tb = u / (C / 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          t4 w;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float f = okq[q] ? (float)v[q][i][e] : 0.f;
            f = f < 0.f ? f * slope : f;
            w[i] = (T)f;
          }
          *reinterpret_cast<t4*>(xs + (4 * tb + e) * XP + 4 * cq) = w;
        }
      }
    }
  }
  __syncthreads();

#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto mfma = [&](const t8& a, const t8& bb, f32x16 c) -> f32x16 {
    if constexpr (std::is_same<T, _Float16>::value)
      return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, bb, c, 0, 0, 0);
    else
      return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bb, c, 0, 0, 0);
  };

  // one GEMM: steps s = slab * k + j (the image's order), A of step s from
  // the packed image (16 bytes per lane and 32-row fragment, one step
  // ahead), B from LDS: 8 channels (16 s + 8 lhi ..) of column
  // col0 + ni * 32 + j * jstride
  auto gemm = [&](const T* wimg, int m_pad, int nsteps, const T* bsrc, int pitch, int col0,
                  int jstride) {
    const T* wl = wimg + ((int64_t)lhi * m_pad + wm + l32) * 8;
    const int64_t wstep = (int64_t)16 * m_pad;
    const T* bl = bsrc + (col0 + l32) * pitch + 8 * lhi;
    auto loadA = [&](int s, t8* a) {
      const T* w = wl + (int64_t)(s < nsteps ? s : nsteps - 1) * wstep;
#pragma unroll
      for (int mi = 0; mi < TM; ++mi) a[mi] = *reinterpret_cast<const t8*>(w + mi * 32 * 8);
    };
    int g = 0, j = 0;
    auto loadB = [&](t8* bb) {
      const T* x = bl + j * jstride * pitch + 16 * g;
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) bb[ni] = *reinterpret_cast<const t8*>(x + ni * 32 * pitch);
      if (++j == k) {
        j = 0;
        ++g;
      }
    };
    auto mma = [&](const t8* a, const t8* bb) {
#pragma unroll
      for (int mi = 0; mi < TM; ++mi)
#pragma unroll
        for (int ni = 0; ni < TN; ++ni) acc[mi][ni] = mfma(a[mi], bb[ni], acc[mi][ni]);
    };
    // A fragments PF - 1 steps ahead in a register ring (slot = step % PF):
    // one step of TM * TN MFMAs does not cover an L2 round trip.  C5 trace:
    // this kernel family 4.94 -> 4.84 ms per step (profiles/r05_r16pf_*)
    constexpr int PF = 4;
    static_assert(PF == 2 || PF == 4, "ring parity");
    t8 ar[PF][TM], bb[2][TN];
#pragma unroll
    for (int i = 0; i < PF - 1; ++i) loadA(i, ar[i]);
    loadB(bb[0]);
    int s = 0;
    for (; s + PF <= nsteps; s += PF) {
#pragma unroll
      for (int u = 0; u < PF; ++u) {
        loadA(s + u + PF - 1, ar[(u + PF - 1) % PF]);
        if (s + u + 1 < nsteps) loadB(bb[(u + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);
        mma(ar[u], bb[u & 1]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // the last nsteps % PF steps: their A fragments are already in slots 0..
#pragma unroll
    for (int u = 0; u < PF - 1; ++u) {
      if (s + u < nsteps) {
        if (s + u + 1 < nsteps) loadB(bb[(u + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);
        mma(ar[u], bb[u & 1]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };

  // ---------------- phase 1: c1 over NG columns from n0 - p2 ---------------
  gemm(reinterpret_cast<const T*>(p.w1), p.m_pad1, S1 * k, xs, XP, wn + xsh, dil);
  __syncthreads();  // every wave's window reads are done: G overlays it

  // gate epilogue -> G (zero outside [0, L)); the 16 columns past NG that
  // phase 2's discarded columns read are zeroed too
#pragma unroll
  for (int mi = 0; mi < TM; ++mi) {
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) {
      const int col = wn + ni * 32 + l32;
      const int t = n0 - p2 + col;
      const bool in = t >= 0 && t < L;
#pragma unroll
      for (int r = 0; r < 16; r += 4) {
        // rows rloc, rloc + 1 (a_q, b_q) and rloc + 2, rloc + 3 (a_q+1, b_q+1)
        const int row = wm + mi * 32 + 4 * lhi + 8 * (r >> 2);
        const float g0 = r16_tanh(acc[mi][ni][r] + erow[row]) *
                         r16_sigmoid(acc[mi][ni][r + 1] + erow[row + 1]);
        const float g1 = r16_tanh(acc[mi][ni][r + 2] + erow[row + 2]) *
                         r16_sigmoid(acc[mi][ni][r + 3] + erow[row + 3]);
        typedef T t2 __attribute__((ext_vector_type(2)));
        t2 v;
        v[0] = (T)(in ? g0 : 0.f);
        v[1] = (T)(in ? g1 : 0.f);
        *reinterpret_cast<t2*>(gs + col * GP + (row >> 1)) = v;
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][ni][r] = 0.f;
    }
  }
  for (int i = tid; i < 16 * H; i += 256) gs[(NG + i / H) * GP + i % H] = (T)0.f;
  __syncthreads();

  // ---------------- phase 2: c2 from G --------------------------------------
  gemm(reinterpret_cast<const T*>(p.w2), p.m_pad2, S2 * k, gs, GP, wn, 1);

  // residual (+ running branch mean) epilogue, 16-bit out.  The residual /
  // running-mean loads of a 32x32 tile are issued unconditionally (clamped
  // to column 0 outside the tile) before any is used.
#pragma unroll
  for (int mi = 0; mi < TM; ++mi) {
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) {
      const int col = wn + ni * 32 + l32;
      const int t = n0 + col;
      const bool st = col < BN && t < Tn;
      const int tc = st ? t : 0;
      float rv[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wm + mi * 32 + 4 * lhi + (r & 3) + 8 * (r >> 2);
        rv[r] = (float)xb[(int64_t)row * p.x_cstride + tc];
      }
      if constexpr (MEAN) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = wm + mi * 32 + 4 * lhi + (r & 3) + 8 * (r >> 2);
          ysum[mi][ni][r] += rv[r] + (acc[mi][ni][r] + erow[C + row]);
        }
        continue;
      }
      T* yb = reinterpret_cast<T*>(p.y) + (int64_t)b * p.y_bstride;
      float yo[16];
      if (p.accumulate) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = wm + mi * 32 + 4 * lhi + (r & 3) + 8 * (r >> 2);
          yo[r] = (float)yb[(int64_t)row * p.y_cstride + tc];
        }
      }
      if (st) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = wm + mi * 32 + 4 * lhi + (r & 3) + 8 * (r >> 2);
          float v = rv[r] + (acc[mi][ni][r] + erow[C + row]);
          if (p.accumulate) v = yo[r] + v;
          if (p.post_div != 1.0f) v = v / p.post_div;
          yb[(int64_t)row * p.y_cstride + t] = (T)(t < L ? v : 0.f);
        }
      }
    }
  }
  }  // members

  if constexpr (MEAN) {
    const float inv_n = 1.0f / (float)G.n;
    T* yb = reinterpret_cast<T*>(p0.y) + (int64_t)b * p0.y_bstride;
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) {
        const int col = wn + ni * 32 + l32;
        const int t = n0 + col;
        if (col < BN && t < Tn) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = wm + mi * 32 + 4 * lhi + (r & 3) + 8 * (r >> 2);
            yb[(int64_t)row * p0.y_cstride + t] = (T)(t < L ? ysum[mi][ni][r] * inv_n : 0.f);
          }
        }
      }
    }
  }
}

template <int C, typename T>
int r16_launch(const R16Group& g, hipStream_t s) {
  int lds = 0, gx = 0;
  for (int i = 0; i < g.n; ++i) {
    const vits_resblock_pair_desc& d = g.d[i];
    const int l = r16_lds_bytes(C, d.k, d.dil);
    if (l > lds) lds = l;
    const int BN = g.mean ? g.bn : r16_ng(C) - (d.k - 1);
    const int x = (d.t_len + BN - 1) / BN;
    if (x > gx) gx = x;
  }
  if (lds > 160 * 1024) return VITS_E_UNSUP;
  if (g.mean)
    hipLaunchKernelGGL((resblock16_kernel<C, T, true>), dim3(gx, 1, g.batch), dim3(256), lds, s,
                       g);
  else
    hipLaunchKernelGGL((resblock16_kernel<C, T, false>), dim3(gx, 1, g.n * g.batch), dim3(256),
                       lds, s, g);
  return vits_launch_status();
}

int r16_check(const vits_resblock_pair_desc& d) {
  VITS_CHECK_ARG(d.x && d.w1 && d.w2 && d.y);
  // other workgroups still read x (halos, residual): never write in place
  VITS_CHECK_ARG(reinterpret_cast<const void*>(d.y) != reinterpret_cast<const void*>(d.x));
  VITS_CHECK_SHAPE(d.channels == 32 || d.channels == 64 || d.channels == 128);
  VITS_CHECK_SHAPE(d.k >= 1 && d.k <= 15 && (d.k & 1) == 1 && d.dil >= 1 && d.t_len > 0);
  VITS_CHECK_SHAPE((d.k - 1) * d.dil <= 96);  // window within the LDS budget
  // images: [cin_pad/16][k][2][m_pad][8], rows = C (c1 gate-interleaved / c2)
  VITS_CHECK_SHAPE(d.m_pad1 >= d.channels && d.m_pad2 >= d.channels && (d.m_pad1 & 3) == 0 &&
                   (d.m_pad2 & 3) == 0);
  VITS_CHECK_SHAPE(d.cin_pad1 >= d.channels && d.cin_pad2 >= d.channels / 2);
  // 8-byte x staging: time-contiguous rows, T % 4 == 0, aligned
  VITS_CHECK_SHAPE((d.t_len & 3) == 0 && (d.x_cstride & 3) == 0 && (d.x_bstride & 3) == 0 &&
                   d.x_cstride >= d.t_len && d.y_cstride >= d.t_len &&
                   (reinterpret_cast<uintptr_t>(d.x) & 7) == 0);
  VITS_CHECK_SHAPE((reinterpret_cast<uintptr_t>(d.w1) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(d.w2) & 15) == 0);
  return VITS_OK;
}

}  // namespace

// resblock_f32p.hip: the 256-channel pairs (a streamed-K tile)
int vits_rp16_256(const vits_resblock_pair_desc* d, int n, int batch, int wdtype,
                  hipStream_t s);

static int r16_run(const vits_resblock_pair_desc* d, int n, int batch, int wdtype, int mean,
                   void* stream) {
  if (!d || n < 1 || n > R16_GROUP || batch < 1) return VITS_E_ARG;
  if (wdtype != VITS_WDT_BF16 && wdtype != VITS_WDT_F16) return VITS_E_ARG;
  // a 256-channel window does not fit this kernel's whole-window staging
  if (d[0].channels == 256 && !mean) return vits_rp16_256(d, n, batch, wdtype, as_stream(stream));
  R16Group g;
  g.n = n;
  g.batch = batch;
  g.mean = mean;
  int kmax = 1;
  for (int i = 0; i < n; ++i) {
    const int rc = r16_check(d[i]);
    if (rc) return rc;
    if (d[i].channels != d[0].channels) return VITS_E_SHAPE;
    if (mean) {
      // one output tile per workgroup over every member: same time axis,
      // the same utterance lengths, and no member may write its input
      VITS_CHECK_SHAPE(d[i].t_len == d[0].t_len && d[i].lengths == d[0].lengths);
      VITS_CHECK_ARG(reinterpret_cast<const void*>(d[0].y) != reinterpret_cast<const void*>(d[i].x));
    }
    if (d[i].k > kmax) kmax = d[i].k;
    g.d[i] = d[i];
  }
  g.bn = r16_ng(d[0].channels) - (kmax - 1);
  hipStream_t s = as_stream(stream);
  const bool f16 = wdtype == VITS_WDT_F16;
  if (d[0].channels == 32)
    return f16 ? r16_launch<32, _Float16>(g, s) : r16_launch<32, __bf16>(g, s);
  if (d[0].channels == 64)
    return f16 ? r16_launch<64, _Float16>(g, s) : r16_launch<64, __bf16>(g, s);
  return f16 ? r16_launch<128, _Float16>(g, s) : r16_launch<128, __bf16>(g, s);
}

extern "C" int vits_resblock_pair16_forward(const vits_resblock_pair_desc* d, int n, int batch,
                                            int wdtype, void* stream) {
  return count_ok(r16_run(d, n, batch, wdtype, 0, stream), VITS_CNT_RESBLOCK);
}

extern "C" int vits_resblock_pair16_mean_forward(const vits_resblock_pair_desc* d, int n,
                                                 int batch, int wdtype, void* stream) {
  return count_ok(r16_run(d, n, batch, wdtype, 1, stream), VITS_CNT_RESBLOCK);
}
