// resblock_f32p.hip — one ResBlock2 dilation pair of the fp32 Generator's
// 32-, 64-, 128- and 256-channel stages as ONE kernel, in the split-fp32
// arithmetic of the pre-split-weight conv (VITS_WDT_F32P, conv1d_impl.h):
//
//   y = x + c2( tanh(a + sa) * sigmoid(b + sb) ) ,   (a | b) = c1(lrelu(x, 0.1))
//
// (modules.py:250-260; c1 = Conv1d(C, C, k, dil d), c2 = Conv1d(C/2, C, k),
// sa / sb the utterance's cond Linear; models.py:306-318 averages the
// branches: the last pair of each branch accumulates into the stage output).
//
// The two-conv path writes the gated tensor (fp32) to HBM, reads it back
// with c2's halo, and re-reads x as the residual; c2 is a short-K GEMM
// (K = C/2 * k) whose own window staging, barriers and epilogue dominate
// it (0.2-0.4 of the split-fp32 ceiling on the headline step).  Here one
// workgroup owns a time tile of BN = NG - (k - 1) outputs and all C
// channels; every wave computes a 64 x 64 sub-tile in both phases:
//   phase 1: the c1 GEMM over NG columns (the tile plus c2's (k-1)/2 halo
//            each side; rows gate-interleaved), exactly the conv kernel's
//            global-A loop: A fragments (hi / mid / lo planes) from the
//            host-split image in L2, one k-step ahead; the x window staged
//            16 channels (C = 256: 64) at a time (lrelu, zero padding, exact
//            three-way bf16 split) into double-buffered [t][16 + 4] planes;
//   gate:    tanh * sigmoid of the fp32 accumulators, split exactly into
//            three bf16 planes G[t][C/2 + 8] in LDS (zero outside [0, L):
//            c2's own zero padding, and the utterance end) - over the X
//            buffers, which are dead by then;
//   phase 2: the c2 GEMM from G (tap j = row shift j), no barriers, then
//            residual (x: L2-resident from phase 1) + bias (+ accumulate /
//            branch-mean division) to HBM.
// Halo columns are recomputed by the neighbouring tile, never exchanged.
// The arithmetic is the two-conv path's to the bit: the same split planes,
// the same k-step order (slab-major, then tap), the same six products per
// fragment pair in the same order, the same gate and epilogue expressions
// (tests/test_resblock_f32p_gpu.py checks equality).  Tiles: C = 64 ->
// 64 x 256 (1 x 4 waves; C = 32: 32 x 256), C = 128 -> 128 x 128 (2 x 2), two workgroups per
// CU; C = 256 -> 256 x 128 (4 x 2 waves, one 512-thread workgroup per CU:
// the same two waves per SIMD).  Every launch holds up to 3 independent
// pairs (the branches of a stage).
//
// MODE 1 / 2: the same tile for a bf16 / fp16 model's 256-channel pairs
// (vits_resblock_pair16_forward routes them here - resblock16.hip stages a
// whole window, which 256 channels do not fit): 16-bit x / y in HBM, one
// operand plane, one MFMA per fragment pair, the gated tensor rounded to the
// 16-bit type in LDS as the two-conv path rounds it in HBM.  C5 (B=4,
// Ty=2500): 9.84 -> 9.07 ms/step (tools/r05_p256.sh).  The 128-channel
// pairs measured the same here as in resblock16 (r05_p128.sh) and stay there.
#include "conv1d_impl.h"

namespace {

using vits_conv::fast_sigmoid;
using vits_conv::fast_tanh;
using vits_conv::split3_bf16x4;

constexpr int RP_GROUP = 3;
struct RpGroup {
  vits_resblock_pair_desc d[RP_GROUP];
  int n;
  int batch;
};

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4v __attribute__((ext_vector_type(4)));

// operand mode: 0 = split fp32 (fp32 x / y, three exact bf16 planes per
// operand, six products), 1 = bf16 / 2 = fp16 models (16-bit x / y as the
// 16-bit decoder holds them, one plane, one product; the gated tensor rounded
// to the 16-bit type as the two-conv path stores it)
template <int MODE>
struct RpT {
  typedef float xt;   // activation element in HBM
  typedef __bf16 lt;  // LDS / MFMA operand element
  static constexpr int NPL = 3;
};
template <>
struct RpT<1> {
  typedef __bf16 xt;
  typedef __bf16 lt;
  static constexpr int NPL = 1;
};
template <>
struct RpT<2> {
  typedef _Float16 xt;
  typedef _Float16 lt;
  static constexpr int NPL = 1;
};
__host__ __device__ constexpr int rp_npl(int mode) { return mode == 0 ? 3 : 1; }

__host__ __device__ constexpr int rp_ng(int C) { return C <= 64 ? 256 : 128; }
// threads: 4 waves (C = 64, 128), 8 waves of 64 x 64 (C = 256: 256 x 128)
__host__ __device__ constexpr int rp_threads(int C) { return C == 256 ? 512 : 256; }
// c1 channels per staged X chunk (one barrier each): 16 where two workgroups
// share a CU (the double-buffered chunk must fit beside nothing but the G
// planes it aliases), 64 for the one-workgroup 256-channel tile (its X
// buffers still fit the LDS: four slabs per barrier)
__host__ __device__ constexpr int rp_kc(int C, int mode = 0) {
  return C == 256 ? 64 : 16;  // (the 16-bit mode measured the same at 32 / 64)
}
__host__ __device__ inline int rp_xcols(int NG, int k, int dil) {
  // NG + (k-1) dil window columns + up to 3 of alignment shift, 4-blocks
  return ((NG + (k - 1) * dil + 3 + 3) >> 2) << 2;
}
// LDS: erow [2C] floats, then max(two X slab buffers, the G planes)
__host__ __device__ inline int rp_lds_bytes(int C, int k, int dil, int mode = 0) {
  const int NG = rp_ng(C), npl = rp_npl(mode);
  const int xs = 2 * npl * rp_xcols(NG, k, dil) * (rp_kc(C, mode) + 4);
  const int gsz = npl * (NG + 16) * (C / 2 + 8);
  return 4 * 2 * C + 2 * (xs > gsz ? xs : gsz) + 64;
}
// minimum waves per SIMD the kernel is compiled for (launch_bounds' second
// argument): two 4-wave workgroups per CU below 256 channels, one 8-wave one
// at 256.  (16-bit 256: two 8-wave workgroups per CU need <= 128 VGPRs and
// spill 24; measured the same on C5, tools/r05_p256b.sh)
__host__ __device__ constexpr int rp_occ(int C, int) { return C == 256 ? 1 : 2; }

template <int C, int MODE = 0>
__global__ __launch_bounds__(rp_threads(C), rp_occ(C, MODE)) void resblock_f32p_kernel(
    const RpGroup G) {
  typedef typename RpT<MODE>::xt xt;
  typedef typename RpT<MODE>::lt lt;
  constexpr int NPL = RpT<MODE>::NPL;
  typedef lt lt8 __attribute__((ext_vector_type(8)));
  typedef lt lt4 __attribute__((ext_vector_type(4)));
  typedef lt lt2 __attribute__((ext_vector_type(2)));
  typedef xt xt4 __attribute__((ext_vector_type(4)));
  constexpr int H = C / 2;
  constexpr int NT = rp_threads(C);
  constexpr int WAVES_M = C >= 64 ? C / 64 : 1;
  constexpr int WAVES_N = NT / 64 / WAVES_M;
  constexpr int NG = 64 * WAVES_N;
  static_assert(NG == rp_ng(C), "tile columns");
  constexpr int TM = C >= 64 ? 2 : 1, TN = 2;  // 64 x 64 per wave (C = 32: 32 x 64)
  constexpr int KC = rp_kc(C, MODE);          // c1 channels per staged chunk
  constexpr int KCP = KC + 4;           // X chunk row pitch (bf16)
  constexpr int GP = H + 8;              // G row pitch (bf16): 16-byte rows
  constexpr int GPL = (NG + 16) * GP;    // G plane (elements)
  constexpr int S1 = C / 16, S2 = H / 16;
  constexpr int NU = ((KC / 4) * ((NG + 102) / 4) + NT - 1) / NT;  // staging units per thread
  typedef lt8 av_t;
  constexpr int NB = NPL == 3 ? TN : 1;  // (mid / lo B planes: split only)

  const int gi = (int)blockIdx.z / G.batch;
  const int b = (int)blockIdx.z - gi * G.batch;
  const vits_resblock_pair_desc& p = G.d[gi];
  const int Tn = p.t_len;
  const int L = p.lengths ? min(Tn, (int)p.lengths[b]) : Tn;
  const int k = p.k;
  const int dil = p.dil;
  const int BN = NG - (k - 1);
  const int n0 = blockIdx.x * BN;
  if (n0 >= Tn) return;
  if (p.lengths && p.len_skip > 0 && n0 >= L + p.len_skip) return;

  extern __shared__ float smem[];
  float* const erow = smem;  // [2C]: c1 bias + cond (gate-interleaved), c2 bias
  lt* const reg = reinterpret_cast<lt*>(smem + 2 * C);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wn = (wid % WAVES_N) * 64;
  const int wm = (wid / WAVES_N) * 64;
  const int l32 = lane & 31;
  const int lhi = lane >> 5;
  const int p1 = (k - 1) * dil / 2;
  const int p2 = (k - 1) / 2;

  {
    const float* cond = p.cond ? p.cond + (int64_t)b * p.cond_bstride : nullptr;
    for (int r = tid; r < 2 * C; r += NT) {
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
  }

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // six products per fragment pair, small terms first (conv1d_impl.h's
  // F32P order: bitwise the conv's sums)
  auto mma = [&](av_t (*a)[TM], const av_t* bh, const av_t* bm, const av_t* bl) {
#pragma unroll
    for (int mi = 0; mi < TM; ++mi)
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) {
        f32x16 c = acc[mi][ni];
        if constexpr (MODE == 0) {
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][mi], bl[ni], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2][mi], bh[ni], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][mi], bm[ni], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][mi], bm[ni], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][mi], bh[ni], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][mi], bh[ni], c, 0, 0, 0);
        } else if constexpr (MODE == 1) {
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][mi], bh[ni], c, 0, 0, 0);
        } else {
          c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0][mi], bh[ni], c, 0, 0, 0);
        }
        acc[mi][ni] = c;
      }
  };
  // A fragments of flat step s (image [cin_pad/16][k][2][NPL][m_pad][8]):
  // plane q, half lhi, rows wm + mi * 32 + l32
  auto loadA = [&](const lt* wl, int64_t wstep, int m_pad, int s, int total,
                   av_t (*a)[TM]) {
    const lt* wp = wl + (int64_t)(s < total ? s : total - 1) * wstep;
#pragma unroll
    for (int q = 0; q < NPL; ++q)
#pragma unroll
      for (int mi = 0; mi < TM; ++mi)
        a[q][mi] = *reinterpret_cast<const av_t*>(wp + ((int64_t)q * m_pad + mi * 32) * 8);
  };

  av_t a0[NPL][TM], a1[NPL][TM];
  av_t bh0[TN], bm0[NB], bl0[NB], bh1[TN], bm1[NB], bl1[NB];

  // ---------------- phase 1: c1 over NG columns from n0 - p2 ---------------
  const xt* xb = reinterpret_cast<const xt*>(p.x) + (int64_t)b * p.x_bstride;
  {
    const int tw0 = n0 - p2 - p1;  // time of window column 0
    const int xstart = tw0 & ~3;   // 16-byte aligned block start
    const int xsh = tw0 - xstart;  // window column c sits at LDS row c + xsh
    const int xcols = rp_xcols(NG, k, dil);
    const int nunits = (KC / 4) * (xcols >> 2);  // channel quads x 4-step blocks
    const int xpl = xcols * KCP;   // plane (elements)
    lt* const xbuf0 = reg;
    lt* const xbuf1 = reg + NPL * xpl;
    const float slope = p.in_slope;
    // unit u: channel quad u % (KC/4), 4-step block u / (KC/4) (a 16-lane
    // group's 8-byte LDS pieces fall on distinct banks)
    xt4 xr[NU][4];
    int xoff[NU];
    bool xok[NU];
#pragma unroll
    for (int q = 0; q < NU; ++q) {
      const int u = tid + NT * q;
      const int tt = xstart + 4 * (u / (KC / 4));
      xok[q] = u < nunits && tt >= 0 && tt < Tn;  // T % 4 == 0: a block is all in or out
      xoff[q] = xok[q] ? 4 * (u % (KC / 4)) * p.x_cstride + tt : 0;
    }
    // loads issued unconditionally (clamped address, zeroed in lstore)
    auto gload = [&](int ch) {
      const xt* base = xb + (int64_t)ch * KC * p.x_cstride;
#pragma unroll
      for (int q = 0; q < NU; ++q) {
        if (q * NT < nunits) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const xt* src = xok[q] ? base + xoff[q] + i * p.x_cstride : xb;
            xr[q][i] = *reinterpret_cast<const xt4*>(src);
          }
        }
      }
    };
    auto lstore = [&](lt* xs) {
#pragma unroll
      for (int q = 0; q < NU; ++q) {
        const int u = tid + NT * q;
        if (q * NT < nunits && u < nunits) {
          f32x4v v[4];
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              float t = (float)xr[q][i][e];
              t = t < 0.f ? t * slope : t;
              v[i][e] = xok[q] ? t : 0.f;
            }
          lt* xh = xs + 4 * (u / (KC / 4)) * KCP + 4 * (u % (KC / 4));
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const f32x4v w = {v[0][e], v[1][e], v[2][e], v[3][e]};
            if constexpr (NPL == 3) {
              bf16x4 h4, m4, l4;
              split3_bf16x4(w, h4, m4, l4);
              *reinterpret_cast<bf16x4*>(xh + e * KCP) = h4;
              *reinterpret_cast<bf16x4*>(xh + xpl + e * KCP) = m4;
              *reinterpret_cast<bf16x4*>(xh + 2 * xpl + e * KCP) = l4;
            } else {
              lt4 w4;
#pragma unroll
              for (int i = 0; i < 4; ++i) w4[i] = (lt)w[i];
              *reinterpret_cast<lt4*>(xh + e * KCP) = w4;
            }
          }
        }
      }
    };
    // B fragments of tap j, slab g of the chunk: rows wn + ni * 32 + l32 +
    // j * dil (+ xsh), channels 16 g + 8 lhi .. + 8 (two 8-byte reads per plane)
    auto loadB = [&](const lt* xs, int j, int g, av_t* bh, av_t* bm, av_t* bl) {
      const int P4 = xpl / 4;
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) {
        const lt4* xp = reinterpret_cast<const lt4*>(
            xs + (wn + ni * 32 + l32 + j * dil + xsh) * KCP + 16 * g + 8 * lhi);
        bh[ni] = __builtin_shufflevector(xp[0], xp[1], 0, 1, 2, 3, 4, 5, 6, 7);
        if constexpr (NPL == 3) {
          bm[ni] = __builtin_shufflevector(xp[P4], xp[P4 + 1], 0, 1, 2, 3, 4, 5, 6, 7);
          bl[ni] = __builtin_shufflevector(xp[2 * P4], xp[2 * P4 + 1], 0, 1, 2, 3, 4, 5, 6, 7);
        }
      }
    };
    const lt* wl = reinterpret_cast<const lt*>(p.w1) +
                   ((int64_t)(lhi * NPL) * p.m_pad1 + wm + l32) * 8;
    const int64_t wstep = (int64_t)16 * NPL * p.m_pad1;
    const int total = S1 * k;
    const int nst = (KC / 16) * k;  // k-steps per chunk: slab-major, then tap
    loadA(wl, wstep, p.m_pad1, 0, total, a0);
    gload(0);
    lstore(xbuf0);
    __syncthreads();
    for (int ch = 0; ch < C / KC; ++ch) {
      const bool more = ch + 1 < C / KC;
      if (more) gload(ch + 1);  // in flight under this chunk's MFMAs
      const lt* xs = (ch & 1) ? xbuf1 : xbuf0;
      const int s0 = ch * nst;
      int j = 0, g = 0;  // (tap, slab) of the next B load
      auto next = [&]() {
        if (++j == k) {
          j = 0;
          ++g;
        }
      };
      loadB(xs, 0, 0, bh0, bm0, bl0);
      int st = 0;
      // the loads of step st + 1 pinned ahead of step st's MFMAs
      for (; st + 2 <= nst; st += 2) {
        next();
        loadA(wl, wstep, p.m_pad1, s0 + st + 1, total, a1);
        loadB(xs, j, g, bh1, bm1, bl1);
        __builtin_amdgcn_sched_barrier(0);
        mma(a0, bh0, bm0, bl0);
        __builtin_amdgcn_sched_barrier(0);
        next();
        loadA(wl, wstep, p.m_pad1, s0 + st + 2, total, a0);
        if (st + 2 < nst) loadB(xs, j, g, bh0, bm0, bl0);
        __builtin_amdgcn_sched_barrier(0);
        mma(a1, bh1, bm1, bl1);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (st < nst) {  // odd step count: the last step, and the next chunk's A
        loadA(wl, wstep, p.m_pad1, s0 + nst, total, a1);
        __builtin_amdgcn_sched_barrier(0);
        mma(a0, bh0, bm0, bl0);
#pragma unroll
        for (int q = 0; q < NPL; ++q)
#pragma unroll
          for (int mi = 0; mi < TM; ++mi) a0[q][mi] = a1[q][mi];
      }
      if (more) lstore((ch & 1) ? xbuf0 : xbuf1);
      __syncthreads();
    }
  }

  // ---------------- gate -> G planes (over the dead X buffers) -------------
  lt* const gs = reg;
#pragma unroll
  for (int mi = 0; mi < TM; ++mi) {
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) {
      const int col = wn + ni * 32 + l32;
      const int t = n0 - p2 + col;
      const bool in = t >= 0 && t < L;
#pragma unroll
      for (int r = 0; r < 16; r += 4) {
        // rows row, row + 1 (a_q, b_q) and row + 2, row + 3 (a_q+1, b_q+1)
        const int row = wm + mi * 32 + 4 * lhi + 8 * (r >> 2);
        const float g0 = fast_tanh(acc[mi][ni][r] + erow[row]) *
                         fast_sigmoid(acc[mi][ni][r + 1] + erow[row + 1]);
        const float g1 = fast_tanh(acc[mi][ni][r + 2] + erow[row + 2]) *
                         fast_sigmoid(acc[mi][ni][r + 3] + erow[row + 3]);
        lt* gp = gs + col * GP + (row >> 1);
        if constexpr (NPL == 3) {
          const f32x4v w = {in ? g0 : 0.f, in ? g1 : 0.f, 0.f, 0.f};
          bf16x4 h4, m4, l4;
          split3_bf16x4(w, h4, m4, l4);
          *reinterpret_cast<bf16x2*>(gp) = __builtin_shufflevector(h4, h4, 0, 1);
          *reinterpret_cast<bf16x2*>(gp + GPL) = __builtin_shufflevector(m4, m4, 0, 1);
          *reinterpret_cast<bf16x2*>(gp + 2 * GPL) = __builtin_shufflevector(l4, l4, 0, 1);
        } else {
          lt2 v2;
          v2[0] = (lt)(in ? g0 : 0.f);
          v2[1] = (lt)(in ? g1 : 0.f);
          *reinterpret_cast<lt2*>(gp) = v2;
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][ni][r] = 0.f;
    }
  }
  // the 16 rows past NG that phase 2's discarded columns read: zero
  for (int i = tid; i < NPL * 16 * H; i += NT) {
    const int pl = i / (16 * H);
    const int e = i - pl * 16 * H;
    gs[pl * GPL + (NG + e / H) * GP + e % H] = (lt)0.f;
  }
  __syncthreads();

  // ---------------- phase 2: c2 from G --------------------------------------
  {
    const lt* wl = reinterpret_cast<const lt*>(p.w2) +
                   ((int64_t)(lhi * NPL) * p.m_pad2 + wm + l32) * 8;
    const int64_t wstep = (int64_t)16 * NPL * p.m_pad2;
    const int total = S2 * k;
    const lt* gl = gs + (wn + l32) * GP + 8 * lhi;
    int j = 0, g = 0;  // tap / slab of the next B load
    auto loadB = [&](av_t* bh, av_t* bm, av_t* bl) {
      const lt* x = gl + j * GP + 16 * g;
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) {
        bh[ni] = *reinterpret_cast<const av_t*>(x + ni * 32 * GP);
        if constexpr (NPL == 3) {
          bm[ni] = *reinterpret_cast<const av_t*>(x + ni * 32 * GP + GPL);
          bl[ni] = *reinterpret_cast<const av_t*>(x + ni * 32 * GP + 2 * GPL);
        }
      }
      if (++j == k) {
        j = 0;
        ++g;
      }
    };
    loadA(wl, wstep, p.m_pad2, 0, total, a0);
    loadB(bh0, bm0, bl0);
    int s = 0;
    for (; s + 2 <= total; s += 2) {
      loadA(wl, wstep, p.m_pad2, s + 1, total, a1);
      loadB(bh1, bm1, bl1);
      __builtin_amdgcn_sched_barrier(0);
      mma(a0, bh0, bm0, bl0);
      __builtin_amdgcn_sched_barrier(0);
      loadA(wl, wstep, p.m_pad2, s + 2, total, a0);
      if (s + 2 < total) loadB(bh0, bm0, bl0);
      __builtin_amdgcn_sched_barrier(0);
      mma(a1, bh1, bm1, bl1);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (s < total) mma(a0, bh0, bm0, bl0);
  }

  // residual (+ accumulate / branch-mean division) epilogue, as the conv's
  // single-output STORE: every load of a 32 x 32 sub-tile issued first
  xt* const yb = reinterpret_cast<xt*>(p.y) + (int64_t)b * p.y_bstride;
#pragma unroll
  for (int mi = 0; mi < TM; ++mi) {
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) {
      const int col = wn + ni * 32 + l32;
      const int t = n0 + col;
      const bool st = col < BN && t < Tn;
      const int tc = st ? t : 0;
      float rv[16], yo[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wm + mi * 32 + 4 * lhi + (r & 3) + 8 * (r >> 2);
        rv[r] = (float)xb[(int64_t)row * p.x_cstride + tc];
      }
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
          const float v = acc[mi][ni][r] + erow[C + row];
          float o = rv[r] + v;  // (the conv's rv + res_scale * v, res_scale 1)
          if (p.accumulate) o = yo[r] + o;
          if (p.post_div != 1.0f) o = o / p.post_div;
          yb[(int64_t)row * p.y_cstride + t] = (xt)(t < L ? o : 0.f);
        }
      }
    }
  }
}

template <int C, int MODE = 0>
int rp_launch(const RpGroup& g, hipStream_t s) {
  int lds = 0, gx = 0;
  for (int i = 0; i < g.n; ++i) {
    const vits_resblock_pair_desc& d = g.d[i];
    const int l = rp_lds_bytes(C, d.k, d.dil, MODE);
    if (l > lds) lds = l;
    const int BN = rp_ng(C) - (d.k - 1);
    const int x = (d.t_len + BN - 1) / BN;
    if (x > gx) gx = x;
  }
  if (lds > 160 * 1024) return VITS_E_UNSUP;
  hipLaunchKernelGGL((resblock_f32p_kernel<C, MODE>), dim3(gx, 1, g.n * g.batch),
                     dim3(rp_threads(C)), lds, s, g);
  return vits_launch_status();
}

int rp_check(const vits_resblock_pair_desc& d, int mode = 0) {
  VITS_CHECK_ARG(d.x && d.w1 && d.w2 && d.y);
  // other workgroups still read x (halos, residual): never write in place
  VITS_CHECK_ARG(reinterpret_cast<const void*>(d.y) != reinterpret_cast<const void*>(d.x));
  VITS_CHECK_SHAPE(d.channels == 32 || d.channels == 64 || d.channels == 128 ||
                   d.channels == 256);
  VITS_CHECK_SHAPE(d.k >= 1 && d.k <= 15 && (d.k & 1) == 1 && d.dil >= 1 && d.t_len > 0);
  VITS_CHECK_SHAPE((d.k - 1) * d.dil <= 96);  // window within the staging units
  // images [cin_pad/16][k][2][3][m_pad][8] bf16, rows = C (c1 gate-interleaved / c2)
  VITS_CHECK_SHAPE(d.m_pad1 >= d.channels && d.m_pad2 >= d.channels && (d.m_pad1 & 3) == 0 &&
                   (d.m_pad2 & 3) == 0);
  VITS_CHECK_SHAPE(d.cin_pad1 >= d.channels && d.cin_pad2 >= d.channels / 2);
  // 4-step x staging (16 bytes fp32 / 8 bytes 16-bit): time-contiguous rows,
  // T % 4 == 0, aligned
  VITS_CHECK_SHAPE((d.t_len & 3) == 0 && (d.x_cstride & 3) == 0 && (d.x_bstride & 3) == 0 &&
                   d.x_cstride >= d.t_len && d.y_cstride >= d.t_len &&
                   (reinterpret_cast<uintptr_t>(d.x) & (mode ? 7 : 15)) == 0);
  // 32-bit staging offsets within one utterance
  VITS_CHECK_SHAPE((int64_t)d.channels * d.x_cstride < (1LL << 31));
  VITS_CHECK_SHAPE((reinterpret_cast<uintptr_t>(d.w1) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(d.w2) & 15) == 0);
  return VITS_OK;
}

}  // namespace

// the 16-bit models' 256-channel pairs (vits_resblock_pair16_forward routes
// them here: resblock16.hip stages whole windows, which a 256-channel window
// does not fit)
int vits_rp16_256(const vits_resblock_pair_desc* d, int n, int batch, int wdtype,
                  hipStream_t s) {
  if (!d || n < 1 || n > RP_GROUP || batch < 1) return VITS_E_ARG;
  if (wdtype != VITS_WDT_BF16 && wdtype != VITS_WDT_F16) return VITS_E_ARG;
  const int mode = wdtype == VITS_WDT_BF16 ? 1 : 2;
  RpGroup g;
  g.n = n;
  g.batch = batch;
  for (int i = 0; i < n; ++i) {
    const int rc = rp_check(d[i], mode);
    if (rc) return rc;
    if (d[i].channels != d[0].channels) return VITS_E_SHAPE;
    g.d[i] = d[i];
  }
  if (d[0].channels != 256) return VITS_E_SHAPE;
  return mode == 1 ? rp_launch<256, 1>(g, s) : rp_launch<256, 2>(g, s);
}

extern "C" int vits_resblock_pair_f32p_forward(const vits_resblock_pair_desc* d, int n, int batch,
                                               void* stream) {
  if (!d || n < 1 || n > RP_GROUP || batch < 1) return VITS_E_ARG;
  RpGroup g;
  g.n = n;
  g.batch = batch;
  for (int i = 0; i < n; ++i) {
    const int rc = rp_check(d[i]);
    if (rc) return rc;
    if (d[i].channels != d[0].channels) return VITS_E_SHAPE;
    g.d[i] = d[i];
  }
  hipStream_t s = as_stream(stream);
  int rc;
  if (d[0].channels == 32)
    rc = rp_launch<32>(g, s);
  else if (d[0].channels == 64)
    rc = rp_launch<64>(g, s);
  else if (d[0].channels == 128)
    rc = rp_launch<128>(g, s);
  else
    rc = rp_launch<256>(g, s);
  return count_ok(rc, VITS_CNT_RESBLOCK);
}
