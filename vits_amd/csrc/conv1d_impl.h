// conv1d_impl.h — the templated MFMA conv kernel and its launchers, shared
// by the per-operand-type translation units conv1d_{f32,bf16,f16}.hip (one
// instantiation set each, compiled in parallel).  See conv1d.hip for the
// design notes.
#pragma once
#include <type_traits>

#include "common.h"

#define VITS_PRIO(x) __builtin_amdgcn_s_setprio(x)

namespace vits_conv {


// internal epilogue variant: STORE with a second output descriptor (row split)
constexpr int EPI_STORE2 = 100;

struct OutDesc {
  float* y;
  int64_t y_bstride;
  int y_cstride;
  int act;
  const float* res;
  int64_t res_bstride;
  int res_cstride;
  float res_scale;
  int accumulate;
  float post_div;
};

__device__ __forceinline__ float apply_act(float v, int act) {
  if (act == VITS_ACT_RELU) return v > 0.f ? v : 0.f;
  if (act == VITS_ACT_TANH) return tanhf(v);
  if (act == VITS_ACT_EXP) return expf(v);
  return v;
}

// element access of an I/O tensor of type OT (float, or the 16-bit operand
// type for the IO16 kernels): OutDesc keeps float* fields, reinterpreted
template <typename OT>
__device__ __forceinline__ float ld_io(const float* base, int64_t i) {
  return (float)reinterpret_cast<const OT*>(base)[i];
}
template <typename OT>
__device__ __forceinline__ void st_io(float* base, int64_t i, float v) {
  reinterpret_cast<OT*>(base)[i] = (OT)v;
}

template <typename OT>
__device__ __forceinline__ void store_std(const OutDesc& o, int b, int ch, int t, float v,
                                          bool masked) {
  v = apply_act(v, o.act);
  if (o.res)
    v = ld_io<OT>(o.res, (int64_t)b * o.res_bstride + (int64_t)ch * o.res_cstride + t) +
        o.res_scale * v;
  const int64_t di = (int64_t)b * o.y_bstride + (int64_t)ch * o.y_cstride + t;
  if (o.accumulate) v = ld_io<OT>(o.y, di) + v;
  if (o.post_div != 1.0f) v = v / o.post_div;
  if (masked) v = 0.f;
  st_io<OT>(o.y, di, v);
}

// Register budget of the global->LDS prefetch (per thread): the host packs
// layers so that kc*k*BM <= VITS_W_TILE and kc*xw_pad <= VITS_X_TILE floats.
// W chunks go global->LDS by LDS-DMA (no registers); X chunks are staged
// through registers (zero padding + leaky-relu prologue on the way).
constexpr int VITS_W_TILE = 4096;
// X staging: element i of the chunk's [kc][xw_pad] window (LDS float i) is
// owned by thread i % 256; its (row, column) -> global offset mapping does
// not depend on the chunk, so it is computed once per workgroup.  The host
// keeps kc * xw_pad <= floats.
template <int BN, bool BF = false, bool IO16 = false>
struct XTile {
  // bf16-MFMA chunks carry >= 16 channels: a wider window budget; 16-bit
  // activations (IO16) stage 2 bytes per element, so twice the elements fit
  // the same registers (the training convs' 32- / 64-channel chunks)
  static constexpr int floats = IO16 ? (BN <= 128 ? 6144 : 10240)
                                     : BF ? (BN <= 128 ? 3072 : 5120) : (BN <= 128 ? 2048 : 4096);
  static constexpr int regs = floats / 256;
};
// bf16 W stage budget in float slots (2 bf16 each): k=11, kc=16, BM=64 fits
constexpr int VITS_W_TILE_BF = 6144;
// split-fp32 (VITS_WDT_F32S) W stage in floats: k=11, kc=16, BM=64 fits
constexpr int VITS_W_TILE_SPL = 11264;
// ... and with the W chunk pre-split through registers (128x128 tiles)
constexpr int VITS_W_TILE_WPS = 8192;
// split fp32 with the weights pre-split on the host (VITS_WDT_F32P): three
// bf16 planes [cin_pad/16][k][2][3][m_pad][8], the A fragments read straight
// from global memory (L2) into registers - W never enters LDS
constexpr int VITS_WDT_F32P_ = VITS_WDT_F32P;
// low-precision element type of weight type WT (VITS_WDT_BF16 / VITS_WDT_F16)
template <int WT>
struct LowP {
  typedef __bf16 T;  // (bf16, split fp32 and its pre-split planes)
};
template <>
struct LowP<VITS_WDT_F16> {
  typedef _Float16 T;
};
typedef __attribute__((address_space(3))) void* lds_void_t;

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x8_t __attribute__((ext_vector_type(8)));
// Exact three-term split of fp32 values into bf16: h = x truncated to bf16,
// m = (x - h) truncated, l = x - h - m (<= 8 significant bits, so exact in
// bf16).  Both subtractions are exact (they clear leading significand bits),
// hence x == h + m + l bit for bit.  Products of two terms have <= 16
// significant bits and are exact in the MFMA's fp32 products; the six terms
// kept (hh, hm, mh, mm, hl, lh) drop m*l' + l*m' + l*l' < 2^-22 |x||w|, the
// order of one fp32 rounding of the product.
__device__ __forceinline__ void split3_bf16(const f32x8_t& x, bf16x8_t& h, bf16x8_t& m,
                                            bf16x8_t& l) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    // (the element is copied out first: __builtin_bit_cast of an ext-vector
    // element expression reads element 0 on this compiler)
    const float xe = x[e];
    const float hf = __uint_as_float(__float_as_uint(xe) & 0xffff0000u);
    const float r = xe - hf;
    const float mf = __uint_as_float(__float_as_uint(r) & 0xffff0000u);
    // hf, mf are bf16 values already: the conversions are exact
    h[e] = (__bf16)hf;
    m[e] = (__bf16)mf;
    l[e] = (__bf16)(r - mf);
  }
}

typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void split3_bf16x4(const float __attribute__((ext_vector_type(4)))& x,
                                              bf16x4_t& h, bf16x4_t& m, bf16x4_t& l) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float xe = x[e];
    const float hf = __uint_as_float(__float_as_uint(xe) & 0xffff0000u);
    const float r = xe - hf;
    const float mf = __uint_as_float(__float_as_uint(r) & 0xffff0000u);
    h[e] = (__bf16)hf;
    m[e] = (__bf16)mf;
    l[e] = (__bf16)(r - mf);
  }
}

__device__ __forceinline__ float fast_sigmoid(float x) {
  return __builtin_amdgcn_rcpf(1.0f + __expf(-x));
}
__device__ __forceinline__ float fast_tanh(float x) {
  // tanh(x) = 2 sigmoid(2x) - 1 ; |err| ~ 1e-7 absolute
  return 2.0f * __builtin_amdgcn_rcpf(1.0f + __expf(-2.0f * x)) - 1.0f;
}

// Up to VITS_CONV_GROUP descriptors of one tile / epilogue / staging kind run
// as ONE launch (blockIdx.z = group member * batch + utterance): the three
// ResBlock2 branches of a Generator stage (k = 3, 7, 11) are independent
// until their mean, so their convs of one pair index share a grid - three
// times the workgroups of a single conv (the 256-channel stage alone is
// 1024 workgroups: 1.3 rounds of the chip's resident slots).
constexpr int VITS_CONV_GROUP = 3;
struct ConvGroup {
  vits_conv1d_desc d[VITS_CONV_GROUP];
  int n;      // members
  int batch;  // utterances per member
};

// IO16 (16-bit operand types only): x, residuals, gmask and the outputs are
// tensors of the operand type (the fp16-autocast training step keeps its
// activations in fp16, as the reference's autocast convs return them),
// half the bytes of the fp32-I/O kernel; accumulation stays fp32.
template <int BM, int BN, int WAVES_M, int WAVES_N, int EPI, int WT, bool V4, bool IO16 = false,
          bool GA = false>
__global__ __launch_bounds__(256, (WT == VITS_WDT_F32S || WT == VITS_WDT_F32P) ? 2 : 3) void conv1d_mfma_kernel(const ConvGroup G) {
  static_assert(!IO16 || WT != VITS_WDT_F32, "IO16 needs a 16-bit operand type");
  const int gi = (int)blockIdx.z / G.batch;
  const vits_conv1d_desc& p = G.d[gi];
  if ((int)blockIdx.x * BN >= p.n_out || (int)blockIdx.y * BM >= p.m) return;
  constexpr bool BF = WT != VITS_WDT_F32;  // 16-channel slab layout, 16-deep k-steps
  // split fp32: the slab layouts hold fp32 (LDS and W image), split into
  // three bf16 terms in registers per fragment (split3_bf16)
  // pre-split weights (VITS_WDT_F32P): the split-fp32 arithmetic with the A
  // fragments loaded from the host-split bf16 planes in global memory, one
  // k-step ahead, into registers; LDS holds only the X window, double
  // buffered (one barrier per chunk); kc == 16, one chunk = one 16-channel slab
  // GA (16-bit operand types): the same global-A structure on the packed
  // 16-bit image [cin_pad/16][k][2][m_pad][8] (one plane)
  static_assert(!GA || WT == VITS_WDT_BF16 || WT == VITS_WDT_F16, "GA: 16-bit types");
  constexpr bool WG = WT == VITS_WDT_F32P || GA;
  constexpr bool SPL = WT == VITS_WDT_F32S || WT == VITS_WDT_F32P;
  constexpr int WQ = SPL ? 8 : 4;  // float slots per (W row, 8 channels)
  // split fp32 on 128x128 tiles: the W chunk is staged pre-split as well
  // (three bf16 planes, one buffer; global -> registers under the MFMAs,
  // split and written between the chunk's two barriers), so the k-step
  // loop runs no VALU split; kc*k*BM <= VITS_W_TILE_WPS
  // (measured on MI355X: k=3 126 -> 137 TF/s on 128x128; no gain on 64x128,
  // whose 2-tap upsamplers lose 20 %)
  constexpr bool WPS = SPL && !WG && BM == 128 && BN == 128;
  constexpr int NWU = VITS_W_TILE_WPS / 8 / 256;  // 8-float W entries per thread
  typedef typename LowP<WT>::T lp_t;
  typedef lp_t lpx8 __attribute__((ext_vector_type(8)));
  typedef lp_t lpx4 __attribute__((ext_vector_type(4)));
  typedef typename std::conditional<IO16, lp_t, float>::type io_t;  // x / res / y element
  typedef typename std::conditional<SPL, float, lp_t>::type xe_t;   // slab-layout LDS element
  constexpr int WM = BM / WAVES_M;
  constexpr int WN = BN / WAVES_N;
  constexpr int TM = WM / 32;
  constexpr int TN = WN / 32;
  static_assert(WAVES_M * WAVES_N == 4, "4 waves per workgroup");
  static_assert(TM >= 1 && TN >= 1, "wave tile >= 32x32");

  extern __shared__ float smem[];
  const int kc = p.kc;
  const int k = p.k;
  const int dil = p.dil;
  const int xw = BN + (k - 1) * dil;
  const int xw_pad = (xw + 3) & ~3;
  const int wrows = kc * k;
  const int wsz = WG ? 0 : (BF && !SPL) ? wrows * BM / 2 : wrows * BM;  // W stage in float slots
  // X window geometry.  Scalar staging (any strides): rows of xw_pad
  // elements starting at column xstart.  V4 staging (time-contiguous rows,
  // 16-byte aligned, tin % 4 == 0): 16-byte blocks from the aligned column
  // xstart - xsh, rows of xrs = 4 * nb elements; the MFMA reads add xsh.
  const int xsh = V4 ? ((p.pad_left & 3) ? 4 - (p.pad_left & 3) : 0) : 0;  // (-pad_left) mod 4
  const int nb = (xw + xsh + 3) >> 2;       // V4: 16-byte blocks per window row
  const int xrs = V4 ? 4 * nb : xw_pad;     // window row length in LDS elements
  const int xsz = kc * xrs;                 // staged window elements
  // bf16 path: the window sits in LDS as bf16 [t][kc + 4] (channel-contiguous
  // per time step, 8-byte aligned rows) so a B fragment is two ds_read_b64
  const int kcp = kc + 4;
  // split fp32: the window is staged pre-split, three bf16 planes [t][kcp]
  // (hi, mid, lo) of xpl elements each, in ONE buffer [W0][W1][X] (the W
  // chunks stay double-buffered; the X chunk is written between two
  // barriers) - the planes cost 1.5x the fp32 bytes, a second X stage would
  // halve the workgroups per CU
  const int xpl = xrs * kcp;
  const int xslots = BF ? (SPL ? (3 * xpl + 1) / 2 : (xpl + 1) / 2) : xsz;  // LDS float slots
  // two stages: [W0][X0][W1][X1] (split fp32: [W0][W1][X])
  float* const stage0 = smem;
  float* const stage1 = SPL ? smem + wsz : smem + wsz + xslots;
  float* const xbuf1 = WG ? smem : WPS ? smem + 3 * wsz / 2 : SPL ? smem + 2 * wsz : stage0 + wsz;  // X of stage 0
  float* const xbuf2 = WG ? smem + xslots : SPL ? xbuf1 : stage1 + wsz;  // X of stage 1

  const int b = (int)blockIdx.z - gi * G.batch;
  const int n0 = blockIdx.x * BN;
  const int m0 = blockIdx.y * BM;
  if (p.lengths && p.len_skip > 0) {
    // bucketed infer: a tile starting past the utterance end + margin
    // neither computes nor writes (see vits_conv1d_desc.len_skip)
    const int tstart = EPI == VITS_EPI_UPSAMPLE ? n0 * p.up_u - p.up_pad : n0;
    if (tstart >= p.lengths[b] + p.len_skip) return;
  }
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  // the epilogue's per-row constants (bias + per-utterance cond) and the
  // utterance length, loaded now: their latency hides under the K loop
  // instead of opening the epilogue (measured within noise, -0.2..-0.6 %
  // over the decoder's shapes: profiles/r05_conv_prefetch_ab.txt)
  const int len_b = p.lengths ? p.lengths[b] : 0x7fffffff;
  const float* cond = p.cond ? p.cond + (int64_t)b * p.cond_bstride : nullptr;
  float pre_e = 0.f, pre_eb = 0.f;
  if (tid < BM) {
    const int row = m0 + tid;
    if (row < p.m) {
      int idx = row;
      if (EPI == VITS_EPI_GATE) idx = (row & 1) ? (p.m >> 1) + (row >> 1) : (row >> 1);
      if (EPI == VITS_EPI_UPSAMPLE) idx = row / p.up_u;
      if (p.bias) pre_eb = pre_e = p.bias[idx];
      if (cond && EPI != VITS_EPI_UPSAMPLE) pre_e += cond[idx];
    }
  }
  const int wm = (wid / WAVES_N) * WM;
  const int wn = (wid % WAVES_N) * WN;
  const int l32 = lane & 31;
  const int lhi = lane >> 5;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const io_t* xb = reinterpret_cast<const io_t*>(p.x) + (int64_t)b * p.x_bstride;
  const int64_t xts = p.x_tstride;
  const int xstart = n0 - p.pad_left - xsh;  // V4: a multiple of 4
  const float slope = p.in_slope;
  const bool act_in = slope != 1.0f;
  // (pre-split W, no W stage in LDS: the 16-bit activations' larger window
  // budget, i.e. 32-channel chunks on 128-column tiles)
  constexpr bool XB = IO16 || WT == VITS_WDT_F32P;
  constexpr int MAXX = XTile<BN, BF, XB>::regs;
  // T4 staging (16-bit activations, V4 rows): a unit is 4 channels x 4 time
  // steps - four 8-byte row loads, transposed in registers into four 8-byte
  // [t][4 channels] pieces, one ds_write_b64 each (the element-wise [t][c]
  // scatter of the other paths costs one ds_write_b16 per element).  Units
  // of a 16-lane group cover 4 channel quads x 4 time blocks: their LDS
  // pieces fall on distinct banks for kcp = 4 (mod 16) halves per row.
  constexpr bool T4 = V4 && (IO16 || SPL);
  constexpr int NU = T4 ? (XTile<BN, BF, XB>::floats / 16 + 48 + 255) / 256
                        : V4 ? MAXX / 4 : MAXX;  // staging units per thread
  constexpr int UW = V4 ? 4 : 1;            // elements per unit (per row)
  typedef float f32x4v __attribute__((ext_vector_type(4)));
  typedef typename std::conditional<IO16, lpx4, f32x4v>::type x4_t;  // 16-byte / 8-byte unit
  typedef typename std::conditional<SPL, f32x4v, lpx4>::type xe4_t;  // T4 LDS piece
  x4_t xreg4[V4 ? NU : 1][T4 ? 4 : 1];
  io_t xreg[V4 ? 1 : NU];
  int xrow[NU];  // window row of unit tid + 256q (1<<24 when it is padding)
  int xoff[NU];  // its global offset relative to row 0 of the chunk
  int xlds[T4 ? NU : 1];  // T4: the unit's LDS element offset ([t][kcp] image)
  const int nbq = (nb + 3) >> 2;
  const int nunits = T4 ? kc * nbq : V4 ? kc * nb : xsz;
  // window column -> element offset in an x row
  auto xcol = [&](int tt) -> int { return tt * (int)xts; };
#pragma unroll
  for (int q = 0; q < NU; ++q) {
    const int u = tid + q * 256;
    if constexpr (T4) {
      const int lo = u & 15, hi = u >> 4;
      const int hq = hi / nbq;
      const int cq = (lo & 3) + 4 * hq;                  // channel quad
      const int tb = (lo >> 2) + 4 * (hi - hq * nbq);    // 4-step time block
      const int tt = xstart + 4 * tb;
      const bool ok = u < nunits && tb < nb && tt >= 0 && tt < p.tin;
      xrow[q] = ok ? 4 * cq : (1 << 24);
      xoff[q] = ok ? 4 * cq * p.x_cstride + xcol(tt) : 0;
      xlds[q] = (u < nunits && tb < nb) ? 4 * tb * kcp + 4 * cq : -1;
    } else {
      const int per = V4 ? nb : xw_pad;
      const int r = u / per;
      const int c = u - r * per;
      const int t = c * UW;  // first window column of the unit
      const int tt = xstart + t;
      const bool ok = u < nunits && (V4 || t < xw) && tt >= 0 && tt < p.tin;
      xrow[q] = ok ? r : (1 << 24);
      xoff[q] = ok ? r * p.x_cstride + xcol(tt) : 0;
    }
  }

  // ---- W chunk: LDS-DMA, one 1 KiB piece (256 floats) per wave instruction;
  // lane l of piece q lands at LDS float q*256 + 4l (lane-linear image)
  const float inv_c8n = 1.0f / (float)(kc >> 3);
  auto wdma = [&](int c0, float* st) {
    // the chunk's W image is R rows of L float slots, HBM row stride S:
    //   f32:  [kc*k][BM] rows of W[c][j][m0..m0+BM)
    //   bf16: [k*kc/8][BM*8 bf16] rows of W[chunk][j][c8][m0..m0+BM][8]
    //   the packed image is [cin_pad/16][k][2][m_pad][8] (16-channel slabs)
    //   and a chunk of kc = 16 s channels is s slabs: LDS row (j, c8) of the
    //   [k][kc/8][BM][8] chunk image comes from slab c8/2, tap j, half c8&1
    const int L = BF ? BM * WQ : BM;
    const float* wsrc = BF ? p.w + ((int64_t)(c0 / 16) * k * 2 * p.m_pad + m0) * WQ
                           : p.w + (int64_t)c0 * k * p.m_pad + m0;
    const int64_t S = BF ? (int64_t)p.m_pad * WQ : p.m_pad;
    const int c8n = kc >> 3;
    const int pieces = (wsz + 255) >> 8;
    for (int q = wid; q < pieces; q += 4) {
      const int e = q * 256 + lane * 4;
      if (e < wsz) {
        const int r = e / L;  // (L a power-of-two constant: a shift)
        const int col = e - r * L;
        int gr = r;
        if (BF) {
          // r / c8n as a float product: r < 2^10 and c8n <= 8 keep
          // (r + 0.5) / c8n >= 1/16 from an integer, far above the product's
          // rounding, so the floor is exact - ~3 VALU instead of the ~12 of
          // the integer division, per piece of every chunk (the training
          // convs' chunk loop is VALU-bound)
          const int j = (int)(((float)r + 0.5f) * inv_c8n);
          const int c8 = r - j * c8n;
          gr = ((c8 >> 1) * k + j) * 2 + (c8 & 1);
        }
        __builtin_amdgcn_global_load_lds(wsrc + (int64_t)gr * S + col,
                                         (lds_void_t)(st + q * 256), 16, 0, 0);
      }
    }
  };
  // ---- W chunk, pre-split path (WPS): global -> registers; split into the
  // three bf16 planes [j][c8][BM][8] (plane stride wsz elements) in wstore
  f32x8_t wreg[WPS ? NWU : 1];
  const int nwe = kc * k * BM / 8;
  auto wgload = [&](int c0) {
    if constexpr (WPS) {
      typedef float f4 __attribute__((ext_vector_type(4)));
      const float* wsrc = p.w + ((int64_t)(c0 / 16) * k * 2 * p.m_pad + m0) * 8;
      const int c8n = kc >> 3;
#pragma unroll
      for (int q = 0; q < NWU; ++q) {
        if (q * 256 < nwe) {
          const int e0 = tid + q * 256;
          const int e = e0 < nwe ? e0 : 0;
          const int r = e / BM;
          const int ml = e - r * BM;
          const int j = r / c8n;
          const int c8 = r - j * c8n;
          const int gr = ((c8 >> 1) * k + j) * 2 + (c8 & 1);
          const f4* src = reinterpret_cast<const f4*>(wsrc + (int64_t)gr * p.m_pad * 8 + ml * 8);
          wreg[q] = __builtin_shufflevector(src[0], src[1], 0, 1, 2, 3, 4, 5, 6, 7);
        }
      }
    }
  };
  auto wstore = [&]() {
    if constexpr (WPS) {
      __bf16* wh = reinterpret_cast<__bf16*>(smem);
#pragma unroll
      for (int q = 0; q < NWU; ++q) {
        const int e = tid + q * 256;
        if (q * 256 < nwe && e < nwe) {
          bf16x8_t h, m, l;
          split3_bf16(wreg[q], h, m, l);
          *reinterpret_cast<bf16x8_t*>(wh + e * 8) = h;
          *reinterpret_cast<bf16x8_t*>(wh + wsz + e * 8) = m;
          *reinterpret_cast<bf16x8_t*>(wh + 2 * wsz + e * 8) = l;
        }
      }
    }
  };
  // ---- X chunk: global -> registers, raw.  Every lane issues its loads
  // unconditionally (padding lanes read the batch's first element) so the
  // compiler cannot tie a wait to each load: all MAXX loads stay in flight
  // under the chunk's MFMAs and are consumed in lstore.
  // first row of K-chunk c0
  auto chunk_base = [&](int c0) -> int64_t { return (int64_t)c0 * p.x_cstride; };
  auto gload = [&](int c0) {
    const io_t* base = xb + chunk_base(c0);
    const int lim = p.cin - c0;  // rows >= lim are channel padding
#pragma unroll
    for (int q = 0; q < NU; ++q) {
      if (q * 256 < nunits) {  // workgroup-uniform: no exec-mask branch
        if constexpr (T4) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const bool ok = xrow[q] + i < lim;
            const io_t* src = ok ? base + xoff[q] + i * p.x_cstride : xb;
            xreg4[q][i] = *reinterpret_cast<const x4_t*>(src);
          }
        } else {
          const bool ok = xrow[q] < lim;
          const io_t* src = ok ? base + xoff[q] : xb;
          if constexpr (V4)
            xreg4[q][0] = *reinterpret_cast<const x4_t*>(src);
          else
            xreg[q] = *src;
        }
      }
    }
  };
  // ---- registers -> LDS stage (zero padding + leaky-relu prologue) -----------
  auto lstore = [&](float* xs, int c0) {
    const int lim = p.cin - c0;
#pragma unroll
    for (int q = 0; q < NU; ++q) {
      if (q * 256 < nunits) {
        const int u = tid + q * 256;
        const bool ok = xrow[q] < lim;
        if constexpr (T4 && SPL) {
          if (xlds[q] >= 0) {
            f32x4v v[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const bool oki = xrow[q] + i < lim;
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                float t = xreg4[q][i][e];
                if (act_in) t = t < 0.f ? t * slope : t;
                v[i][e] = oki ? t : 0.f;
              }
            }
            __bf16* xh = reinterpret_cast<__bf16*>(xs) + xlds[q];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const f32x4v w = {v[0][e], v[1][e], v[2][e], v[3][e]};
              lpx4 h4, m4, l4;
              split3_bf16x4(w, h4, m4, l4);
              *reinterpret_cast<lpx4*>(xh + e * kcp) = h4;
              *reinterpret_cast<lpx4*>(xh + xpl + e * kcp) = m4;
              *reinterpret_cast<lpx4*>(xh + 2 * xpl + e * kcp) = l4;
            }
          }
        } else if constexpr (T4) {
          if (xlds[q] >= 0) {
            // rows i of the unit -> 4 time steps of 4 channels; padding rows
            // / blocks are zero, the leaky-relu prologue runs in fp32 (the
            // reference's autocast leaky_relu rounds once, from fp32)
            xe4_t v[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const bool oki = xrow[q] + i < lim;
              if (act_in) {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                  float t = (float)xreg4[q][i][e];
                  t = t < 0.f ? t * slope : t;
                  v[i][e] = (xe_t)(oki ? t : 0.f);
                }
              } else {
                v[i] = oki ? xreg4[q][i] : xe4_t{};
              }
            }
            xe_t* xh = reinterpret_cast<xe_t*>(xs) + xlds[q];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const xe4_t w = {v[0][e], v[1][e], v[2][e], v[3][e]};
              *reinterpret_cast<xe4_t*>(xh + e * kcp) = w;
            }
          }
        } else if (u < nunits) {
          if constexpr (V4) {
            f32x4v v;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              float t = (float)xreg4[q][0][e];
              if (act_in) t = t < 0.f ? t * slope : t;
              v[e] = ok ? t : 0.f;
            }
            const int r = u / nb;
            const int c = u - r * nb;
            if constexpr (BF) {
              xe_t* xh = reinterpret_cast<xe_t*>(xs);
#pragma unroll
              for (int e = 0; e < 4; ++e) xh[(4 * c + e) * kcp + r] = (xe_t)v[e];
            } else {
              *reinterpret_cast<f32x4v*>(xs + r * xrs + 4 * c) = v;
            }
          } else {
            float v = (float)xreg[q];
            if (act_in) v = v < 0.f ? v * slope : v;
            v = ok ? v : 0.f;
            if constexpr (SPL) {
              const int r = u / xw_pad;
              const int t = u - r * xw_pad;
              const float hf = __uint_as_float(__float_as_uint(v) & 0xffff0000u);
              const float rr = v - hf;
              const float mf = __uint_as_float(__float_as_uint(rr) & 0xffff0000u);
              __bf16* xh = reinterpret_cast<__bf16*>(xs) + t * kcp + r;
              xh[0] = (__bf16)hf;
              xh[xpl] = (__bf16)mf;
              xh[2 * xpl] = (__bf16)(rr - mf);
            } else if constexpr (BF) {
              const int r = u / xw_pad;
              const int t = u - r * xw_pad;
              reinterpret_cast<xe_t*>(xs)[t * kcp + r] = (xe_t)v;
            } else {
              xs[u] = v;
            }
          }
        }
      }
    }
  };

  const int nchunks = p.cin_pad / kc;
  const int half = kc >> 1;
  const int steps = k * half;  // MFMA k-steps per chunk

  if constexpr (WG) {
    // ---- W from global memory (VITS_WDT_F32P / GA) --------------------------
    // A chunk of kc = 16 G channels is G slabs; its k-steps run slab-major
    // (g, then tap j), so the flat step s = slab * k + j walks the weight
    // image contiguously: the A fragments of step s (plane q of NPL, row r,
    // half lhi) are the 16 bytes at
    //   w + ((s * 2 + lhi) * NPL + q) * m_pad * 8 + r * 8   (16-bit elements),
    // i.e. 32 consecutive rows = 512 contiguous bytes per load instruction.
    // NPL = 3 (F32P: hi / mid / lo planes, six MFMAs per fragment pair) or 1
    // (GA: the bf16 / fp16 image, one MFMA).
    constexpr int NPL = SPL ? 3 : 1;
    constexpr int NB = SPL ? TN : 1;  // (mid / lo B planes: split only)
    typedef lpx8 av_t;
    const int G = kc >> 4;
    const int nst = G * k;  // k-steps per chunk
    const int total = nchunks * nst;
    const lp_t* wbase = reinterpret_cast<const lp_t*>(p.w) +
                        ((int64_t)(lhi * NPL) * p.m_pad + m0 + wm + l32) * 8;
    const int64_t wstep = (int64_t)16 * NPL * p.m_pad;
    auto loadA = [&](int s, av_t (*a)[TM]) {
      const lp_t* wp = wbase + (int64_t)(s < total ? s : total - 1) * wstep;
#pragma unroll
      for (int q = 0; q < NPL; ++q)
#pragma unroll
        for (int mi = 0; mi < TM; ++mi)
          a[q][mi] = *reinterpret_cast<const av_t*>(wp + ((int64_t)q * p.m_pad + mi * 32) * 8);
    };
    // B fragments of tap j, slab g of the chunk: rows wn + ni*32 + l32 + j*dil
    // of the [t][kcp] window plane(s), channels 16 g + 8 lhi .. + 8
    const lp_t* const xlane0 = reinterpret_cast<const lp_t*>(xbuf1) +
                               (wn + l32 + xsh) * kcp + 8 * lhi;
    const int xdelta = (int)(reinterpret_cast<const lp_t*>(xbuf2) -
                             reinterpret_cast<const lp_t*>(xbuf1));
    auto loadB = [&](int buf, int j, int g, av_t* bh, av_t* bm, av_t* bl) {
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) {
        const lpx4* xp = reinterpret_cast<const lpx4*>(
            xlane0 + buf * xdelta + (ni * 32 + j * dil) * kcp + 16 * g);
        bh[ni] = __builtin_shufflevector(xp[0], xp[1], 0, 1, 2, 3, 4, 5, 6, 7);
        if constexpr (SPL) {
          const int P4 = xpl / 4;  // plane stride in 8-byte pieces
          bm[ni] = __builtin_shufflevector(xp[P4], xp[P4 + 1], 0, 1, 2, 3, 4, 5, 6, 7);
          bl[ni] = __builtin_shufflevector(xp[2 * P4], xp[2 * P4 + 1], 0, 1, 2, 3, 4, 5, 6, 7);
        }
      }
    };
    // split: the same six products in the same order as the F32S path
    // (bitwise the same result): small terms first
    auto mma = [&](av_t (*a)[TM], const av_t* bh, const av_t* bm, const av_t* bl) {
#pragma unroll
      for (int mi = 0; mi < TM; ++mi)
#pragma unroll
        for (int ni = 0; ni < TN; ++ni) {
          f32x16 c = acc[mi][ni];
          if constexpr (SPL) {
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][mi], bl[ni], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2][mi], bh[ni], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][mi], bm[ni], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][mi], bm[ni], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][mi], bh[ni], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][mi], bh[ni], c, 0, 0, 0);
          } else if constexpr (WT == VITS_WDT_F16) {
            c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0][mi], bh[ni], c, 0, 0, 0);
          } else {
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][mi], bh[ni], c, 0, 0, 0);
          }
          acc[mi][ni] = c;
        }
    };
    if constexpr (!SPL && V4 && BN <= 128) {
      // GA: one MFMA per fragment pair leaves TM * TN MFMAs (~128 cycles)
      // between a step's A load and its use - less than an L2 round trip.
      // The A fragments run PF - 1 steps ahead in a register ring instead
      // (ring slot = step % PF within a chunk; the chunk's last nst % PF
      // steps leave the ring rotated, which a switch undoes).  C5 trace
      // (profiles/r05_gapf_*): WN in_layer convs 714 -> 672 us, upsamplers
      // 716 -> 700 us per step.  Only the 16-byte-staged 128-column tiles:
      // the element-staged and 256-column ones reach 168 VGPRs and spill.
      constexpr int PF = 4;
      static_assert(PF == 2 || PF == 4, "ring parity");
      av_t ar[PF][1][TM];
      av_t bb[2][TN];
#pragma unroll
      for (int i = 0; i < PF - 1; ++i) loadA(i, ar[i]);
      gload(0);
      lstore(xbuf1, 0);
      __syncthreads();
      for (int ch = 0; ch < nchunks; ++ch) {
        const bool more = ch + 1 < nchunks;
        if (more) gload((ch + 1) * kc);  // in flight under this chunk's MFMAs
        const int buf = ch & 1;
        const int s0 = ch * nst;
        int j = 0, g = 0;
        auto next = [&]() {
          if (++j == k) {
            j = 0;
            ++g;
          }
        };
        loadB(buf, 0, 0, bb[0], nullptr, nullptr);
        int st = 0;
        for (; st + PF <= nst; st += PF) {
#pragma unroll
          for (int u = 0; u < PF; ++u) {
            loadA(s0 + st + u + PF - 1, ar[(u + PF - 1) % PF]);
            next();
            if (st + u + 1 < nst) loadB(buf, j, g, bb[(u + 1) & 1], nullptr, nullptr);
            __builtin_amdgcn_sched_barrier(0);
            mma(ar[u], bb[u & 1], nullptr, nullptr);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
        const int r = nst - st;  // 0 .. PF - 1 steps left
#pragma unroll
        for (int u = 0; u < PF - 1; ++u) {
          if (u < r) {
            loadA(s0 + st + u + PF - 1, ar[(u + PF - 1) % PF]);
            next();
            if (st + u + 1 < nst) loadB(buf, j, g, bb[(u + 1) & 1], nullptr, nullptr);
            __builtin_amdgcn_sched_barrier(0);
            mma(ar[u], bb[u & 1], nullptr, nullptr);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
        // the next chunk's first PF - 1 steps sit in slots r .. r + PF - 2
        // (mod PF): move them to 0 .. PF - 2
        auto rot = [&](auto R) {
          constexpr int rr = decltype(R)::value;
          av_t t[PF - 1][TM];
#pragma unroll
          for (int i = 0; i < PF - 1; ++i)
#pragma unroll
            for (int mi = 0; mi < TM; ++mi) t[i][mi] = ar[(i + rr) % PF][0][mi];
#pragma unroll
          for (int i = 0; i < PF - 1; ++i)
#pragma unroll
            for (int mi = 0; mi < TM; ++mi) ar[i][0][mi] = t[i][mi];
        };
        if (r == 1) rot(std::integral_constant<int, 1>());
        if constexpr (PF > 2) {
          if (r == 2) rot(std::integral_constant<int, 2>());
        }
        if constexpr (PF > 3) {
          if (r == 3) rot(std::integral_constant<int, 3>());
        }
        if (more) lstore(buf ? xbuf1 : xbuf2, (ch + 1) * kc);
        __syncthreads();
      }
    } else {
    av_t a0[NPL][TM], a1[NPL][TM];
    av_t bh0[TN], bm0[NB], bl0[NB], bh1[TN], bm1[NB], bl1[NB];
    loadA(0, a0);
    gload(0);
    lstore(xbuf1, 0);
    __syncthreads();
    for (int ch = 0; ch < nchunks; ++ch) {
      const bool more = ch + 1 < nchunks;
      if (more) gload((ch + 1) * kc);  // in flight under this chunk's MFMAs
      const int buf = ch & 1;
      const int s0 = ch * nst;
      // (j, g) of step st; next() advances it: taps fastest, then slabs
      int j = 0, g = 0;
      auto next = [&]() {
        if (++j == k) {
          j = 0;
          ++g;
        }
      };
      loadB(buf, 0, 0, bh0, bm0, bl0);
      int st = 0;
      // the loads of step st + 1 are pinned ahead of step st's MFMAs
      // (sched_barrier): left alone, the scheduler sinks the global A loads
      // into the middle of the MFMA block and the next block then waits on
      // them (measured: ~12 MFMAs of cover instead of 24)
      for (; st + 2 <= nst; st += 2) {
        next();
        loadA(s0 + st + 1, a1);
        loadB(buf, j, g, bh1, bm1, bl1);
        __builtin_amdgcn_sched_barrier(0);
        mma(a0, bh0, bm0, bl0);
        __builtin_amdgcn_sched_barrier(0);
        next();
        loadA(s0 + st + 2, a0);  // (st + 2 == nst: the next chunk's first step)
        if (st + 2 < nst) loadB(buf, j, g, bh0, bm0, bl0);
        __builtin_amdgcn_sched_barrier(0);
        mma(a1, bh1, bm1, bl1);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (st < nst) {  // odd step count: the last step, and the next chunk's A
        loadA(s0 + nst, a1);
        __builtin_amdgcn_sched_barrier(0);
        mma(a0, bh0, bm0, bl0);
#pragma unroll
        for (int q = 0; q < NPL; ++q)
#pragma unroll
          for (int mi = 0; mi < TM; ++mi) a0[q][mi] = a1[q][mi];
      }
      if (more) lstore(buf ? xbuf1 : xbuf2, (ch + 1) * kc);
      __syncthreads();
    }
    }  // (GA ring / one step ahead)
  } else {

  if constexpr (WPS)
    wgload(0);
  else
    wdma(0, stage0);
  gload(0);
  wstore();
  lstore(xbuf1, 0);
  __syncthreads();

  for (int ch = 0; ch < nchunks; ++ch) {
    float* cur = (ch & 1) ? stage1 : stage0;
    float* nxt = (ch & 1) ? stage0 : stage1;
    const bool more = ch + 1 < nchunks;
    if (more) {  // both in flight under the MFMAs below
      if constexpr (WPS)
        wgload((ch + 1) * kc);
      else
        wdma((ch + 1) * kc, nxt);
      gload((ch + 1) * kc);
    }

    const float* ws = WPS ? smem : cur;  // (WPS: one W buffer)
    const float* xs = (ch & 1) ? xbuf2 : xbuf1;
    if constexpr (WPS) {
      // both operands pre-split in LDS: A = one 16-byte read per plane of
      // the W planes [j][c8][row][8], B as below; six MFMAs per (mi, ni)
      const __bf16* wh = reinterpret_cast<const __bf16*>(ws);
      const int c8n = kc >> 3;
      const int G = kc >> 4;
      const int nsteps = k * G;
      auto load = [&](int st, bf16x8_t* ah, bf16x8_t* am, bf16x8_t* al, bf16x8_t* bh,
                      bf16x8_t* bm, bf16x8_t* bl) {
        const int j = st / G;
        const int g = st - j * G;
#pragma unroll
        for (int mi = 0; mi < TM; ++mi) {
          const bf16x8_t* ap = reinterpret_cast<const bf16x8_t*>(
              wh + ((j * c8n + 2 * g + lhi) * BM + wm + mi * 32 + l32) * 8);
          ah[mi] = ap[0];
          am[mi] = ap[wsz / 8];
          al[mi] = ap[wsz / 4];
        }
#pragma unroll
        for (int ni = 0; ni < TN; ++ni) {
          const lpx4* xp = reinterpret_cast<const lpx4*>(
              reinterpret_cast<const __bf16*>(xs) + (wn + ni * 32 + l32 + j * dil + xsh) * kcp +
              16 * g + 8 * lhi);
          const int P4 = xpl / 4;
          bh[ni] = __builtin_shufflevector(xp[0], xp[1], 0, 1, 2, 3, 4, 5, 6, 7);
          bm[ni] = __builtin_shufflevector(xp[P4], xp[P4 + 1], 0, 1, 2, 3, 4, 5, 6, 7);
          bl[ni] = __builtin_shufflevector(xp[2 * P4], xp[2 * P4 + 1], 0, 1, 2, 3, 4, 5, 6, 7);
        }
      };
      auto mma = [&](const bf16x8_t* ah, const bf16x8_t* am, const bf16x8_t* al,
                     const bf16x8_t* bh, const bf16x8_t* bm, const bf16x8_t* bl) {
#pragma unroll
        for (int mi = 0; mi < TM; ++mi)
#pragma unroll
          for (int ni = 0; ni < TN; ++ni) {
            f32x16 c = acc[mi][ni];
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[mi], bl[ni], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[mi], bh[ni], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[mi], bm[ni], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[mi], bm[ni], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[mi], bh[ni], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[mi], bh[ni], c, 0, 0, 0);
            acc[mi][ni] = c;
          }
      };
      bf16x8_t ah0[TM], am0[TM], al0[TM], bh0[TN], bm0[TN], bl0[TN];
      bf16x8_t ah1[TM], am1[TM], al1[TM], bh1[TN], bm1[TN], bl1[TN];
      load(0, ah0, am0, al0, bh0, bm0, bl0);
      int st = 0;
      for (; st + 2 <= nsteps; st += 2) {
        load(st + 1, ah1, am1, al1, bh1, bm1, bl1);
        mma(ah0, am0, al0, bh0, bm0, bl0);
        load(st + 2, ah0, am0, al0, bh0, bm0, bl0);
        mma(ah1, am1, al1, bh1, bm1, bl1);
      }
      if (st < nsteps) mma(ah0, am0, al0, bh0, bm0, bl0);
    } else if constexpr (SPL) {
      // k-step = (tap j, 16 channels) as in the 16-bit path below, on fp32
      // slabs: A = two 16-byte reads of W image [j][c8][row][8], B = two of
      // the [t][kcp] window; each fragment split into three bf16 terms, six
      // MFMAs per (mi, ni)
      const char* wbytes = reinterpret_cast<const char*>(ws);
      const int c8n = kc >> 3;
      const int G = kc >> 4;
      const int nsteps = k * G;
      typedef float f4 __attribute__((ext_vector_type(4)));
      auto load = [&](int st, f32x8_t* a, bf16x8_t* bh, bf16x8_t* bm, bf16x8_t* bl) {
        const int j = st / G;
        const int g = st - j * G;
#pragma unroll
        for (int mi = 0; mi < TM; ++mi) {
          const f4* ap = reinterpret_cast<const f4*>(
              wbytes + ((int64_t)((j * c8n + 2 * g + lhi) * BM + wm + mi * 32 + l32) << 5));
          a[mi] = __builtin_shufflevector(ap[0], ap[1], 0, 1, 2, 3, 4, 5, 6, 7);
        }
#pragma unroll
        for (int ni = 0; ni < TN; ++ni) {
          const lpx4* xp = reinterpret_cast<const lpx4*>(
              reinterpret_cast<const __bf16*>(xs) + (wn + ni * 32 + l32 + j * dil + xsh) * kcp +
              16 * g + 8 * lhi);
          const int P4 = xpl / 4;  // plane stride in 8-byte pieces
          bh[ni] = __builtin_shufflevector(xp[0], xp[1], 0, 1, 2, 3, 4, 5, 6, 7);
          bm[ni] = __builtin_shufflevector(xp[P4], xp[P4 + 1], 0, 1, 2, 3, 4, 5, 6, 7);
          bl[ni] = __builtin_shufflevector(xp[2 * P4], xp[2 * P4 + 1], 0, 1, 2, 3, 4, 5, 6, 7);
        }
      };
      auto mma = [&](const f32x8_t* a, const bf16x8_t* bh, const bf16x8_t* bm,
                     const bf16x8_t* bl) {
        bf16x8_t ah[TM], am[TM], al[TM];
#pragma unroll
        for (int mi = 0; mi < TM; ++mi) split3_bf16(a[mi], ah[mi], am[mi], al[mi]);
        // small terms first
#pragma unroll
        for (int mi = 0; mi < TM; ++mi)
#pragma unroll
          for (int ni = 0; ni < TN; ++ni) {
            f32x16 c = acc[mi][ni];
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[mi], bl[ni], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[mi], bh[ni], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[mi], bm[ni], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[mi], bm[ni], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[mi], bh[ni], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[mi], bh[ni], c, 0, 0, 0);
            acc[mi][ni] = c;
          }
      };
      f32x8_t a0[TM], a1[TM];
      bf16x8_t bh0[TN], bm0[TN], bl0[TN], bh1[TN], bm1[TN], bl1[TN];
      load(0, a0, bh0, bm0, bl0);
      int st = 0;
      for (; st + 2 <= nsteps; st += 2) {
        load(st + 1, a1, bh1, bm1, bl1);
        mma(a0, bh0, bm0, bl0);
        load(st + 2, a0, bh0, bm0, bl0);
        mma(a1, bh1, bm1, bl1);
      }
      if (st < nsteps) mma(a0, bh0, bm0, bl0);
    } else if constexpr (BF) {
      // k-step = (tap j, 16 channels): A = one 16-byte read per 32-row
      // fragment of the W image [j][c8][row][8], B = 8 channels of the
      // [t][kcp] window at column n + j*dil.  A of step st = (j, group g),
      // g fastest, sits at image row j * c8n + 2 g + lhi = 2 st + lhi
      // (c8n = 2 G): linear in st.  B's window offset j * dil * kcp + 16 g
      // is advanced incrementally (no division by G in the loop), and the
      // loads of step st + 1 are pinned ahead of step st's MFMAs
      // (sched_barrier), as on the GA path
      const char* wlane = reinterpret_cast<const char*>(ws) +
                          ((int64_t)(lhi * BM + wm + l32) << 4);
      const lp_t* xlane = reinterpret_cast<const lp_t*>(xs) + (wn + l32 + xsh) * kcp + 8 * lhi;
      const int G = kc >> 4;       // 16-channel groups per tap
      const int nsteps = k * G;    // k-steps of this chunk
      const int jstep = dil * kcp - 16 * (G - 1);
      int boff = 0, g = 0;         // B offset / group of the next load
      auto load = [&](int st, lpx8* a, lpx8* bb) {
#pragma unroll
        for (int mi = 0; mi < TM; ++mi)
          a[mi] = *reinterpret_cast<const lpx8*>(wlane + ((int64_t)(2 * st * BM + mi * 32) << 4));
#pragma unroll
        for (int ni = 0; ni < TN; ++ni) {
          const lp_t* xp = xlane + boff + ni * 32 * kcp;
          const lpx4 lo = *reinterpret_cast<const lpx4*>(xp);
          const lpx4 hi = *reinterpret_cast<const lpx4*>(xp + 4);
          bb[ni] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        }
        if (++g == G) {
          g = 0;
          boff += jstep;
        } else {
          boff += 16;
        }
      };
      auto mma = [&](const lpx8* a, const lpx8* bb) {
#pragma unroll
        for (int mi = 0; mi < TM; ++mi)
#pragma unroll
          for (int ni = 0; ni < TN; ++ni)
            if constexpr (WT == VITS_WDT_F16)
              acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[mi], bb[ni], acc[mi][ni], 0, 0, 0);
            else
              acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[mi], bb[ni], acc[mi][ni], 0, 0, 0);
      };
      // two register sets: the fragments of step s+1 are read under the
      // MFMAs of step s (the read past the last step stays inside the
      // stage's padded LDS and is never consumed)
      lpx8 a0[TM], b0[TN], a1[TM], b1[TN];
      // no scalar load may be pending when the loop starts: SMEM returns out
      // of order with LDS, and the waitcnt pass would then wait for ALL LDS
      // reads (lgkmcnt(0)) at each step's first MFMA instead of leaving the
      // next step's TM + TN reads in flight
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0), vmcnt / expcnt untouched
      load(0, a0, b0);
      int st = 0;
      // each step first waits for its own fragments (issued a whole MFMA
      // block earlier, so normally landed), then issues the next step's
      // reads, then its MFMAs: left to itself the waitcnt pass put an
      // lgkmcnt(0) AFTER the next step's reads, i.e. no LDS latency cover
      for (; st + 2 <= nsteps; st += 2) {
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
        load(st + 1, a1, b1);
        __builtin_amdgcn_sched_barrier(0);
        mma(a0, b0);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_waitcnt(0xc07f);
        load(st + 2, a0, b0);
        __builtin_amdgcn_sched_barrier(0);
        mma(a1, b1);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (st < nsteps) mma(a0, b0);
    } else {
      // k-step s = (tap j, channel pair cp), cp fastest: A rows (2cp + lhi)*k + j
      // of W, B row 2cp + lhi of X shifted by j*dil.  Two register sets ping-
      // pong so the LDS reads of step s+1 are in flight under the MFMAs of s;
      // the read after the last step runs past the chunk into padded LDS and
      // is never consumed.
      const float* wa = ws + lhi * k * BM + wm + l32;
      const float* xa = xs + lhi * xrs + wn + l32 + xsh;
      const int sa = 2 * k * BM;
      const int sb = 2 * xrs;
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
          pa = wa + j * BM;
          pb = xa + j * dil;
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
        VITS_PRIO(1);
  #pragma unroll
        for (int mi = 0; mi < TM; ++mi)
  #pragma unroll
          for (int ni = 0; ni < TN; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[mi], b0[ni], acc[mi][ni], 0, 0, 0);
        VITS_PRIO(0);
  #pragma unroll
        for (int mi = 0; mi < TM; ++mi) a0[mi] = pa[mi * 32];
  #pragma unroll
        for (int ni = 0; ni < TN; ++ni) b0[ni] = pb[ni * 32];
        advance();
        VITS_PRIO(1);
  #pragma unroll
        for (int mi = 0; mi < TM; ++mi)
  #pragma unroll
          for (int ni = 0; ni < TN; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[mi], b1[ni], acc[mi][ni], 0, 0, 0);
        VITS_PRIO(0);
      }
      if (s < steps) {
  #pragma unroll
        for (int mi = 0; mi < TM; ++mi)
  #pragma unroll
          for (int ni = 0; ni < TN; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[mi], b0[ni], acc[mi][ni], 0, 0, 0);
      }
    }
    if constexpr (SPL) {
      __syncthreads();  // every wave is done with the (single) X buffer
      if (more) {
        wstore();  // (WPS: the single W buffer too)
        lstore(xbuf1, (ch + 1) * kc);
      }
    } else {
      if (more) lstore(nxt + wsz, (ch + 1) * kc);
    }
    __syncthreads();
  }
  }  // !WG

  // ---- epilogue -----------------------------------------------------------
  OutDesc o0{p.out0.y, p.out0.y_bstride, p.out0.y_cstride, p.out0.act, p.out0.res,
             p.out0.res_bstride, p.out0.res_cstride, p.out0.res_scale, p.out0.accumulate,
             p.out0.post_div};
  // per-row additive constant (bias + per-utterance cond) of this tile's BM
  // rows (loaded by BM threads before the K loop) into LDS: the stages are
  // free after the last barrier of the K loop
  float* const erow = smem;
  // GATE with a pre-activation output (out1.y: the training gate's saved
  // input, bias but no cond, as the reference's in_layer output x_in)
  float* const ebias = smem + BM;
  const bool gate_pre = EPI == VITS_EPI_GATE && p.out1.y != nullptr;
  if (tid < BM) {
    erow[tid] = pre_e;
    if (EPI == VITS_EPI_GATE) ebias[tid] = pre_eb;
  }
  __syncthreads();

  if constexpr (EPI == VITS_EPI_UPSAMPLE) {
    // Polyphase output row = oc * u + phase lands at time n * u + phase - pad:
    // stored from the MFMA layout, each store instruction writes 32 samples
    // at stride u (C5 probe: 160 us of the four upsamplers' 716 per step).
    // A plain store (no act / residual / accumulate / division - every
    // upsampler) goes through LDS instead: the tile [BM][BN + 2] (io_t, the
    // value rounded once, as st_io does), then each channel's contiguous run
    // of BN * u samples with consecutive threads on consecutive samples.
    // C5 trace: the four upsamplers 729 -> 657 us per step; headline
    // 20.16 -> 20.03 ms (profiles/r05_uplds_*).
    if (o0.act == VITS_ACT_NONE && !o0.res && !o0.accumulate && o0.post_div == 1.0f) {
      constexpr int TP = BN + 2;
      io_t* const tile = reinterpret_cast<io_t*>(smem + BM);
#pragma unroll
      for (int mi = 0; mi < TM; ++mi)
#pragma unroll
        for (int ni = 0; ni < TN; ++ni) {
          const int col = wn + ni * 32 + l32;
          const int rloc = wm + mi * 32 + 4 * lhi;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int ro = rloc + (r & 3) + 8 * (r >> 2);
            tile[ro * TP + col] = (io_t)(acc[mi][ni][r] + erow[ro]);
          }
        }
      __syncthreads();
      const int u = p.up_u;
      const float inv_u = 1.0f / (float)u;  // (exact floor for j < 2^14, u <= 64)
      const int oc0 = m0 / u;
      const int oc1 = min((m0 + BM - 1) / u, p.m / u - 1);
      const int span = BN * u;
      const int tb = n0 * u - p.up_pad;  // time of j = 0
      io_t* const yb = reinterpret_cast<io_t*>(o0.y) + (int64_t)b * o0.y_bstride;
      for (int oc = oc0; oc <= oc1; ++oc) {
        io_t* const yc = yb + (int64_t)oc * o0.y_cstride;
        const int rb = oc * u - m0;  // tile row of phase 0
        for (int j = tid; j < span; j += 256) {
          const int nl = (int)(((float)j + 0.5f) * inv_u);
          const int ph = j - nl * u;
          const int rl = rb + ph;
          const int t = tb + j;
          if (rl >= 0 && rl < BM && n0 + nl < p.n_out && t >= 0 && t < p.t_out)
            yc[t] = t >= len_b ? (io_t)0.f : tile[rl * TP + nl];
        }
      }
      return;
    }
  }

#pragma unroll
  for (int mi = 0; mi < TM; ++mi) {
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) {
      const int n = n0 + wn + ni * 32 + l32;
      const int rloc = wm + mi * 32 + 4 * lhi;  // tile-local row of register 0
      const int rbase = m0 + rloc;
      if (EPI == VITS_EPI_GATE) {
        // packed rows 2q (tanh half) / 2q+1 (sigmoid half) live in the same
        // lane in registers r, r+1 (r even): no cross-lane traffic.
        if (n < p.n_out) {
#pragma unroll
          for (int r = 0; r < 16; r += 2) {
            const int ro = (r & 3) + 8 * (r >> 2);
            const int row = rbase + ro;
            if (row < p.m) {
              const float va = acc[mi][ni][r] + erow[rloc + ro];
              const float vb = acc[mi][ni][r + 1] + erow[rloc + ro + 1];
              const float v = fast_tanh(va) * fast_sigmoid(vb);
              store_std<io_t>(o0, b, row >> 1, n, v, n >= len_b);
              if (gate_pre) {
                const bool mk = n >= len_b;
                const int64_t pb = (int64_t)b * p.out1.y_bstride + n;
                const float xa = mk ? 0.f : acc[mi][ni][r] + ebias[rloc + ro];
                const float xb = mk ? 0.f : acc[mi][ni][r + 1] + ebias[rloc + ro + 1];
                st_io<io_t>(p.out1.y, pb + (int64_t)(row >> 1) * p.out1.y_cstride, xa);
                st_io<io_t>(p.out1.y, pb + (int64_t)((p.m >> 1) + (row >> 1)) * p.out1.y_cstride,
                            xb);
              }
            }
          }
        }
      } else if (EPI == VITS_EPI_UPSAMPLE) {
        const int u = p.up_u;
        // row / u without the integer-division sequence per element:
        // (row + 0.5) / u lies >= 0.5/u from an integer, and for rows < 2^14
        // and u <= 64 (checked on the host) the fp32 product's error is
        // below that, so its floor is exact
        const float inv_u = 1.0f / (float)u;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int ro = (r & 3) + 8 * (r >> 2);
          const int row = rbase + ro;
          if (row < p.m && n < p.n_out) {
            const int oc = (int)(((float)row + 0.5f) * inv_u);
            const int ph = row - oc * u;
            const int t = n * u + ph - p.up_pad;
            if (t >= 0 && t < p.t_out) {
              const float v = acc[mi][ni][r] + erow[rloc + ro];
              store_std<io_t>(o0, b, oc, t, v, t >= len_b);
            }
          }
        }
      } else if (EPI == EPI_STORE2) {
        OutDesc o1{p.out1.y, p.out1.y_bstride, p.out1.y_cstride, p.out1.act, p.out1.res,
                   p.out1.res_bstride, p.out1.res_cstride, p.out1.res_scale,
                   p.out1.accumulate, p.out1.post_div};
        // the 16 rows of a 32x32 sub-tile lie in one 32-row block: when that
        // block is on one side of the split (split % 32 == 0: every WN
        // res_skip layer), every residual / accumulator load of the
        // sub-tile is issued before the first store (store_std per element
        // waited one memory round trip per row)
        const int blk = rbase - 4 * lhi;
        if (n < p.n_out && (blk + 32 <= p.split || blk >= p.split)) {
          const bool s1 = blk >= p.split;
          const OutDesc& o = s1 ? o1 : o0;
          const int cofs = s1 ? p.split : 0;
          float v[16], rv[16], yo[16];
#pragma unroll
          for (int r = 0; r < 16; ++r)
            v[r] = apply_act(acc[mi][ni][r] + erow[rloc + (r & 3) + 8 * (r >> 2)], o.act);
          const int64_t rb = (int64_t)b * o.res_bstride + n;
          const int64_t yb = (int64_t)b * o.y_bstride + n;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = rbase + (r & 3) + 8 * (r >> 2);
            const int ch = row < p.m ? row - cofs : 0;
            rv[r] = o.res ? ld_io<io_t>(o.res, rb + (int64_t)ch * o.res_cstride) : 0.f;
            yo[r] = o.accumulate ? ld_io<io_t>(o.y, yb + (int64_t)ch * o.y_cstride) : 0.f;
          }
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = rbase + (r & 3) + 8 * (r >> 2);
            float t = v[r];
            if (o.res) t = rv[r] + o.res_scale * t;
            if (o.accumulate) t = yo[r] + t;
            if (o.post_div != 1.0f) t = t / o.post_div;
            if (n >= len_b) t = 0.f;
            if (row < p.m) st_io<io_t>(o.y, yb + (int64_t)(row - cofs) * o.y_cstride, t);
          }
        } else if (n < p.n_out) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int ro = (r & 3) + 8 * (r >> 2);
            const int row = rbase + ro;
            if (row < p.m) {
              const float v = acc[mi][ni][r] + erow[rloc + ro];
              if (row < p.split)
                store_std<io_t>(o0, b, row, n, v, n >= len_b);
              else
                store_std<io_t>(o1, b, row - p.split, n, v, n >= len_b);
            }
          }
        }
      } else {
        // single-output STORE: every residual / accumulator load of this
        // 32x32 sub-tile is issued before the first store, so the 16 round
        // trips overlap (res may alias y: each element is still read before
        // it is written, by the same lane).
        const int ncol = n;
        if (n < p.n_out) {
          // (row blocks of RH: 8 would halve the temporaries of tiles with 8
          // live accumulator sub-tiles)
          constexpr int RH = 16;
#pragma unroll
          for (int r0 = 0; r0 < 16; r0 += RH) {
          float v[RH];
#pragma unroll
          for (int i = 0; i < RH; ++i) {
            const int r = r0 + i;
            v[i] = apply_act(acc[mi][ni][r] + erow[rloc + (r & 3) + 8 * (r >> 2)], o0.act);
          }
          if (p.gmask) {  // leaky-relu derivative of the forward input
            const int64_t gb = (int64_t)b * p.gmask_bstride + ncol;
            float gv[RH];
#pragma unroll
            for (int i = 0; i < RH; ++i) {
              const int r = r0 + i;
              const int row = rbase + (r & 3) + 8 * (r >> 2);
              gv[i] = ld_io<io_t>(p.gmask, gb + (int64_t)(row < p.m ? row : 0) * p.gmask_cstride);
            }
#pragma unroll
            for (int i = 0; i < RH; ++i) v[i] = gv[i] > 0.f ? v[i] : v[i] * p.gmask_slope;
          }
          const int64_t yb = (int64_t)b * o0.y_bstride + ncol;
          if (o0.res) {
            const int64_t rb = (int64_t)b * o0.res_bstride + ncol;
            float rv[RH];
#pragma unroll
            for (int i = 0; i < RH; ++i) {
              const int r = r0 + i;
              const int row = rbase + (r & 3) + 8 * (r >> 2);
              rv[i] = ld_io<io_t>(o0.res, rb + (int64_t)(row < p.m ? row : 0) * o0.res_cstride);
            }
#pragma unroll
            for (int i = 0; i < RH; ++i) v[i] = rv[i] + o0.res_scale * v[i];
          }
          if (o0.accumulate) {
            float yo[RH];
#pragma unroll
            for (int i = 0; i < RH; ++i) {
              const int r = r0 + i;
              const int row = rbase + (r & 3) + 8 * (r >> 2);
              yo[i] = ld_io<io_t>(o0.y, yb + (int64_t)(row < p.m ? row : 0) * o0.y_cstride);
            }
#pragma unroll
            for (int i = 0; i < RH; ++i) v[i] = yo[i] + v[i];
          }
          const bool msk = n >= len_b;
#pragma unroll
          for (int i = 0; i < RH; ++i) {
            const int r = r0 + i;
            const int row = rbase + (r & 3) + 8 * (r >> 2);
            float t = v[i];
            if (o0.post_div != 1.0f) t = t / o0.post_div;
            if (msk) t = 0.f;
            if (row < p.m) st_io<io_t>(o0.y, yb + (int64_t)row * o0.y_cstride, t);
          }
          }
        }
      }
    }
  }
}

template <int BM, int BN, int WM_, int WN_, int WT, bool V4, bool IO16, bool GA = false>
int launch_tile_v(const ConvGroup& g, hipStream_t s, const size_t* xrs) {
  constexpr bool BF = WT != VITS_WDT_F32;
  size_t lds = 0;
  int gx = 0, gy = 0;
  for (int i = 0; i < g.n; ++i) {
    const vits_conv1d_desc& d = g.d[i];
    constexpr bool WG = WT == VITS_WDT_F32P || GA;
    constexpr bool SPL = WT == VITS_WDT_F32S || WT == VITS_WDT_F32P;
    const size_t wsz = WG ? 0 : (BF && !SPL) ? (size_t)d.kc * d.k * BM / 2 : (size_t)d.kc * d.k * BM;
    const size_t xsz = (size_t)d.kc * xrs[i];
    if (wsz > (size_t)(SPL ? (BM == 128 && BN == 128 ? VITS_W_TILE_WPS : VITS_W_TILE_SPL)
                           : BF ? VITS_W_TILE_BF : VITS_W_TILE) ||
        xsz > (size_t)XTile<BN, BF, IO16 || WT == VITS_WDT_F32P>::floats)
      return VITS_E_UNSUP;
    if (WT == VITS_WDT_F32P && d.kc != 16 && d.kc != 32) return VITS_E_UNSUP;
    // 32-bit window offsets
    const int64_t maxcol = (int64_t)(d.tin + BN) * d.x_tstride;
    if ((int64_t)d.kc * d.x_cstride + maxcol >= (1LL << 31)) return VITS_E_UNSUP;
    if (V4 && (IO16 || SPL)) {  // T4 staging: kc/4 channel quads x ceil(nb/4)*4 blocks
      constexpr int nu = (XTile<BN, BF, IO16 || WT == VITS_WDT_F32P>::floats / 16 + 48 + 255) / 256;
      if (d.kc % 16 || (size_t)d.kc * ((xrs[i] / 4 + 3) / 4) > (size_t)nu * 256)
        return VITS_E_UNSUP;
    }
    const size_t xslots = BF ? (SPL ? (3 * xrs[i] * (d.kc + 4) + 1) / 2 : (xrs[i] * (d.kc + 4) + 1) / 2) : xsz;
    // + tail pad: the software pipeline reads one k-step past the last chunk
    // (split fp32: one X buffer)
    const size_t wst = WG ? 0 : (SPL && BM == 128 && BN == 128) ? 3 * wsz / 2 : 2 * wsz;  // W stage(s)
    // split fp32 ([W0][W1][X] / [W][X]): a W read-ahead lands in the next W
    // stage or in X; only the B read-ahead of the last plane runs past the
    // end, by < (dil + 2) window rows of kc + 4 bf16 - a tail that keeps the
    // k=7, d=5 64x128 tile at two workgroups per CU
    const size_t tail = SPL ? (size_t)(d.dil + 2) * (d.kc + 4) / 2 + 64
                            : 2 * (size_t)d.k * BM + 2 * xrs[i] + 64;
    // (WG: two X buffers, no W)
    const size_t tail_wg = WG && !SPL ? (size_t)(d.dil + 2) * (d.kc + 4) / 2 + 64 : tail;
    size_t l = sizeof(float) * (wst + ((SPL && !WG) ? 1 : 2) * xslots + tail_wg);
    // UPSAMPLE: the output tile staged after the row constants
    const size_t lup = sizeof(float) * BM + (size_t)BM * (BN + 2) * (IO16 ? 2 : 4) + 64;
    if (d.epi == VITS_EPI_UPSAMPLE && lup > l) l = lup;
    if (l > lds) lds = l;
    const int x = (d.n_out + BN - 1) / BN, y = (d.m + BM - 1) / BM;
    if (x > gx) gx = x;
    if (y > gy) gy = y;
  }
  if (lds > 160 * 1024) return VITS_E_UNSUP;
  dim3 grid(gx, gy, g.n * g.batch);
  dim3 block(256);
  const vits_conv1d_desc& d = g.d[0];
  switch (d.epi) {
    case VITS_EPI_STORE:
      if (d.split < d.m)
        hipLaunchKernelGGL((conv1d_mfma_kernel<BM, BN, WM_, WN_, EPI_STORE2, WT, V4, IO16, GA>), grid, block, lds, s, g);
      else
        hipLaunchKernelGGL((conv1d_mfma_kernel<BM, BN, WM_, WN_, VITS_EPI_STORE, WT, V4, IO16, GA>), grid, block, lds, s, g);
      break;
    case VITS_EPI_GATE:
      hipLaunchKernelGGL((conv1d_mfma_kernel<BM, BN, WM_, WN_, VITS_EPI_GATE, WT, V4, IO16, GA>), grid, block, lds, s, g);
      break;
    case VITS_EPI_UPSAMPLE:
      hipLaunchKernelGGL((conv1d_mfma_kernel<BM, BN, WM_, WN_, VITS_EPI_UPSAMPLE, WT, V4, IO16, GA>), grid, block, lds, s, g);
      break;
    default:
      return VITS_E_UNSUP;
  }
  return vits_launch_status();
}

// 16-byte X staging when every window row is a 16-byte-aligned run of time
// steps (the [B][C][T] activations with T % 4 == 0) and the wider window
// still fits the stage; element-wise staging otherwise.  A group runs one
// staging kind: mixed members are UNSUP (the caller launches them apart).
template <int BM, int BN, int WM_, int WN_, int WT, bool GA = false>
int launch_tile(const ConvGroup& g, hipStream_t s) {
  constexpr bool BF = WT != VITS_WDT_F32;
  size_t xrs4[VITS_CONV_GROUP], xrs1[VITS_CONV_GROUP];
  int nv4 = 0, nio = 0;
  for (int i = 0; i < g.n; ++i) {
    const vits_conv1d_desc& d = g.d[i];
    const int xw = BN + (d.k - 1) * d.dil;
    xrs1[i] = (xw + 3) & ~3;
    const int xsh = (d.pad_left & 3) ? 4 - (d.pad_left & 3) : 0;
    xrs4[i] = 4 * ((xw + xsh + 3) >> 2);
    // 16-byte (fp32) / 8-byte (IO16) blocks of 4 time steps
    const int align = d.io16 ? 7 : 15;
    const bool v4 = d.x_tstride == 1 && (d.x_cstride & 3) == 0 && (d.x_bstride & 3) == 0 &&
                    (d.tin & 3) == 0 && d.pad_left >= 0 &&
                    (reinterpret_cast<uintptr_t>(d.x) & align) == 0 &&
                    (size_t)d.kc * xrs4[i] <=
                        (size_t)((d.io16 || WT == VITS_WDT_F32P) ? XTile<BN, BF, true>::floats
                                                                  : XTile<BN, BF>::floats);
    nv4 += v4;
    nio += d.io16 != 0;
  }
  if (nio != 0 && (nio != g.n || !BF || WT == VITS_WDT_F32S || WT == VITS_WDT_F32P))
    return VITS_E_UNSUP;
  if constexpr (BF && WT != VITS_WDT_F32S && WT != VITS_WDT_F32P) {  // (split: fp32 I/O only)
    if (nio) {
      if (nv4 == g.n) return launch_tile_v<BM, BN, WM_, WN_, WT, true, true, GA>(g, s, xrs4);
      if (nv4 != 0) return VITS_E_UNSUP;
      return launch_tile_v<BM, BN, WM_, WN_, WT, false, true, GA>(g, s, xrs1);
    }
  }
  if (nv4 == g.n) return launch_tile_v<BM, BN, WM_, WN_, WT, true, false, GA>(g, s, xrs4);
  if (nv4 != 0) return VITS_E_UNSUP;
  return launch_tile_v<BM, BN, WM_, WN_, WT, false, false, GA>(g, s, xrs1);
}

template <int WT, bool GA = false>
int conv1d_dispatch(const ConvGroup& g, hipStream_t s) {
  constexpr bool BF = WT != VITS_WDT_F32;
  const vits_conv1d_desc& d = g.d[0];
  long blocks = 0;  // whole launch, for the small-grid fallbacks below
  for (int i = 0; i < g.n; ++i) {
    const vits_conv1d_desc& e = g.d[i];
    if (e.tile != d.tile || e.epi != d.epi || (e.split < e.m) != (d.split < d.m) ||
        e.wdtype != d.wdtype)
      return VITS_E_UNSUP;
    const int bm = d.tile == VITS_TILE_128x128 ? 128 : d.tile == VITS_TILE_32x256 ? 32 : 64;
    const int bn = d.tile == VITS_TILE_64x256 || d.tile == VITS_TILE_32x256 ? 256 : 128;
    blocks += (long)((e.n_out + bn - 1) / bn) * ((e.m + bm - 1) / bm) * g.batch;
  }
  switch (d.tile) {
    case VITS_TILE_128x128: {
      // a 128x128 grid that cannot fill the chip twice over (256 CUs) runs
      // as 64x128 tiles: same packing (its W/X budgets are a subset), twice
      // the workgroups
      if (blocks < 512) return launch_tile<64, 128, 2, 2, WT, GA>(g, s);
      return launch_tile<128, 128, 2, 2, WT, GA>(g, s);
    }
    case VITS_TILE_64x128:
      return launch_tile<64, 128, 2, 2, WT, GA>(g, s);
    case VITS_TILE_64x256: {
      // same fallback for 64x256 grids (the flow / text-side convs at
      // T ~ 500) when the chunk's input window also fits the 128-column tile
      bool fits128 = true;
      for (int i = 0; i < g.n; ++i) {
        const int xw_pad128 = (128 + (g.d[i].k - 1) * g.d[i].dil + 3) & ~3;
        fits128 = fits128 && g.d[i].kc * xw_pad128 <= ((g.d[i].io16 || WT == VITS_WDT_F32P)
                                                          ? XTile<128, BF, true>::floats
                                                          : XTile<128, BF>::floats);
      }
      if (blocks < 512 && fits128) return launch_tile<64, 128, 2, 2, WT, GA>(g, s);
      if constexpr (WT == VITS_WDT_F32S || WT == VITS_WDT_F32P) {
        // split fp32: 2x2 waves (32x128 per wave) - each A-fragment split
        // feeds four B fragments instead of two (k=11 convs +1..3 %)
        return launch_tile<64, 256, 2, 2, WT, GA>(g, s);
      }
      return launch_tile<64, 256, 1, 4, WT, GA>(g, s);
    }
    case VITS_TILE_32x256:
      return launch_tile<32, 256, 1, 4, WT, GA>(g, s);
    default:
      return VITS_E_UNSUP;
  }
}

}  // namespace vits_conv

// per-type entry points (defined in conv1d_{f32,bf16,f16}.hip)
int vits_conv1d_dispatch_f32(const vits_conv::ConvGroup& g, hipStream_t s);
int vits_conv1d_dispatch_bf16(const vits_conv::ConvGroup& g, hipStream_t s);
int vits_conv1d_dispatch_f16(const vits_conv::ConvGroup& g, hipStream_t s);
int vits_conv1d_dispatch_f32s(const vits_conv::ConvGroup& g, hipStream_t s);
int vits_conv1d_dispatch_f32p(const vits_conv::ConvGroup& g, hipStream_t s);
int vits_conv1d_dispatch_bf16g(const vits_conv::ConvGroup& g, hipStream_t s);
int vits_conv1d_dispatch_f16g(const vits_conv::ConvGroup& g, hipStream_t s);
