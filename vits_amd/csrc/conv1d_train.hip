// conv1d_train.hip — the backward side of the MFMA conv for the training
// step (train_stft.py:162-236 through SynthesizerTrn.forward and the MWSD
// discriminator): every stride-1 Conv1d of WN / ResBlock2 / couplings /
// posterior encoder / Generator / WaveDiscriminator runs its forward, input
// gradient and weight gradient on 16-bit MFMA with fp32 accumulation (the
// reference runs these convs under fp16 autocast, train_stft.py:165,216).
//
//  * vits_conv1d_pack16: the layer's fp32 weight [Cout][Cin][k] (weight-norm
//    / spectral-norm already applied by the caller) -> the 16-bit image the
//    forward kernel streams ([cin_pad/16][k][2][m_pad][8], conv1d_impl.h),
//    either as is (forward) or transposed and tap-flipped (input gradient:
//    dX = conv(dY, W'[ci][co][k-1-j], pad' = (k-1)*dil - pad), which the
//    forward kernel then runs unchanged).
//  * vits_conv1d_wgrad: dW[co][ci][j] = sum_{b,t} dY[b][co][t] * X~[b][ci][t - pad + j*dil]
//    (X~ = leaky-relu prologue of X when the forward fused one) and
//    dbias[co] = sum_{b,t} dY[b][co][t].  GEMM rows = co, columns = ci (one
//    accumulator set per tap), reduction over (b, t).
//
// wgrad structure: workgroup = 4 waves = 64 co x 64 ci x all k taps; each
// wave owns a 32 co x 32 ci block of every tap (k accumulators).  Per chunk
// of KT = 64 time steps the workgroup stages
//    dY[64 co][64 t]              f16, row-major (t contiguous)  -> A operand
//    X~[64 + (k-1)*dil t][64 ci]  f16, time-major (ci contiguous) -> B operand
// into LDS (double-buffered, next chunk's global loads in flight under the
// current chunk's MFMAs).  The A fragment (8 consecutive t of one co row) is
// one ds_read_b128; the B fragment of tap j (8 consecutive t of one ci,
// starting at any row t + j*dil) is two ds_read_b64_tr_b16 transposed
// reads, so every tap reuses the one staged window at an arbitrary row
// offset — no im2col, no per-tap copies.  The reduction over (b, t) is
// split across workgroups (>= 16 chunks each, so the fp32 atomics that
// combine them stay far below the chip's atomic byte rate); partial tiles
// are added with global_atomic_add_f32 into a [k][Cout][Cin] accumulator
// (two 128-byte row segments per wave instruction).
#include <type_traits>

#include "common.h"

namespace {

typedef short s16x4 __attribute__((__vector_size__(4 * sizeof(short))));
typedef __attribute__((address_space(3))) s16x4* lds_s16x4_ptr;
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int WG_M = 64;               // co rows per workgroup
constexpr int WG_N = 64;               // ci columns per workgroup
constexpr int KT = 64;                 // time steps per chunk
constexpr int DY_LD = KT + 8;          // halves per staged dY row (144 B)
constexpr int X_LD = WG_N + 4;         // halves per staged X row (136 B, 8-B aligned)
constexpr int MAX_WR = 128;            // staged window rows: KT + (k-1)*dil <= MAX_WR
constexpr int DY_HALVES = WG_M * DY_LD;
constexpr int X_HALVES = MAX_WR * X_LD;
constexpr int STAGE_HALVES = DY_HALVES + X_HALVES;

template <int WT>
struct Op16 {
  typedef _Float16 T;
  typedef f16x8 V8;
};
template <>
struct Op16<VITS_WDT_BF16> {
  typedef __bf16 T;
  typedef bf16x8 V8;
};

template <int WT>
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  typedef typename Op16<WT>::T T;
  T ha = (T)a, hb = (T)b;
  uint16_t ua, ub;
  __builtin_memcpy(&ua, &ha, 2);
  __builtin_memcpy(&ub, &hb, 2);
  return (uint32_t)ua | ((uint32_t)ub << 16);
}

// PARTIAL: each (b, t)-split workgroup stores its partial tile with plain
// stores into ws[split][k][cout][cin] (+ bias partials ws_b[split][cout]);
// wgrad_reduce_kernel then sums the splits.  Otherwise fp32 atomics into
// p.dw_t / p.dbias.
// VEC: 16-byte staging loads (the [B][C][T] tensors with 16-byte aligned
// rows and tin % 4 == 0): dY as 4 consecutive steps of one row, X as 4
// consecutive steps of a channel pair from a 4-aligned window start (sh
// rows of shift, read back with the same shift) - a quarter of the load
// instructions of the element-wise map.
// IO16 (with VEC): dY and X are tensors of the 16-bit operand type (the
// fp16 activations of the autocast training step); the 8-byte blocks stay
// raw in registers until they are written to LDS.
template <int NK, int WT, bool PARTIAL, bool VEC, bool IO16 = false>
__global__ __launch_bounds__(256, NK <= 5 ? 2 : 1) void wgrad_kernel(const vits_conv1d_wgrad_desc p,
                                                                     int tchunks, int total_chunks,
                                                                     int chunks_per_wg,
                                                                     float* __restrict__ ws,
                                                                     float* __restrict__ ws_b) {
  typedef typename Op16<WT>::V8 V8;
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int l32 = lane & 31;
  const int lhi = lane >> 5;
  const int wm = (wid >> 1) * 32;  // wave's co offset in the tile
  const int wn = (wid & 1) * 32;   // wave's ci offset in the tile
  const int m0 = blockIdx.z * WG_M;
  const int c0 = blockIdx.y * WG_N;
  const int ch_begin = blockIdx.x * chunks_per_wg;
  const int ch_end = min(total_chunks, ch_begin + chunks_per_wg);
  const int dil = p.dil;
  const int wr = KT + (NK - 1) * dil;  // staged window rows
  const float slope = p.in_slope;
  const bool act_in = slope != 1.0f;
  const bool do_bias = p.dbias != nullptr && blockIdx.y == 0;

  f32x16 acc[NK];
#pragma unroll
  for (int j = 0; j < NK; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
  float bsum[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) bsum[q] = 0.f;

  // ---- staging maps (fixed per thread) ------------------------------------
  // dY: pair e = tid + 256 q -> row (e >> 5), columns 2 (e & 31) + {0, 1}
  const int dy_row0 = tid >> 5;   // + 8 q
  const int dy_col = 2 * (tid & 31);
  // X: wave w stages channel pairs (2 (w + 4 i), +1), i < 8, window rows
  // lane + 64 h, h < 2: every global load instruction reads 64 consecutive
  // time steps of one channel row (256 B).
  float dyv[16];
  float xv[32];
  typedef float f32x4v __attribute__((ext_vector_type(4)));
  // VEC window: rows from the 4-aligned start t0 - pad_left - sh
  const int sh = VEC ? ((p.pad_left & 3) ? 4 - (p.pad_left & 3) : 0) : 0;

  // x addressing: channel v -> row base, window column t -> offset in the row
  auto vbase = [&](int v) -> int64_t { return (int64_t)v * p.x_cstride; };
  auto xcol = [&](int t) -> int { return t; };

  typedef typename Op16<WT>::T T16;
  typedef T16 t16x4 __attribute__((ext_vector_type(4)));
  t16x4 dyr[IO16 ? 4 : 1], xr[IO16 ? 8 : 1];  // raw IO16 blocks
  auto gload_io16 = [&](int chunk) {
    const int b = chunk / tchunks;
    const int t0 = (chunk - b * tchunks) * KT;
    const T16* dyb = reinterpret_cast<const T16*>(p.dy) + (int64_t)b * p.dy_bstride;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int u = tid + 256 * q;
      const int co = m0 + (u >> 4);
      const int t = t0 + 4 * (u & 15);
      const T16* src = dyb + (int64_t)co * p.dy_cstride + t;
      t16x4 v = {};
      if (co < p.cout) {
        if (t + 3 < p.n_out) {
          v = *reinterpret_cast<const t16x4*>(src);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = t + e < p.n_out ? src[e] : (T16)0.f;
        }
      }
      dyr[q] = v;
    }
    const T16* xb = reinterpret_cast<const T16*>(p.x) + (int64_t)b * p.x_bstride;
    const int ts = t0 - p.pad_left - sh;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int u = tid + 256 * q;
      const int ci = c0 + 2 * (u >> 5);
      const int r4 = 4 * (u & 31);
      const int t = ts + r4;
      const bool tok = r4 < wr + sh && t >= 0 && t < p.tin;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        t16x4 v = {};
        if (tok && ci + e < p.cin)
          v = *reinterpret_cast<const t16x4*>(xb + vbase(ci + e) + xcol(t));
        xr[2 * q + e] = v;
      }
    }
  };
  auto unpack_io16 = [&]() {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int e = 0; e < 4; ++e) dyv[4 * q + e] = (float)dyr[q][e];
#pragma unroll
      for (int e = 0; e < 2; ++e)
#pragma unroll
        for (int i = 0; i < 4; ++i) xv[8 * q + 4 * e + i] = (float)xr[2 * q + e][i];
    }
  };

  auto gload_vec = [&](int chunk) {
    if constexpr (IO16) {
      gload_io16(chunk);
      return;
    }
    const int b = chunk / tchunks;
    const int t0 = (chunk - b * tchunks) * KT;
    const float* dyb = p.dy + (int64_t)b * p.dy_bstride;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int u = tid + 256 * q;
      const int co = m0 + (u >> 4);
      const int t = t0 + 4 * (u & 15);
      const float* src = dyb + (int64_t)co * p.dy_cstride + t;
      f32x4v v = {0.f, 0.f, 0.f, 0.f};
      if (co < p.cout) {
        if (t + 3 < p.n_out) {
          v = *reinterpret_cast<const f32x4v*>(src);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = t + e < p.n_out ? src[e] : 0.f;
        }
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) dyv[4 * q + e] = v[e];
    }
    const float* xb = p.x + (int64_t)b * p.x_bstride;
    const int ts = t0 - p.pad_left - sh;  // multiple of 4
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int u = tid + 256 * q;
      const int ci = c0 + 2 * (u >> 5);
      const int r4 = 4 * (u & 31);
      const int t = ts + r4;
      const bool tok = r4 < wr + sh && t >= 0 && t < p.tin;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        f32x4v v = {0.f, 0.f, 0.f, 0.f};
        if (tok && ci + e < p.cin)
          v = *reinterpret_cast<const f32x4v*>(xb + vbase(ci + e) + xcol(t));
#pragma unroll
        for (int i = 0; i < 4; ++i) xv[8 * q + 4 * e + i] = v[i];
      }
    }
  };
  auto lstore_vec = [&](uint16_t* st) {
    if constexpr (IO16) {
      // raw 16-bit blocks: dY as one 8-byte store per unit, X channel pairs
      // interleaved bitwise when no prologue runs - the same bits as the
      // float round trip below (exact for 16-bit values) in a quarter of the
      // VALU work (the kernel is VALU-issue-bound)
      typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int u = tid + 256 * q;
        if (do_bias)
          bsum[q] += ((float)dyr[q][0] + (float)dyr[q][1]) + ((float)dyr[q][2] + (float)dyr[q][3]);
        *reinterpret_cast<t16x4*>(st + (u >> 4) * DY_LD + 4 * (u & 15)) = dyr[q];
      }
      uint32_t* xl = reinterpret_cast<uint32_t*>(st + DY_HALVES);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int u = tid + 256 * q;
        const int cl = 2 * (u >> 5);
        const int r4 = 4 * (u & 31);
        if (r4 < wr + sh) {
          if (!act_in) {
            const u16x4 a = __builtin_bit_cast(u16x4, xr[2 * q]);
            const u16x4 b = __builtin_bit_cast(u16x4, xr[2 * q + 1]);
#pragma unroll
            for (int i = 0; i < 4; ++i)
              xl[((r4 + i) * X_LD + cl) >> 1] = (uint32_t)a[i] | ((uint32_t)b[i] << 16);
          } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              float v0 = (float)xr[2 * q][i], v1 = (float)xr[2 * q + 1][i];
              v0 = v0 < 0.f ? v0 * slope : v0;
              v1 = v1 < 0.f ? v1 * slope : v1;
              xl[((r4 + i) * X_LD + cl) >> 1] = pack2<WT>(v0, v1);
            }
          }
        }
      }
      return;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int u = tid + 256 * q;
      const float a0 = dyv[4 * q], a1 = dyv[4 * q + 1], a2 = dyv[4 * q + 2], a3 = dyv[4 * q + 3];
      if (do_bias) bsum[q] += (a0 + a1) + (a2 + a3);
      uint32_t* d = reinterpret_cast<uint32_t*>(st + (u >> 4) * DY_LD + 4 * (u & 15));
      d[0] = pack2<WT>(a0, a1);
      d[1] = pack2<WT>(a2, a3);
    }
    uint32_t* xl = reinterpret_cast<uint32_t*>(st + DY_HALVES);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int u = tid + 256 * q;
      const int cl = 2 * (u >> 5);
      const int r4 = 4 * (u & 31);
      if (r4 < wr + sh) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float v0 = xv[8 * q + i], v1 = xv[8 * q + 4 + i];
          if (act_in) {
            v0 = v0 < 0.f ? v0 * slope : v0;
            v1 = v1 < 0.f ? v1 * slope : v1;
          }
          xl[((r4 + i) * X_LD + cl) >> 1] = pack2<WT>(v0, v1);
        }
      }
    }
  };

  // element-wise map; with IO16 the 16-bit values stay raw in registers
  // (dyh / xh) until lstore converts them
  typedef typename std::conditional<IO16, T16, float>::type el_t;
  el_t dyh[16], xh[32];
  auto gload = [&](int chunk) {
    const int b = chunk / tchunks;
    const int t0 = (chunk - b * tchunks) * KT;
    const el_t* dyb = reinterpret_cast<const el_t*>(p.dy) + (int64_t)b * p.dy_bstride;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int co = m0 + dy_row0 + 8 * q;
      const int t = t0 + dy_col;
      const el_t* src = dyb + (int64_t)co * p.dy_cstride + t;
      const bool rok = co < p.cout;
      dyh[2 * q] = (rok && t < p.n_out) ? src[0] : (el_t)0.f;
      dyh[2 * q + 1] = (rok && t + 1 < p.n_out) ? src[1] : (el_t)0.f;
    }
    const el_t* xb = reinterpret_cast<const el_t*>(p.x) + (int64_t)b * p.x_bstride;
    const int ts = t0 - p.pad_left;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int ci = c0 + 2 * (wid + 4 * i);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int r = lane + 64 * h;
        const int t = ts + r;
        const bool tok = r < wr && t >= 0 && t < p.tin;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const bool ok = tok && ci + e < p.cin;
          xh[(i * 2 + h) * 2 + e] = ok ? xb[vbase(ci + e) + xcol(t)] : (el_t)0.f;
        }
      }
    }
  };
  auto lstore = [&](uint16_t* st) {
#pragma unroll
    for (int i = 0; i < 16; ++i) dyv[i] = (float)dyh[i];
#pragma unroll
    for (int i = 0; i < 32; ++i) xv[i] = (float)xh[i];
    uint32_t* dyl = reinterpret_cast<uint32_t*>(st);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float a = dyv[2 * q], bv = dyv[2 * q + 1];
      if (do_bias) bsum[q] += a + bv;
      dyl[((dy_row0 + 8 * q) * DY_LD + dy_col) >> 1] = pack2<WT>(a, bv);
    }
    uint32_t* xl = reinterpret_cast<uint32_t*>(st + DY_HALVES);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int cl = 2 * (wid + 4 * i);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int r = lane + 64 * h;
        float v0 = xv[(i * 2 + h) * 2], v1 = xv[(i * 2 + h) * 2 + 1];
        if (act_in) {
          v0 = v0 < 0.f ? v0 * slope : v0;
          v1 = v1 < 0.f ? v1 * slope : v1;
        }
        if (h == 0 || r < wr) xl[(r * X_LD + cl) >> 1] = pack2<WT>(v0, v1);
      }
    }
  };

  // ---- fragment addressing --------------------------------------------------
  // A (dY rows): lane -> co row wm + l32, t = 16 s + 8 lhi .. + 7
  // B (tap j): 16-lane group g = lane >> 4 reads ci columns wn + 16 (g & 1) + 4 pp
  //   (pp = lane & 3) of rows 16 s + 8 (g >> 1) + qq (+4) + j dil (qq = (lane >> 2) & 3)
  const int g = lane >> 4;
  const int qq = (lane >> 2) & 3;
  const int pp = lane & 3;
  const int a_off = (wm + l32) * DY_LD + 8 * lhi;
  const int b_off = DY_HALVES + (8 * (g >> 1) + qq + sh) * X_LD + wn + 16 * (g & 1) + 4 * pp;

  if (ch_begin < ch_end) {
    if constexpr (VEC) {
      gload_vec(ch_begin);
      lstore_vec(lds);
    } else {
      gload(ch_begin);
      lstore(lds);
    }
  }
  __syncthreads();
  for (int ch = ch_begin; ch < ch_end; ++ch) {
    const int it = ch - ch_begin;
    uint16_t* cur = lds + (it & 1) * STAGE_HALVES;
    uint16_t* nxt = lds + ((it + 1) & 1) * STAGE_HALVES;
    const bool more = ch + 1 < ch_end;
    if (more) {
      if constexpr (VEC)
        gload_vec(ch + 1);
      else
        gload(ch + 1);
    }
#pragma unroll
    for (int s = 0; s < KT / 16; ++s) {
      const V8 a = *reinterpret_cast<const V8*>(cur + a_off + 16 * s);
#pragma unroll
      for (int j = 0; j < NK; ++j) {
        const uint16_t* bp = cur + b_off + (16 * s + j * dil) * X_LD;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_ptr)(bp));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_ptr)(bp + 4 * X_LD));
        const s16x4 both[2] = {lo, hi};
        V8 bb;
        __builtin_memcpy(&bb, both, 16);
        if constexpr (WT == VITS_WDT_F16)
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, bb, acc[j], 0, 0, 0);
        else
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bb, acc[j], 0, 0, 0);
      }
    }
    if (more) {
      if constexpr (VEC)
        lstore_vec(nxt);
      else
        lstore(nxt);
    }
    __syncthreads();
  }

  // ---- epilogue: dw_t[j][co][ci] (atomics) or the split's partial tile ------
  const int ci = c0 + wn + l32;
  float* dst = PARTIAL ? ws + (int64_t)blockIdx.x * NK * p.cout * p.cin : p.dw_t;
#pragma unroll
  for (int j = 0; j < NK; ++j) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = m0 + wm + 8 * (r >> 2) + 4 * lhi + (r & 3);
      if (co < p.cout && ci < p.cin) {
        float* a = dst + ((int64_t)j * p.cout + co) * p.cin + ci;
        if constexpr (PARTIAL)
          *a = acc[j][r];
        else
          unsafeAtomicAdd(a, acc[j][r]);
      }
    }
  }
  if (do_bias && VEC) {
    // VEC map: row (tid >> 4) + 16 q is shared by 16 consecutive lanes
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float v = bsum[q];
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 16);
      const int co = m0 + (tid >> 4) + 16 * q;
      if ((tid & 15) == 0 && co < p.cout) {
        if constexpr (PARTIAL)
          ws_b[(int64_t)blockIdx.x * p.cout + co] = v;
        else
          unsafeAtomicAdd(p.dbias + co, v);
      }
    }
  } else if (do_bias) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      float v = bsum[q];
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 32);
      const int co = m0 + dy_row0 + 8 * q;
      if ((tid & 31) == 0 && co < p.cout) {
        if constexpr (PARTIAL)
          ws_b[(int64_t)blockIdx.x * p.cout + co] = v;
        else
          unsafeAtomicAdd(p.dbias + co, v);
      }
    }
  }
}

// ---- fp32 weight gradient (the fp32 training step, autocast off) ---------------
// Same GEMM as wgrad_kernel (rows co, columns ci, one accumulator set per
// tap, reduction over (b, t) split across workgroups into partial tiles) on
// the exact-fp32 MFMA v_mfma_f32_32x32x2_f32: every product is an fp32
// product, accumulated in fp32 (an fmaf chain per k-step pair), so the
// result carries the reference's fp32 conv-backward precision.  Per chunk of
// KT32 = 32 time steps the workgroup stages fp32
//    dY[64 co][32 t]                 row-major, odd row stride (33)
//    X~[32 + (k-1)*dil t][64 ci]     time-major, odd row stride (65)
// both conflict-free for the staging stores (consecutive lanes: consecutive
// t) and for the fragment reads (A: 32 rows of one column, B: 32 consecutive
// ci of one row).  A k-step covers 2 time steps: A = dY[co][2s + lhi], B_j =
// X~[2s + lhi + j*dil][ci].  Double-buffered (next chunk's loads in flight
// under the current chunk's MFMAs), 67 KB of LDS: two workgroups per CU.
constexpr int KT32 = 32;
constexpr int MAX_WR32 = 96;                 // KT32 + (k-1)*dil <= 96
constexpr int DY32_LD = KT32 + 1;
constexpr int X32_LD = WG_N + 1;
constexpr int DY32_FLOATS = WG_M * DY32_LD;
constexpr int STAGE32 = DY32_FLOATS + MAX_WR32 * X32_LD;
constexpr int NXQ32 = WG_N * MAX_WR32 / 256;  // staged X elements per thread (24)

template <int NK>
__global__ __launch_bounds__(256, 2) void wgrad_f32_kernel(const vits_conv1d_wgrad_desc p,
                                                           int tchunks, int total_chunks,
                                                           int chunks_per_wg,
                                                           float* __restrict__ ws,
                                                           float* __restrict__ ws_b) {
  extern __shared__ __attribute__((aligned(16))) float lds32[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int l32 = lane & 31;
  const int lhi = lane >> 5;
  const int wm = (wid >> 1) * 32;
  const int wn = (wid & 1) * 32;
  const int m0 = blockIdx.z * WG_M;
  const int c0 = blockIdx.y * WG_N;
  const int ch_begin = blockIdx.x * chunks_per_wg;
  const int ch_end = min(total_chunks, ch_begin + chunks_per_wg);
  const int dil = p.dil;
  const int wr = KT32 + (NK - 1) * dil;
  const float slope = p.in_slope;
  const bool act_in = slope != 1.0f;
  const bool do_bias = p.dbias != nullptr && blockIdx.y == 0;

  f32x16 acc[NK];
#pragma unroll
  for (int j = 0; j < NK; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
  float bsum[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) bsum[q] = 0.f;

  // dY element (row (tid >> 5) + 8 q, column tid & 31); X element e = tid +
  // 256 q -> (channel e / 96, window row e % 96)
  const int dy_row0 = tid >> 5;
  const int dy_col = tid & 31;
  float dyv[8], xv[NXQ32];
  auto gload = [&](int chunk) {
    const int b = chunk / tchunks;
    const int t0 = (chunk - b * tchunks) * KT32;
    const float* dyb = p.dy + (int64_t)b * p.dy_bstride;
    const int t = t0 + dy_col;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int co = m0 + dy_row0 + 8 * q;
      dyv[q] = (co < p.cout && t < p.n_out) ? dyb[(int64_t)co * p.dy_cstride + t] : 0.f;
    }
    const float* xb = p.x + (int64_t)b * p.x_bstride;
    const int ts = t0 - p.pad_left;
#pragma unroll
    for (int q = 0; q < NXQ32; ++q) {
      const int e = tid + 256 * q;
      const int cl = e / MAX_WR32;
      const int r = e - cl * MAX_WR32;
      const int tt = ts + r;
      const bool ok = r < wr && tt >= 0 && tt < p.tin && c0 + cl < p.cin;
      xv[q] = ok ? xb[(int64_t)(c0 + cl) * p.x_cstride + tt] : 0.f;
    }
  };
  auto lstore = [&](float* st) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      if (do_bias) bsum[q] += dyv[q];
      st[(dy_row0 + 8 * q) * DY32_LD + dy_col] = dyv[q];
    }
    float* xl = st + DY32_FLOATS;
#pragma unroll
    for (int q = 0; q < NXQ32; ++q) {
      const int e = tid + 256 * q;
      const int cl = e / MAX_WR32;
      const int r = e - cl * MAX_WR32;
      float v = xv[q];
      if (act_in) v = v < 0.f ? v * slope : v;
      if (r < wr) xl[r * X32_LD + cl] = v;
    }
  };

  const int a_off = (wm + l32) * DY32_LD + lhi;
  const int b_off = DY32_FLOATS + lhi * X32_LD + wn + l32;
  if (ch_begin < ch_end) {
    gload(ch_begin);
    lstore(lds32);
  }
  __syncthreads();
  for (int ch = ch_begin; ch < ch_end; ++ch) {
    const int it = ch - ch_begin;
    float* cur = lds32 + (it & 1) * STAGE32;
    float* nxt = lds32 + ((it + 1) & 1) * STAGE32;
    const bool more = ch + 1 < ch_end;
    if (more) gload(ch + 1);
#pragma unroll
    for (int s = 0; s < KT32 / 2; ++s) {
      const float a = cur[a_off + 2 * s];
#pragma unroll
      for (int j = 0; j < NK; ++j) {
        const float bv = cur[b_off + (2 * s + j * dil) * X32_LD];
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bv, acc[j], 0, 0, 0);
      }
    }
    if (more) lstore(nxt);
    __syncthreads();
  }

  const int ci = c0 + wn + l32;
  float* dst = ws + (int64_t)blockIdx.x * NK * p.cout * p.cin;
#pragma unroll
  for (int j = 0; j < NK; ++j) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = m0 + wm + 8 * (r >> 2) + 4 * lhi + (r & 3);
      if (co < p.cout && ci < p.cin) dst[((int64_t)j * p.cout + co) * p.cin + ci] = acc[j][r];
    }
  }
  if (do_bias) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      float v = bsum[q];
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 32);
      const int co = m0 + dy_row0 + 8 * q;
      if ((tid & 31) == 0 && co < p.cout) ws_b[(int64_t)blockIdx.x * p.cout + co] = v;
    }
  }
}

// dw[co][ci][j] = sum_s ws[s][j][co][ci] (the parameter layout, written, not
// accumulated: no zeroing), dbias[co] = sum_s ws_b[s][co].  A workgroup
// reduces E = 256 / P consecutive slab elements with P lanes each over the
// splits (coalesced reads along the slab, <= ~16 loads per thread), then
// combines the P partial sums in LDS.  Blocks past the slab's do the bias.
template <int P>
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ ws,
                                                           const float* __restrict__ ws_b,
                                                           int splits, int k, int cout, int cin,
                                                           int slab_blocks, float* __restrict__ dw,
                                                           float* __restrict__ dbias) {
  constexpr int E = 256 / P;
  __shared__ float red[256];
  const int tid = threadIdx.x;
  const int el = tid % E;
  const int q = tid / E;
  const int64_t n = (int64_t)cout * cin;
  const bool bias_blk = (int)blockIdx.x >= slab_blocks;
  const int64_t total = bias_blk ? cout : n * k;
  const float* src = bias_blk ? ws_b : ws;
  const int64_t e = (int64_t)(bias_blk ? blockIdx.x - slab_blocks : blockIdx.x) * E + el;
  float a0 = 0.f, a1 = 0.f;
  if (e < total) {
    int s = q;
    for (; s + P < splits; s += 2 * P) {
      a0 += src[(int64_t)s * total + e];
      a1 += src[(int64_t)(s + P) * total + e];
    }
    if (s < splits) a0 += src[(int64_t)s * total + e];
  }
  red[tid] = a0 + a1;
  __syncthreads();
#pragma unroll
  for (int off = P / 2; off > 0; off >>= 1) {
    if (q < off) red[tid] += red[tid + off * E];
    __syncthreads();
  }
  if (q == 0 && e < total) {
    if (bias_blk) {
      dbias[e] = red[tid];
    } else {
      const int64_t j = e / n;
      const int64_t i = e - j * n;
      dw[i * k + j] = red[tid];
    }
  }
}

// (b, t)-chunks per workgroup.  Atomic mode: >= 16 chunks (1024 time steps)
// per workgroup (512 FLOP per atomic byte), beyond that about 1024
// workgroups.  Split mode: about 2048 workgroups, >= 4 chunks each, and the
// partial tiles (splits x k x cout x cin floats) capped near 2x the work's
// own input bytes so the workspace pass stays small next to the MFMA work.
struct WgradSplit {
  int tchunks, total, cpw, splits;
};
WgradSplit wgrad_split(const vits_conv1d_wgrad_desc& d, int batch, bool partial) {
  WgradSplit w;
  const int kt = d.wdtype == VITS_WDT_F32 ? KT32 : KT;
  w.tchunks = (d.n_out + kt - 1) / kt;
  w.total = batch * w.tchunks;
  const int tiles = ((d.cout + WG_M - 1) / WG_M) * ((d.cin + WG_N - 1) / WG_N);
  if (!partial) {
    w.cpw = (int)(((int64_t)w.total * tiles + 1023) / 1024);
    const int min_cpw = w.total < 16 ? w.total : 16;
    if (w.cpw < min_cpw) w.cpw = min_cpw;
  } else {
    // 16 chunks per workgroup (measured best on the training shapes,
    // tools/wgrad_split_bench.py: faster than the atomic mode on every one,
    // 92.8 -> 76 us enc_q WN, 127.6 -> 81.5 us MWD scale 0), then at most
    // ~2048 workgroups
    w.cpw = (int)(((int64_t)w.total * tiles + 2047) / 2048);
    const int min_cpw = w.total < 16 ? w.total : 16;
    if (w.cpw < min_cpw) w.cpw = min_cpw;
    // fewer than one workgroup per CU: halve the chunks per workgroup
    // (the MWD scale-4 shape: 60 -> 43 us)
    if (w.cpw == 16 && (int64_t)((w.total + 15) / 16) * tiles < 256) w.cpw = 8;
  }
  if (d.reserved > 0) w.cpw = d.reserved < w.total ? d.reserved : w.total;  // explicit override
  w.splits = (w.total + w.cpw - 1) / w.cpw;
  return w;
}

int wgrad_f32_dispatch(const vits_conv1d_wgrad_desc& d, int batch, hipStream_t s, float* ws,
                       float* ws_b) {
  const WgradSplit w = wgrad_split(d, batch, true);
  dim3 grid(w.splits, (d.cin + WG_N - 1) / WG_N, (d.cout + WG_M - 1) / WG_M);
  const size_t lds = 2 * STAGE32 * sizeof(float);
  switch (d.k) {
#define VITS_WG32_CASE(NK)                                                                         \
  case NK:                                                                                         \
    hipLaunchKernelGGL((wgrad_f32_kernel<NK>), grid, dim3(256), lds, s, d, w.tchunks, w.total,    \
                       w.cpw, ws, ws_b);                                                           \
    break;
    VITS_WG32_CASE(1)
    VITS_WG32_CASE(2)
    VITS_WG32_CASE(3)
    VITS_WG32_CASE(4)
    VITS_WG32_CASE(5)
    VITS_WG32_CASE(7)
    VITS_WG32_CASE(9)
    VITS_WG32_CASE(11)
#undef VITS_WG32_CASE
    default:
      return VITS_E_UNSUP;
  }
  return vits_launch_status();
}

template <int WT, bool PARTIAL>
int wgrad_dispatch(const vits_conv1d_wgrad_desc& d, int batch, hipStream_t s, float* ws,
                   float* ws_b) {
  const WgradSplit w = wgrad_split(d, batch, PARTIAL);
  const int tchunks = w.tchunks, total = w.total, cpw = w.cpw;
  dim3 grid(w.splits, (d.cin + WG_N - 1) / WG_N, (d.cout + WG_M - 1) / WG_M);
  const size_t lds = 2 * STAGE_HALVES * sizeof(uint16_t);
  const int sh = (d.pad_left & 3) ? 4 - (d.pad_left & 3) : 0;
  const uintptr_t al = d.io16 ? 7 : 15;
  const bool vec = (d.dy_cstride & 3) == 0 && (d.dy_bstride & 3) == 0 &&
                   (reinterpret_cast<uintptr_t>(d.dy) & al) == 0 && (d.x_cstride & 3) == 0 &&
                   (d.x_bstride & 3) == 0 && (reinterpret_cast<uintptr_t>(d.x) & al) == 0 &&
                   (d.tin & 3) == 0 && KT + (d.k - 1) * d.dil + sh <= MAX_WR &&
                   (d.k > 1 || d.io16);  // k = 1 (tools/wgrad_split_bench.py: 40 -> 53 us)
                                         // keeps the element-wise map for fp32 inputs
  switch (d.k) {
#define VITS_WG_CASE(NK)                                                                           \
  case NK:                                                                                         \
    if (d.io16 && vec)                                                                             \
      hipLaunchKernelGGL((wgrad_kernel<NK, WT, PARTIAL, true, true>), grid, dim3(256), lds, s, d,  \
                         tchunks, total, cpw, ws, ws_b);                                           \
    else if (d.io16)                                                                               \
      hipLaunchKernelGGL((wgrad_kernel<NK, WT, PARTIAL, false, true>), grid, dim3(256), lds, s, d, \
                         tchunks, total, cpw, ws, ws_b);                                           \
    else if (vec)                                                                                  \
      hipLaunchKernelGGL((wgrad_kernel<NK, WT, PARTIAL, true>), grid, dim3(256), lds, s, d,        \
                         tchunks, total, cpw, ws, ws_b);                                           \
    else                                                                                           \
      hipLaunchKernelGGL((wgrad_kernel<NK, WT, PARTIAL, false>), grid, dim3(256), lds, s, d,       \
                         tchunks, total, cpw, ws, ws_b);                                           \
    break;
    VITS_WG_CASE(1)
    VITS_WG_CASE(2)
    VITS_WG_CASE(3)
    VITS_WG_CASE(4)
    VITS_WG_CASE(5)
    VITS_WG_CASE(7)
    VITS_WG_CASE(9)
    VITS_WG_CASE(11)
#undef VITS_WG_CASE
    default:
      return VITS_E_UNSUP;
  }
  return vits_launch_status();
}

// ---- weight image for the 16-bit forward kernel ------------------------------
// element i of the image out[c/16][j][(c%16)/8][m][c%8] (rows m / channels c
// are (co, ci) or, transposed, (ci, co) with the tap order reversed)
// element i of the image out[c/16][j][(c%16)/8][m][c%8] (rows m / channels c
// are (co, ci) or, transposed, (ci, co) with the tap order reversed; gate:
// gate-interleaved rows, row 2q = output q, 2q+1 = cout/2 + q, VITS_EPI_GATE)
template <typename T>
__device__ __forceinline__ void pack16_elem32(const float* __restrict__ w, int cout, int cin,
                                              int k, int transpose, T* __restrict__ out,
                                              int m_pad, int i, int gate) {
  const int c8 = i & 7;
  int r = i >> 3;
  const int rq = r / m_pad;
  const int m = r - rq * m_pad;
  const int half = rq & 1;
  const int jq = rq >> 1;
  const int cg = jq / k;
  const int j = jq - cg * k;
  const int c = cg * 16 + half * 8 + c8;
  float v = 0.f;
  if (!transpose) {
    const int src = gate ? ((m & 1) ? (cout >> 1) + (m >> 1) : (m >> 1)) : m;
    if (m < cout && c < cin) v = w[(src * cin + c) * k + j];
  } else {
    if (m < cin && c < cout) v = w[(c * cin + m) * k + (k - 1 - j)];
  }
  out[i] = (T)v;
}

// both images (forward and transposed / tap-reversed for the input
// gradient) in ONE launch: the training forward packs the backward's image
// too, one graph node instead of two per conv
template <typename T>
__global__ void pack16_pair_kernel(const float* __restrict__ w, int cout, int cin, int k,
                                   T* __restrict__ out, int m_pad, int total,
                                   T* __restrict__ out_t, int m_pad_t, int total_t) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total + total_t;
       i += gridDim.x * blockDim.x) {
    if (i < total)
      pack16_elem32<T>(w, cout, cin, k, 0, out, m_pad, i, 0);
    else
      pack16_elem32<T>(w, cout, cin, k, 1, out_t, m_pad_t, i - total, 0);
  }
}

// both images of up to PACK_LIST layers per launch (vits_conv1d_pack16_pairs):
// blockIdx.y = layer, blockIdx.x strides over that layer's two images (32-bit
// index math: one image is < 2^31 elements, checked on the host)
constexpr int PACK_LIST = 48;
struct PackList {
  vits_pack16_layer l[PACK_LIST];
  int n;
};

template <typename T>
__global__ __launch_bounds__(256) void pack16_pairs_kernel(const PackList L) {
  const vits_pack16_layer& e = L.l[blockIdx.y];
  const int total = e.cin_pad * e.k * e.m_pad;
  const int end = total + e.cin_pad_t * e.k * e.m_pad_t;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < end; i += gridDim.x * 256) {
    if (i < total)
      pack16_elem32<T>(e.w, e.cout, e.cin, e.k, 0, reinterpret_cast<T*>(e.img), e.m_pad, i,
                       e.gate);
    else
      pack16_elem32<T>(e.w, e.cout, e.cin, e.k, 1, reinterpret_cast<T*>(e.img_t), e.m_pad_t,
                       i - total, 0);
  }
}

template <typename T>
__global__ void pack16_kernel(const float* __restrict__ w, int cout, int cin, int k, int transpose,
                              T* __restrict__ out, int m_pad, int cin_pad,
                              float* __restrict__ zero, int64_t zero_n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < zero_n;
       i += (int64_t)gridDim.x * blockDim.x)
    zero[i] = 0.f;
  const int total = cin_pad * k * m_pad;  // (< 2^31, checked on the host)
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x)
    pack16_elem32<T>(w, cout, cin, k, transpose, out, m_pad, i, 0);
}

}  // namespace

extern "C" int vits_conv1d_wgrad(const vits_conv1d_wgrad_desc* d, int batch, void* stream) {
  if (!d) return VITS_E_ARG;
  VITS_CHECK_ARG(d->dy && d->x && d->dw_t);
  VITS_CHECK_ARG(batch > 0 && d->cout > 0 && d->cin > 0 && d->k > 0 && d->dil > 0);
  VITS_CHECK_SHAPE(d->n_out > 0 && d->tin > 0);
  if (KT + (d->k - 1) * d->dil > MAX_WR) return VITS_E_UNSUP;
  hipStream_t s = as_stream(stream);
  if (d->wdtype == VITS_WDT_F16)
    return count_ok(wgrad_dispatch<VITS_WDT_F16, false>(*d, batch, s, 0, 0), VITS_CNT_WGRAD_16);
  if (d->wdtype == VITS_WDT_BF16)
    return count_ok(wgrad_dispatch<VITS_WDT_BF16, false>(*d, batch, s, 0, 0), VITS_CNT_WGRAD_16);
  return d->wdtype == VITS_WDT_F32 ? VITS_E_UNSUP : VITS_E_ARG;  // (fp32: split mode only)
}

extern "C" int64_t vits_conv1d_wgrad_workspace(const vits_conv1d_wgrad_desc* d, int batch) {
  if (!d || batch <= 0 || d->cout <= 0 || d->cin <= 0 || d->k <= 0 || d->n_out <= 0) return 0;
  const WgradSplit w = wgrad_split(*d, batch, true);
  return (int64_t)w.splits * ((int64_t)d->k * d->cout * d->cin + d->cout);
}

extern "C" int vits_conv1d_wgrad_split(const vits_conv1d_wgrad_desc* d, int batch, float* workspace,
                                       int64_t workspace_floats, void* stream) {
  if (!d) return VITS_E_ARG;
  VITS_CHECK_ARG(d->dy && d->x && d->dw_t && workspace);
  VITS_CHECK_ARG(batch > 0 && d->cout > 0 && d->cin > 0 && d->k > 0 && d->dil > 0);
  VITS_CHECK_SHAPE(d->n_out > 0 && d->tin > 0);
  if (d->wdtype != VITS_WDT_F32 && KT + (d->k - 1) * d->dil > MAX_WR) return VITS_E_UNSUP;
  if (workspace_floats < vits_conv1d_wgrad_workspace(d, batch)) return VITS_E_ARG;
  const WgradSplit w = wgrad_split(*d, batch, true);
  float* ws_b = workspace + (int64_t)w.splits * d->k * d->cout * d->cin;
  hipStream_t s = as_stream(stream);
  int rc;
  const bool f32 = d->wdtype == VITS_WDT_F32;
  if (f32) {
    // fp32 operands: element-wise staging
    if (d->io16) return VITS_E_UNSUP;
    if (KT32 + (d->k - 1) * d->dil > MAX_WR32) return VITS_E_UNSUP;
    rc = wgrad_f32_dispatch(*d, batch, s, workspace, ws_b);
  } else if (d->wdtype == VITS_WDT_F16)
    rc = wgrad_dispatch<VITS_WDT_F16, true>(*d, batch, s, workspace, ws_b);
  else if (d->wdtype == VITS_WDT_BF16)
    rc = wgrad_dispatch<VITS_WDT_BF16, true>(*d, batch, s, workspace, ws_b);
  else
    return VITS_E_ARG;
  if (rc) return rc;
  // split-lanes per element: enough that each thread sums <= ~16 splits
  int P = 1;
  while (P < 64 && P * 16 < w.splits) P *= 2;
  const int E = 256 / P;
  const int64_t slab = (int64_t)d->k * d->cout * d->cin;
  const int slab_blocks = (int)((slab + E - 1) / E);
  const int bias_blocks = d->dbias ? (d->cout + E - 1) / E : 0;
  const dim3 grid(slab_blocks + bias_blocks);
  switch (P) {
#define VITS_RED_CASE(PP)                                                                          \
  case PP:                                                                                         \
    hipLaunchKernelGGL(wgrad_reduce_kernel<PP>, grid, dim3(256), 0, s, workspace, ws_b, w.splits, \
                       d->k, d->cout, d->cin, slab_blocks, d->dw_t, d->dbias);                    \
    break;
    VITS_RED_CASE(1)
    VITS_RED_CASE(2)
    VITS_RED_CASE(4)
    VITS_RED_CASE(8)
    VITS_RED_CASE(16)
    VITS_RED_CASE(32)
    VITS_RED_CASE(64)
#undef VITS_RED_CASE
  }
  return count_ok(vits_launch_status(), f32 ? VITS_CNT_WGRAD_F32 : VITS_CNT_WGRAD_16, 2);
}

extern "C" int vits_conv1d_pack16_pair(const float* w, int cout, int cin, int k, void* out,
                                       int m_pad, int cin_pad, void* out_t, int m_pad_t,
                                       int cin_pad_t, int wdtype, void* stream) {
  VITS_CHECK_ARG(w && out && out_t && cout > 0 && cin > 0 && k > 0);
  VITS_CHECK_SHAPE(m_pad % 128 == 0 && m_pad >= cout && cin_pad % 16 == 0 && cin_pad >= cin);
  VITS_CHECK_SHAPE(m_pad_t % 128 == 0 && m_pad_t >= cin && cin_pad_t % 16 == 0 &&
                   cin_pad_t >= cout);
  const int64_t total = (int64_t)cin_pad * k * m_pad;
  const int64_t total_t = (int64_t)cin_pad_t * k * m_pad_t;
  VITS_CHECK_SHAPE(total + total_t < ((int64_t)1 << 31));  // (32-bit index math)
  const int64_t nblk = (total + total_t + 2047) / 2048;
  const int blocks = (int)(nblk < 8192 ? nblk : 8192);
  hipStream_t s = as_stream(stream);
  if (wdtype == VITS_WDT_F16)
    hipLaunchKernelGGL(pack16_pair_kernel<_Float16>, dim3(blocks), dim3(256), 0, s, w, cout, cin,
                       k, reinterpret_cast<_Float16*>(out), m_pad, (int)total,
                       reinterpret_cast<_Float16*>(out_t), m_pad_t, (int)total_t);
  else if (wdtype == VITS_WDT_BF16)
    hipLaunchKernelGGL(pack16_pair_kernel<__bf16>, dim3(blocks), dim3(256), 0, s, w, cout, cin, k,
                       reinterpret_cast<__bf16*>(out), m_pad, (int)total,
                       reinterpret_cast<__bf16*>(out_t), m_pad_t, (int)total_t);
  else
    return VITS_E_ARG;
  return count_ok(vits_launch_status(), VITS_CNT_PACK);
}

extern "C" int vits_conv1d_pack16(const float* w, int cout, int cin, int k, int transpose, void* out,
                                  int m_pad, int cin_pad, int wdtype, float* zero, int64_t zero_n,
                                  void* stream) {
  VITS_CHECK_ARG(zero_n >= 0 && (zero_n == 0 || zero));
  VITS_CHECK_ARG(w && out && cout > 0 && cin > 0 && k > 0);
  const int rows = transpose ? cin : cout;
  const int chans = transpose ? cout : cin;
  VITS_CHECK_SHAPE(m_pad % 128 == 0 && m_pad >= rows && cin_pad % 16 == 0 && cin_pad >= chans);
  const int64_t total = (int64_t)cin_pad * k * m_pad;
  VITS_CHECK_SHAPE(total < ((int64_t)1 << 31));  // (32-bit index math)
  const int64_t most = total > zero_n ? total : zero_n;
  const int64_t nblk = (most + 255) / 256;
  const int blocks = (int)(nblk < 4096 ? nblk : 4096);
  hipStream_t s = as_stream(stream);
  if (wdtype == VITS_WDT_F16)
    hipLaunchKernelGGL(pack16_kernel<_Float16>, dim3(blocks), dim3(256), 0, s, w, cout, cin, k,
                       transpose, reinterpret_cast<_Float16*>(out), m_pad, cin_pad, zero, zero_n);
  else if (wdtype == VITS_WDT_BF16)
    hipLaunchKernelGGL(pack16_kernel<__bf16>, dim3(blocks), dim3(256), 0, s, w, cout, cin, k,
                       transpose, reinterpret_cast<__bf16*>(out), m_pad, cin_pad, zero, zero_n);
  else
    return VITS_E_ARG;
  return count_ok(vits_launch_status(), VITS_CNT_PACK);
}

extern "C" int vits_conv1d_pack16_pairs(const vits_pack16_layer* layers, int n, int wdtype,
                                        void* stream) {
  VITS_CHECK_ARG(n >= 0 && (n == 0 || layers));
  VITS_CHECK_ARG(wdtype == VITS_WDT_F16 || wdtype == VITS_WDT_BF16);
  hipStream_t s = as_stream(stream);
  for (int b0 = 0; b0 < n; b0 += PACK_LIST) {
    PackList L;
    L.n = n - b0 < PACK_LIST ? n - b0 : PACK_LIST;
    int64_t most = 0;
    for (int q = 0; q < L.n; ++q) {
      const vits_pack16_layer& e = layers[b0 + q];
      VITS_CHECK_ARG(e.w && e.img && e.img_t && e.cout > 0 && e.cin > 0 && e.k > 0);
      VITS_CHECK_ARG(e.gate == 0 || (e.gate == 1 && (e.cout & 1) == 0));
      VITS_CHECK_SHAPE(e.m_pad % 128 == 0 && e.m_pad >= e.cout && e.cin_pad % 16 == 0 &&
                       e.cin_pad >= e.cin);
      VITS_CHECK_SHAPE(e.m_pad_t % 128 == 0 && e.m_pad_t >= e.cin && e.cin_pad_t % 16 == 0 &&
                       e.cin_pad_t >= e.cout);
      const int64_t both = (int64_t)e.cin_pad * e.k * e.m_pad +
                           (int64_t)e.cin_pad_t * e.k * e.m_pad_t;
      VITS_CHECK_SHAPE(both < ((int64_t)1 << 31) &&
                       (int64_t)e.cout * e.cin * e.k < ((int64_t)1 << 31));
      L.l[q] = e;
      if (both > most) most = both;
    }
    // ~8 elements per thread for the largest layer, at most 1024 blocks each
    const int64_t bx = (most + 2047) / 2048;
    const dim3 grid((unsigned)(bx < 1024 ? (bx < 1 ? 1 : bx) : 1024), (unsigned)L.n);
    if (wdtype == VITS_WDT_F16)
      hipLaunchKernelGGL(pack16_pairs_kernel<_Float16>, grid, dim3(256), 0, s, L);
    else
      hipLaunchKernelGGL(pack16_pairs_kernel<__bf16>, grid, dim3(256), 0, s, L);
    const int rc = count_ok(vits_launch_status(), VITS_CNT_PACK);
    if (rc) return rc;
  }
  return VITS_OK;
}
