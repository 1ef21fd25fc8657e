// mas.hip — monotonic alignment search on gfx950.
//
// Replaces the external Cython `monotonic_align.maximum_path` that
// SynthesizerTrn.forward calls at models.py:498 (layout [b, t_t(frames),
// t_s(tokens)] per models.py:486-497).  The package is not vendored in the
// reference (README.md:9); the algorithm restated here and in
// oracle/mas_oracle.c is the canonical VITS core.pyx:
//   forward:  for y < t_t, x in [max(0, t_s+y-t_t), min(t_s, y+1)):
//               v_cur  = x == y ? -1e9 : V[y-1][x]
//               v_prev = x == 0 ? (y == 0 ? 0 : -1e9) : V[y-1][x-1]
//               V[y][x] += max(v_prev, v_cur)      (Cython max: b > a ? b : a)
//   backtrack: idx = t_s-1; for y = t_t-1 .. 0:
//               P[y][idx] = 1
//               if idx != 0 && (idx == y || V[y-1][idx] < V[y-1][idx-1]): idx--
// Only fp32 adds and compares: the result is bit-exact by construction.
//
// Design (one workgroup = 4 waves = one utterance):
//  * the DP is a wavefront over rows: wave 0 holds a whole row in registers,
//    XPL contiguous columns per lane; column x-1 of lane 0's first element
//    comes from lane-1 by one shuffle, so a row costs ~XPL VALU ops and one
//    cross-lane op, no barrier;
//  * waves 1-3 stream the next chunk of neg_cent rows (R rows, coalesced)
//    into an LDS double buffer while wave 0 consumes the current one, one
//    barrier per chunk;
//  * the backtrack decision for (y, x) is V[y-1][x] < V[y-1][x-1]; each lane
//    ORs it into a register word per column (bit y mod 32) and stores the
//    words once per 32 rows (LDS, or the global workspace when they do not
//    fit): no per-row ballot, SALU hop or LDS store on the DP's chain;
//  * the backtrack runs on wave 0: per 32-row block, lane l holds the
//    decision word of column index - l (the path moves at most one column
//    per row), and each row is a readlane + bit test - no memory latency
//    per row;
//  * the path is written in one coalesced pass from the per-row column index.
// (Round 5: per-row ballots + a one-lane backtrack, 194 us at B=64, 500 x 100.)
#include "common.h"

namespace {

// rows per streamed chunk: as many as keep the two ring buffers within
// MAS_RING_BYTES, so wave 0's compute per chunk outlasts one HBM round trip
constexpr int MAS_RING_BYTES = 64 * 1024;
__host__ __device__ inline int mas_rows(int xpl) {
  int r = MAS_RING_BYTES / (2 * 64 * xpl * (int)sizeof(float));
  return r > 64 ? 64 : (r < 4 ? 4 : r);
}
constexpr float MAS_NEG = -1e9f;
constexpr int MAS_BITS_LDS_MAX = 48 * 1024;

template <typename T>
__device__ __forceinline__ float to_f(T v);
template <>
__device__ __forceinline__ float to_f<float>(float v) { return v; }
template <>
__device__ __forceinline__ float to_f<_Float16>(_Float16 v) { return (float)v; }
template <>
__device__ __forceinline__ float to_f<int32_t>(int32_t v) { return (float)v; }
template <>
__device__ __forceinline__ float to_f<uint16_t>(uint16_t v) {  // bf16 bits
  return __uint_as_float(((uint32_t)v) << 16);
}

__device__ __forceinline__ float load_dt(const void* p, int dt, int64_t i) {
  switch (dt) {
    case VITS_DT_F16: return to_f(reinterpret_cast<const _Float16*>(p)[i]);
    case VITS_DT_BF16: return to_f(reinterpret_cast<const uint16_t*>(p)[i]);
    case VITS_DT_I32: return to_f(reinterpret_cast<const int32_t*>(p)[i]);
    default: return reinterpret_cast<const float*>(p)[i];
  }
}

__device__ __forceinline__ void store_dt(void* p, int dt, int64_t i, float v) {
  switch (dt) {
    case VITS_DT_F16: reinterpret_cast<_Float16*>(p)[i] = (_Float16)v; break;
    case VITS_DT_BF16: reinterpret_cast<uint16_t*>(p)[i] = (uint16_t)(__float_as_uint(v) >> 16); break;
    case VITS_DT_I32: reinterpret_cast<int32_t*>(p)[i] = (int32_t)v; break;
    default: reinterpret_cast<float*>(p)[i] = v;
  }
}

// lengths from the mask, as monotonic_align/__init__.py: mask.sum(1)[:,0]
// and mask.sum(2)[:,0] (sums of 0/1 values are exact in fp32).
__global__ __launch_bounds__(64) void mas_lengths_kernel(const void* mask, int dt, int t_t, int t_s,
                                                         int32_t* tt_len, int32_t* ts_len) {
  const int b = blockIdx.x;
  const int lane = threadIdx.x;
  const int64_t base = (int64_t)b * t_t * t_s;
  float sy = 0.f, sx = 0.f;
  for (int y = lane; y < t_t; y += 64) sy += load_dt(mask, dt, base + (int64_t)y * t_s);
  for (int x = lane; x < t_s; x += 64) sx += load_dt(mask, dt, base + x);
  sy = wave_sum(sy);
  sx = wave_sum(sx);
  if (lane == 0) {
    tt_len[b] = (int32_t)sy;
    ts_len[b] = (int32_t)sx;
  }
}

template <int XPL, bool BITS_LDS>
__global__ __launch_bounds__(256) void mas_kernel(const float* __restrict__ neg_cent,
                                                  const int32_t* __restrict__ tt_len,
                                                  const int32_t* __restrict__ ts_len, void* path,
                                                  int path_dt, int T_t, int T_s,
                                                  uint32_t* __restrict__ bits_global,
                                                  int bits_in_lds) {
  extern __shared__ __align__(16) unsigned char smem_raw[];
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int W = 64 * XPL;  // padded row width in LDS (>= T_s)

  const int R = mas_rows(XPL);
  float* ring = reinterpret_cast<float*>(smem_raw);             // [2][R][W]
  int32_t* idx_row = reinterpret_cast<int32_t*>(ring + 2 * R * W);  // [T_t]
  // decision words [ceil(T_t / 32)][W]: bit (y mod 32) of word (y / 32, x).
  // Compile-time address space: LDS (ds_read/write) or the global workspace
  // -- a runtime select would make every access a FLAT op waiting on both
  // counters
  uint32_t* bits;
  if constexpr (BITS_LDS)
    bits = reinterpret_cast<uint32_t*>(idx_row + ((T_t + 3) & ~3));
  else
    bits = bits_global + (int64_t)b * ((T_t + 31) >> 5) * W;

  int t_t = tt_len[b];
  int t_s = ts_len[b];
  t_t = t_t < 0 ? 0 : (t_t > T_t ? T_t : t_t);
  t_s = t_s < 0 ? 0 : (t_s > T_s ? T_s : t_s);

  const float* nc = neg_cent + (int64_t)b * T_t * T_s;
  const int nchunks = (t_t + R - 1) / R;

  // chunk -> LDS by LDS-DMA (4 bytes per lane, 64 floats per wave
  // instruction, all in flight at once; no registers, no per-load waits).
  // Columns >= t_s and rows >= t_t read clamped in-bounds addresses: the DP
  // never uses them (x < hi <= t_s, y < t_t).
  auto load_chunk = [&](int ch, int buf, int w0, int nw) {
    float* dst = ring + buf * R * W;
    const int y0 = ch * R;
    const int pieces = R * W / 64;
    for (int q = (tid >> 6) - w0; q < pieces; q += nw) {
      const int r = (q * 64) / W;
      const int x = q * 64 - r * W + (tid & 63);
      const int y = min(y0 + r, T_t - 1);
      const int xc = min(x, T_s - 1);
      __builtin_amdgcn_global_load_lds(nc + (int64_t)y * T_s + xc,
                                       (__attribute__((address_space(3))) void*)(dst + q * 64),
                                       4, 0, 0);
    }
  };

  if (nchunks > 0) load_chunk(0, 0, 0, 4);
  __syncthreads();

  float vp[XPL];
  uint32_t dw[XPL];  // this lane's decision words of the current 32-row block
  // the DP band: cell (y, x) is updated iff lo <= x < hi, lo = max(0, t_s +
  // y - t_t), hi = min(t_s, y + 1), i.e. iff 0 <= y - x <= D = t_t - t_s
  // and x < t_s: one unsigned compare of y - xs against D, with xs = x, or
  // a value no y reaches for columns outside [0, t_s) (and every column
  // when t_s > t_t: then no cell is updated)
  const int D = t_t - t_s;
  const uint32_t Du = D < 0 ? 0u : (uint32_t)D;
  int xs[XPL];
#pragma unroll
  for (int i = 0; i < XPL; ++i) {
    vp[i] = 0.f;
    dw[i] = 0u;
    const int x = lane * XPL + i;
    xs[i] = (x < t_s && D >= 0) ? x : 0x40000000;
  }
  const int xbase = lane * XPL;

  for (int ch = 0; ch < nchunks; ++ch) {
    if (wid != 0) {
      if (ch + 1 < nchunks) load_chunk(ch + 1, (ch + 1) & 1, 1, 3);
    } else {
      const float* rows = ring + (ch & 1) * R * W;
      const int y0 = ch * R;
      const int yend = min(t_t, y0 + R);
      // two row registers, no moves between them: row y + 2's scores are
      // read into ra right after row y consumed it, i.e. one row of work
      // ahead of their use (reads past the chunk's last row land in
      // allocated LDS and are never used)
      float ra[XPL], rb[XPL];
      auto rd = [&](float* r, int y) {
        const float* src = rows + (y - y0) * W + xbase;
#pragma unroll
        for (int i = 0; i < XPL; ++i) r[i] = src[i];
      };
      auto row = [&](int y, const float* cur) {
        // column x-1 of this lane's first element: lane-1's last register,
        // one DPP wave shift; lane 0 (x = 0) receives the DP's left
        // boundary V[y-1][-1] = (y == 0 ? 0 : -1e9) as the shift's fill
        const float bnd = y == 0 ? 0.f : MAS_NEG;
        const float left = __int_as_float(__builtin_amdgcn_update_dpp(
            __float_as_int(bnd), __float_as_int(vp[XPL - 1]), 0x138, 0xf, 0xf, false));
        const uint32_t bit = 1u << (y & 31);
        float vn[XPL];
#pragma unroll
        for (int i = 0; i < XPL; ++i) {
          const float vcur_raw = vp[i];
          const float vprev_raw = (i == 0) ? left : vp[i - 1];
          // backtrack decision at (y, x): V[y-1][x] < V[y-1][x-1]
          // (consulted only for y >= 1, x >= 1)
          dw[i] |= (vcur_raw < vprev_raw) ? bit : 0u;
          const uint32_t dy = (uint32_t)(y - xs[i]);
          const float v_cur = dy == 0u ? MAS_NEG : vcur_raw;         // x == y
          const float mx = (v_cur > vprev_raw) ? v_cur : vprev_raw;  // Cython max(v_prev, v_cur)
          const float upd = cur[i] + mx;
          vn[i] = dy <= Du ? upd : cur[i];
        }
#pragma unroll
        for (int i = 0; i < XPL; ++i) vp[i] = vn[i];
        if ((y & 31) == 31 || y == t_t - 1) {  // block of 32 rows complete
#pragma unroll
          for (int i = 0; i < XPL; ++i) {
            bits[(int64_t)(y >> 5) * W + xbase + i] = dw[i];
            dw[i] = 0u;
          }
        }
      };
      rd(ra, y0);
      rd(rb, y0 + 1);
      for (int y = y0; y < yend; y += 2) {
        row(y, ra);
        rd(ra, y + 2);
        if (y + 1 < yend) {
          row(y + 1, rb);
          rd(rb, y + 3);
        }
      }
    }
    __syncthreads();
  }

  // ---- backtrack (wave 0) ---------------------------------------------------
  // index is wave-uniform; per 32-row block lane l < 32 holds the decision
  // word of column top - l, top = index at the block's last row
  if (wid == 0 && t_t > 0 && t_s > 0) {
    int index = t_s - 1;
    int my_idx = 0;  // lane l: the path column of row 32 * blk + l
    for (int blk = (t_t - 1) >> 5; blk >= 0; --blk) {
      const int top = index;
      const int col = top - lane;
      const uint32_t wv = (lane < 32 && col >= 0) ? bits[(int64_t)blk * W + col] : 0u;
      const int yhi = min(t_t - 1, blk * 32 + 31);
      for (int y = yhi; y >= blk * 32; --y) {
        my_idx = (lane == (y & 31)) ? index : my_idx;
        if (index != 0) {
          bool dec = (index == y);
          if (!dec && y >= 1) {
            const uint32_t w = __builtin_amdgcn_readlane(wv, top - index);
            dec = (w >> (y & 31)) & 1u;
          }
          if (dec) index = index - 1;
        }
      }
      if (lane < 32 && blk * 32 + lane <= yhi) idx_row[blk * 32 + lane] = my_idx;
    }
  }
  __syncthreads();

  // ---- write the full path tile ---------------------------------------------
  // one wave per row, lanes along the row: coalesced, no index division
  const int64_t pbase = (int64_t)b * T_t * T_s;
  for (int y = wid; y < T_t; y += 4) {
    const int sel = (y < t_t && t_s > 0) ? idx_row[y] : -1;
    const int64_t rbase = pbase + (int64_t)y * T_s;
    for (int x = lane; x < T_s; x += 64) store_dt(path, path_dt, rbase + x, x == sel ? 1.f : 0.f);
  }
}

int pick_xpl(int t_s) {
  const int need = (t_s + 63) / 64;
  int xpl = 1;
  while (xpl < need) xpl <<= 1;
  return xpl;
}

size_t bits_bytes(int t_t, int xpl) {
  return (size_t)((t_t + 31) / 32) * 64 * xpl * sizeof(uint32_t);
}

int mas_run(const float* neg_cent, const int32_t* tt, const int32_t* ts, void* path, int path_dt,
            int batch, int T_t, int T_s, void* workspace, int64_t ws_bytes, hipStream_t s) {
  const int xpl = pick_xpl(T_s);
  if (xpl > 32) return VITS_E_UNSUP;
  const size_t ring = sizeof(float) * 2 * mas_rows(xpl) * 64 * xpl;
  const size_t idx = sizeof(int32_t) * ((T_t + 3) & ~3);
  const size_t bb = bits_bytes(T_t, xpl);
  int in_lds = bb <= (size_t)MAS_BITS_LDS_MAX && ring + idx + bb <= 150 * 1024;
  size_t lds = ring + idx + (in_lds ? bb : 0);
  uint32_t* gbits = nullptr;
  if (!in_lds) {
    if (!workspace || ws_bytes < (int64_t)(bb * batch)) return VITS_E_ARG;
    gbits = reinterpret_cast<uint32_t*>(workspace);
  }
  // (three rows of slack past the ring: the DP reads up to 3 rows ahead)
  lds += sizeof(float) * 3 * 64 * xpl;
  if (lds > 160 * 1024) return VITS_E_UNSUP;
  dim3 grid(batch), block(256);
#define MAS_CASE(X)                                                                         \
  case X:                                                                                   \
    if (in_lds)                                                                             \
      hipLaunchKernelGGL((mas_kernel<X, true>), grid, block, lds, s, neg_cent, tt, ts, path, \
                         path_dt, T_t, T_s, gbits, in_lds);                                 \
    else                                                                                    \
      hipLaunchKernelGGL((mas_kernel<X, false>), grid, block, lds, s, neg_cent, tt, ts, path, \
                         path_dt, T_t, T_s, gbits, in_lds);                                 \
    break;
  switch (xpl) {
    MAS_CASE(1)
    MAS_CASE(2)
    MAS_CASE(4)
    MAS_CASE(8)
    MAS_CASE(16)
    MAS_CASE(32)
    default:
      return VITS_E_UNSUP;
  }
#undef MAS_CASE
  return vits_launch_status();
}

}  // namespace

extern "C" int64_t vits_maximum_path_workspace(int batch, int t_t, int t_s) {
  if (batch <= 0 || t_t <= 0 || t_s <= 0) return 0;
  const int xpl = pick_xpl(t_s);
  const size_t ring = sizeof(float) * 2 * mas_rows(xpl) * 64 * xpl;
  const size_t idx = sizeof(int32_t) * ((t_t + 3) & ~3);
  const size_t bb = bits_bytes(t_t, xpl);
  const bool in_lds = bb <= (size_t)MAS_BITS_LDS_MAX && ring + idx + bb <= 150 * 1024;
  // always reserve room for the two length vectors of vits_maximum_path
  return (int64_t)(in_lds ? 0 : bb * batch) + 2 * sizeof(int32_t) * (int64_t)batch + 256;
}

extern "C" int vits_maximum_path_lengths(const float* neg_cent, const int32_t* t_t_len,
                                         const int32_t* t_s_len, void* path, int path_dtype,
                                         int batch, int t_t, int t_s, void* workspace,
                                         int64_t workspace_bytes, void* stream) {
  VITS_CHECK_ARG(neg_cent && t_t_len && t_s_len && path && batch > 0 && t_t > 0 && t_s > 0);
  VITS_CHECK_ARG(path_dtype >= 0 && path_dtype <= 3);
  return mas_run(neg_cent, t_t_len, t_s_len, path, path_dtype, batch, t_t, t_s, workspace,
                 workspace_bytes, as_stream(stream));
}

extern "C" int vits_maximum_path(const float* neg_cent, const void* mask, int mask_dtype,
                                 void* path, int path_dtype, int batch, int t_t, int t_s,
                                 void* workspace, int64_t workspace_bytes, void* stream) {
  VITS_CHECK_ARG(neg_cent && mask && path && workspace && batch > 0 && t_t > 0 && t_s > 0);
  VITS_CHECK_ARG(mask_dtype >= 0 && mask_dtype <= 3 && path_dtype >= 0 && path_dtype <= 3);
  if (workspace_bytes < vits_maximum_path_workspace(batch, t_t, t_s)) return VITS_E_ARG;
  // lengths live at the tail of the workspace
  char* wsb = reinterpret_cast<char*>(workspace);
  const int64_t lens_off = workspace_bytes - 2 * sizeof(int32_t) * (int64_t)batch;
  const int64_t aligned = lens_off & ~(int64_t)15;
  int32_t* tt = reinterpret_cast<int32_t*>(wsb + aligned);
  int32_t* ts = tt + batch;
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(mas_lengths_kernel, dim3(batch), dim3(64), 0, s, mask, mask_dtype, t_t, t_s,
                     tt, ts);
  int rc = vits_launch_status();
  if (rc) return rc;
  return mas_run(neg_cent, tt, ts, path, path_dtype, batch, t_t, t_s, workspace, aligned, s);
}
