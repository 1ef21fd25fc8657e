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
//  * the backtrack decision for (y, x) is V[y-1][x] < V[y-1][x-1]; wave 0
//    produces it for a whole row with one ballot per register column and
//    keeps the bits in LDS (global workspace when they do not fit), so the
//    sequential backtrack reads one bit per row from LDS;
//  * the path is written in one coalesced pass from the per-row column index.
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
                                                  uint64_t* __restrict__ bits_global,
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
  // compile-time address space for the decision bits: LDS (ds_read/write)
  // or the global workspace -- a runtime select would make every access a
  // FLAT op waiting on both counters
  uint64_t* bits;
  if constexpr (BITS_LDS)
    bits = reinterpret_cast<uint64_t*>(idx_row + ((T_t + 1) & ~1));
  else
    bits = bits_global + (int64_t)b * T_t * XPL;

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
#pragma unroll
  for (int i = 0; i < XPL; ++i) vp[i] = 0.f;
  const int xbase = lane * XPL;

  for (int ch = 0; ch < nchunks; ++ch) {
    if (wid != 0) {
      if (ch + 1 < nchunks) load_chunk(ch + 1, (ch + 1) & 1, 1, 3);
    } else {
      const float* rows = ring + (ch & 1) * R * W;
      const int y0 = ch * R;
      const int yend = min(t_t, y0 + R);
      // the next row's scores are read from LDS while this row computes
      float nxt[XPL];
      if (y0 < yend) {
#pragma unroll
        for (int i = 0; i < XPL; ++i) nxt[i] = rows[xbase + i];
      }
      for (int y = y0; y < yend; ++y) {
        float cur[XPL];
#pragma unroll
        for (int i = 0; i < XPL; ++i) cur[i] = nxt[i];
        if (y + 1 < yend) {
          const float* rown = rows + (y + 1 - y0) * W + xbase;
#pragma unroll
          for (int i = 0; i < XPL; ++i) nxt[i] = rown[i];
        }
        const int lo = max(0, t_s + y - t_t);
        const int hi = min(t_s, y + 1);
        // column x-1 of this lane's first element: lane-1's last register,
        // one DPP wave shift (no LDS round trip; lane 0 never uses it)
        const float left = __int_as_float(
            __builtin_amdgcn_update_dpp(0, __float_as_int(vp[XPL - 1]), 0x138, 0xf, 0xf, false));
        float vn[XPL];
#pragma unroll
        for (int i = 0; i < XPL; ++i) {
          const int x = xbase + i;
          const float vcur_raw = vp[i];
          const float vprev_raw = (i == 0) ? left : vp[i - 1];
          // decision bit for the backtrack at (y, x): V[y-1][x] < V[y-1][x-1]
          const bool dec = (y >= 1) && (x >= 1) && (vcur_raw < vprev_raw);
          const unsigned long long m = __ballot(dec);
          if (lane == 0) bits[(int64_t)y * XPL + i] = m;
          float v = cur[i];
          if (x >= lo && x < hi) {
            const float v_cur = (x == y) ? MAS_NEG : vcur_raw;
            const float v_prev = (x == 0) ? (y == 0 ? 0.f : MAS_NEG) : vprev_raw;
            const float mx = (v_cur > v_prev) ? v_cur : v_prev;  // Cython max(v_prev, v_cur)
            v = v + mx;
          }
          vn[i] = v;
        }
#pragma unroll
        for (int i = 0; i < XPL; ++i) vp[i] = vn[i];
      }
    }
    __syncthreads();
  }

  // ---- backtrack (one lane) -------------------------------------------------
  if (tid == 0) {
    int index = t_s - 1;
    for (int y = t_t - 1; y >= 0; --y) {
      idx_row[y] = index;
      if (index != 0) {
        bool dec = (index == y);
        if (!dec && y >= 1 && index >= 0) {
          const int l = index / XPL;
          const int i = index - l * XPL;
          dec = (bits[(int64_t)y * XPL + i] >> l) & 1ull;
        }
        if (dec) index = index - 1;
      }
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

size_t bits_bytes(int t_t, int xpl) { return (size_t)t_t * xpl * sizeof(uint64_t); }

int mas_run(const float* neg_cent, const int32_t* tt, const int32_t* ts, void* path, int path_dt,
            int batch, int T_t, int T_s, void* workspace, int64_t ws_bytes, hipStream_t s) {
  const int xpl = pick_xpl(T_s);
  if (xpl > 32) return VITS_E_UNSUP;
  const size_t ring = sizeof(float) * 2 * mas_rows(xpl) * 64 * xpl;
  const size_t idx = sizeof(int32_t) * ((T_t + 1) & ~1);
  const size_t bb = bits_bytes(T_t, xpl);
  int in_lds = bb <= (size_t)MAS_BITS_LDS_MAX && ring + idx + bb <= 150 * 1024;
  size_t lds = ring + idx + (in_lds ? bb : 0);
  uint64_t* gbits = nullptr;
  if (!in_lds) {
    if (!workspace || ws_bytes < (int64_t)(bb * batch)) return VITS_E_ARG;
    gbits = reinterpret_cast<uint64_t*>(workspace);
  }
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
  const size_t idx = sizeof(int32_t) * ((t_t + 1) & ~1);
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
