// negcent.hip — the alignment score matrix of SynthesizerTrn.forward
// (models.py:483-490) on gfx950 fp32 MFMA, one kernel instead of the
// reference's exp / 2 matmuls / 2 reductions / 3 adds:
//
//   s = exp(-2 logs_p)                                  [B][C][t_s]
//   neg_cent[b][y][x] = sum_d ( -0.5 log(2 pi) - logs_p[d][x]
//                               - 0.5 z_p[d][y]^2 s[d][x]
//                               + z_p[d][y] m_p[d][x] s[d][x]
//                               - 0.5 m_p[d][x]^2 s[d][x] )
//
// GEMM view per utterance: rows y (t_t, mel frames), columns x (t_s, text
// tokens), K = 2C: A = [-0.5 z^2 | z] (read from z_p [C][t_t], y contiguous),
// B = [s | m s] (computed on the fly from m_p / logs_p [C][t_s]).  The
// per-column constant sum_d(-0.5 log 2pi - logs - 0.5 m^2 s) is reduced by
// the same wave.  One wave = one 32x32 output tile; lane l holds column
// x0 + (l & 31), so every load and the store are 128-byte coalesced.
#include "common.h"

namespace {

__global__ __launch_bounds__(64) void neg_cent_kernel(const float* __restrict__ z,
                                                      const float* __restrict__ m,
                                                      const float* __restrict__ logs,
                                                      float* __restrict__ out, int C, int Tt,
                                                      int Ts) {
  const int lane = threadIdx.x;
  const int l32 = lane & 31;
  const int lhi = lane >> 5;
  const int x0 = blockIdx.x * 32;
  const int y0 = blockIdx.y * 32;
  const int b = blockIdx.z;
  const float* zb = z + (int64_t)b * C * Tt;
  const float* mb = m + (int64_t)b * C * Ts;
  const float* lb = logs + (int64_t)b * C * Ts;
  const int x = x0 + l32;
  const int y = y0 + l32;
  const bool xv = x < Ts;
  const bool yv = y < Tt;
  constexpr float kHalfLog2Pi = 0.918938533204672742f;  // 0.5 * log(2 pi)

  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  float colc = 0.f;  // this lane's half of the per-column constant
  for (int d0 = 0; d0 < C; d0 += 2) {
    const int d = d0 + lhi;
    float zv = 0.f, sv = 0.f, msv = 0.f;
    if (d < C) {
      if (yv) zv = zb[(int64_t)d * Tt + y];
      if (xv) {
        const float lv = lb[(int64_t)d * Ts + x];
        const float mv = mb[(int64_t)d * Ts + x];
        sv = expf(-2.0f * lv);
        msv = mv * sv;
        colc += -kHalfLog2Pi - lv - 0.5f * (mv * mv) * sv;
      }
    }
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(-0.5f * zv * zv, sv, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(zv, msv, acc, 0, 0, 0);
  }
  colc += __shfl_xor(colc, 32, 64);
  if (!xv) return;
  float* ob = out + (int64_t)b * Tt * Ts;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = y0 + (r & 3) + 8 * (r >> 2) + 4 * lhi;
    if (row < Tt) ob[(int64_t)row * Ts + x] = acc[r] + colc;
  }
}

// v2: one workgroup = one 32-column x tile of one utterance and 8 y tiles
// (two per wave, y0 and y0 + 128, as two independent accumulator chains).  The B operand of every d (s = exp(-2 logs), m s) and the
// per-column constant are computed ONCE per workgroup into LDS (v1 recomputed
// them in each of the t_t/32 waves of a column tile, exp included), and each
// wave prefetches its z_p rows 8 channel pairs ahead of the MFMAs, so the
// kernel runs at the MFMA rate instead of the load latency.
constexpr int NC_PF = 8;  // channel pairs per prefetch group

__global__ __launch_bounds__(256) void neg_cent_kernel2(const float* __restrict__ z,
                                                        const float* __restrict__ m,
                                                        const float* __restrict__ logs,
                                                        float* __restrict__ out, int C, int Tt,
                                                        int Ts) {
  extern __shared__ float lds[];
  float* sS = lds;                 // [C][32]   s
  float* sMS = lds + C * 32;       // [C][32]   m s
  float* cpart = sMS + C * 32;     // [8][32]   per-column constant partials
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int l32 = lane & 31;
  const int lhi = lane >> 5;
  const int x0 = blockIdx.x * 32;
  const int b = blockIdx.z;
  const float* mb = m + (int64_t)b * C * Ts;
  const float* lb = logs + (int64_t)b * C * Ts;
  constexpr float kHalfLog2Pi = 0.918938533204672742f;  // 0.5 * log(2 pi)
  {
    const int xl = tid & 31;
    const int x = x0 + xl;
    float cp = 0.f;
    // 8 rows (d) per thread in flight at once: the loads of a group are all
    // issued before the first is used (a load-use chain per row would
    // serialise ~C/8 global latencies)
    constexpr int G = 8;
    for (int d0 = tid >> 5; d0 < C; d0 += 8 * G) {
      float lv[G], mv[G];
#pragma unroll
      for (int i = 0; i < G; ++i) {
        const int d = d0 + 8 * i;
        const bool ok = d < C && x < Ts;
        lv[i] = ok ? lb[(int64_t)d * Ts + x] : 0.f;
        mv[i] = ok ? mb[(int64_t)d * Ts + x] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < G; ++i) {
        const int d = d0 + 8 * i;
        if (d < C) {
          float sv = 0.f, msv = 0.f;
          if (x < Ts) {
            sv = expf(-2.0f * lv[i]);
            msv = mv[i] * sv;
            cp += -kHalfLog2Pi - lv[i] - 0.5f * (mv[i] * mv[i]) * sv;
          }
          sS[d * 32 + xl] = sv;
          sMS[d * 32 + xl] = msv;
        }
      }
    }
    cpart[tid] = cp;
  }
  __syncthreads();
  // two y tiles per wave (rows y0 and y0 + 128): two independent MFMA
  // accumulator chains sharing every B-operand LDS read
  const int y0 = (blockIdx.y * 8 + wid) * 32;
  if (y0 >= Tt) return;
  float colc = 0.f;
#pragma unroll
  for (int q = 0; q < 8; ++q) colc += cpart[q * 32 + l32];
  const int ya = y0 + l32;
  const int yb = ya + 128;
  const bool yva = ya < Tt;
  const bool yvb = yb < Tt;
  const float* zb = z + (int64_t)b * C * Tt;
  const float* za = zb + (yva ? ya : 0);
  const float* zbb = zb + (yvb ? yb : 0);
  f32x16 acc0, acc1;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    acc0[r] = 0.f;
    acc1[r] = 0.f;
  }
  const int pairs = (C + 1) >> 1;
  float zna[NC_PF], znb[NC_PF];
  auto zload = [&](int p0) {
#pragma unroll
    for (int i = 0; i < NC_PF; ++i) {
      const int d = 2 * (p0 + i) + lhi;
      zna[i] = (yva && d < C) ? za[(int64_t)d * Tt] : 0.f;
      znb[i] = (yvb && d < C) ? zbb[(int64_t)d * Tt] : 0.f;
    }
  };
  zload(0);
  for (int p0 = 0; p0 < pairs; p0 += NC_PF) {
    float zca[NC_PF], zcb[NC_PF];
#pragma unroll
    for (int i = 0; i < NC_PF; ++i) {
      zca[i] = zna[i];
      zcb[i] = znb[i];
    }
    if (p0 + NC_PF < pairs) zload(p0 + NC_PF);
#pragma unroll
    for (int i = 0; i < NC_PF; ++i) {
      const int d = 2 * (p0 + i) + lhi;
      const bool dv = d < C;
      const float sv = dv ? sS[d * 32 + l32] : 0.f;
      const float msv = dv ? sMS[d * 32 + l32] : 0.f;
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(-0.5f * zca[i] * zca[i], sv, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(-0.5f * zcb[i] * zcb[i], sv, acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(zca[i], msv, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(zcb[i], msv, acc1, 0, 0, 0);
    }
  }
  const int x = x0 + l32;
  if (x >= Ts) return;
  float* ob = out + (int64_t)b * Tt * Ts;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = y0 + (r & 3) + 8 * (r >> 2) + 4 * lhi;
    if (row < Tt) ob[(int64_t)row * Ts + x] = acc0[r] + colc;
    if (row + 128 < Tt) ob[(int64_t)(row + 128) * Ts + x] = acc1[r] + colc;
  }
}

// v3: the same GEMM in fp32 arithmetic on the bf16 MFMA - the conv kernels'
// exact three-way split (conv1d_impl.h split3_bf16: x == h + m + l bit for
// bit), six v_mfma_f32_32x32x16_bf16 per 16-deep step instead of eight
// 32x32x2 f32 MFMAs at 1/16 of the rate.  A 16-deep step covers channels
// 8t .. 8t + 8 of BOTH terms: lanes of the low half hold -0.5 z^2, of the
// high half z (A); s and m s likewise (B).  B is computed once per workgroup
// into three bf16 planes [t][half][x][8] (one 16-byte read per lane and
// plane); A is split in registers from z loaded one step ahead.  Error:
// the split products are exact, the three dropped cross terms < 2^-22 of
// the product, fp32 accumulation - the f32 MFMA kernel's error level
// (tests/test_kernels_gpu.py::test_neg_cent, 2e-6 of max|nc| vs fp64).
typedef __bf16 nc_bf16x8 __attribute__((ext_vector_type(8)));
typedef float nc_f32x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void nc_split3(const nc_f32x8& x, nc_bf16x8& h, nc_bf16x8& m,
                                          nc_bf16x8& l) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float xe = x[e];
    const float hf = __uint_as_float(__float_as_uint(xe) & 0xffff0000u);
    const float r = xe - hf;
    const float mf = __uint_as_float(__float_as_uint(r) & 0xffff0000u);
    h[e] = (__bf16)hf;
    m[e] = (__bf16)mf;
    l[e] = (__bf16)(r - mf);
  }
}

constexpr int NC3_PF = 2;  // 16-deep steps per z prefetch group

__host__ __device__ inline int nc3_lds_bytes(int C) {
  const int ns = (C + 7) / 8;
  return 3 * ns * 2 * 32 * 8 * 2 + 256 * 4;
}

__global__ __launch_bounds__(256, 2) void neg_cent_kernel3(const float* __restrict__ z,
                                                           const float* __restrict__ m,
                                                           const float* __restrict__ logs,
                                                           float* __restrict__ out, int C, int Tt,
                                                           int Ts, int batch) {
  extern __shared__ float lds3[];
  const int NS = (C + 7) >> 3;          // 16-deep steps
  const int PL = NS * 2 * 32 * 8;       // elements per B plane
  __bf16* const bpl = reinterpret_cast<__bf16*>(lds3);
  float* const cpart = lds3 + (3 * PL) / 2;  // [8][32] per-column constant partials
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int l32 = lane & 31;
  const int lhi = lane >> 5;
  // 1-D grid, XCD-aware: workgroups wg, wg + 8, ... run on one XCD (the
  // dispatcher deals workgroups round-robin over the 8 XCDs), so the nx
  // column tiles of one (utterance, row block) are given consecutive
  // multiples of 8 - their z rows are fetched into that XCD's L2 once
  // instead of once per XCD
  const int nx = (Ts + 31) >> 5;
  const int nyb = (Tt + 255) >> 8;
  const int wg = blockIdx.x;
  const int xt = (wg >> 3) % nx;
  const int yq = (wg / (8 * nx)) * 8 + (wg & 7);  // (row block, utterance) index
  if (yq >= nyb * batch) return;
  const int b = yq / nyb;
  const int yblk = yq - b * nyb;
  const int x0 = xt * 32;
  const float* mb = m + (int64_t)b * C * Ts;
  const float* lb = logs + (int64_t)b * C * Ts;
  constexpr float kHalfLog2Pi = 0.918938533204672742f;  // 0.5 * log(2 pi)
  {
    // B = (s, m s) of channel d, column x -> planes [d / 8][half][x][d % 8]
    const int xl = tid & 31;
    const int x = x0 + xl;
    float cp = 0.f;
    constexpr int G = 8;  // rows per thread in flight
    for (int d0 = tid >> 5; d0 < NS * 8; d0 += 8 * G) {
      float lv[G], mv[G];
#pragma unroll
      for (int i = 0; i < G; ++i) {
        const int d = d0 + 8 * i;
        const bool ok = d < C && x < Ts;
        lv[i] = ok ? lb[(int64_t)d * Ts + x] : 0.f;
        mv[i] = ok ? mb[(int64_t)d * Ts + x] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < G; ++i) {
        const int d = d0 + 8 * i;
        if (d < NS * 8) {
          float sv = 0.f, msv = 0.f;
          if (d < C && x < Ts) {
            sv = expf(-2.0f * lv[i]);
            msv = mv[i] * sv;
            cp += -kHalfLog2Pi - lv[i] - 0.5f * (mv[i] * mv[i]) * sv;
          }
          const int t = d >> 3, e = d & 7;
#pragma unroll
          for (int hh = 0; hh < 2; ++hh) {
            const float v = hh ? msv : sv;
            const float hf = __uint_as_float(__float_as_uint(v) & 0xffff0000u);
            const float r = v - hf;
            const float mf = __uint_as_float(__float_as_uint(r) & 0xffff0000u);
            const int o = ((t * 2 + hh) * 32 + xl) * 8 + e;
            bpl[o] = (__bf16)hf;
            bpl[PL + o] = (__bf16)mf;
            bpl[2 * PL + o] = (__bf16)(r - mf);
          }
        }
      }
    }
    cpart[tid] = cp;
  }
  __syncthreads();
  // two y tiles per wave (rows y0 and y0 + 128), sharing every B read
  const int y0 = (yblk * 8 + wid) * 32;
  if (y0 >= Tt) return;
  float colc = 0.f;
#pragma unroll
  for (int q = 0; q < 8; ++q) colc += cpart[q * 32 + l32];
  const int ya = y0 + l32;
  const int yb = ya + 128;
  const bool yva = ya < Tt;
  const bool yvb = yb < Tt;
  const float* zb = z + (int64_t)b * C * Tt;
  const float* za = zb + (yva ? ya : 0);
  const float* zbb = zb + (yvb ? yb : 0);
  f32x16 acc0, acc1;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    acc0[r] = 0.f;
    acc1[r] = 0.f;
  }
  // z of channels 8t .. 8t + 8 for this lane's rows (loaded one step ahead)
  auto zload = [&](int t, float* va, float* vb) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int d = 8 * t + i;  // (t past NS: d >= C, zero)
      va[i] = (yva && d < C) ? za[(int64_t)d * Tt] : 0.f;
      vb[i] = (yvb && d < C) ? zbb[(int64_t)d * Tt] : 0.f;
    }
  };
  auto mma6 = [&](const float* zv, const nc_bf16x8& bh, const nc_bf16x8& bm, const nc_bf16x8& bl,
                  f32x16 c) -> f32x16 {
    nc_f32x8 v;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = lhi ? zv[i] : -0.5f * zv[i] * zv[i];
    nc_bf16x8 ah, am, al;
    nc_split3(v, ah, am, al);
    // small terms first (the conv kernels' order)
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, c, 0, 0, 0);
    return c;
  };
  // z of a group of NC3_PF steps in flight while the other group's MFMAs
  // run (two register groups, ping-pong): at one step of look-ahead the
  // strided z rows left the kernel latency-bound (44 us for the C3 shape)
  constexpr int PF = NC3_PF;
  float zga[PF][8], zgb[PF][8], zha[PF][8], zhb[PF][8];
  auto gload = [&](int t0, float (*va)[8], float (*vb)[8]) {
#pragma unroll
    for (int u = 0; u < PF; ++u) zload(t0 + u, va[u], vb[u]);
  };
  auto gmma = [&](int t0, float (*va)[8], float (*vb)[8]) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int t = t0 + u;
      if (t < NS) {
        const nc_bf16x8* bp = reinterpret_cast<const nc_bf16x8*>(bpl) + (t * 2 + lhi) * 32 + l32;
        const nc_bf16x8 bh = bp[0];
        const nc_bf16x8 bm = bp[PL / 8];
        const nc_bf16x8 bl = bp[PL / 4];
        acc0 = mma6(va[u], bh, bm, bl, acc0);
        acc1 = mma6(vb[u], bh, bm, bl, acc1);
      }
    }
  };
  gload(0, zga, zgb);
  for (int t0 = 0; t0 < NS; t0 += 2 * PF) {
    if (t0 + PF < NS) gload(t0 + PF, zha, zhb);
    gmma(t0, zga, zgb);
    if (t0 + PF >= NS) break;
    if (t0 + 2 * PF < NS) gload(t0 + 2 * PF, zga, zgb);
    gmma(t0 + PF, zha, zhb);
  }
  const int x = x0 + l32;
  if (x >= Ts) return;
  float* ob = out + (int64_t)b * Tt * Ts;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = y0 + (r & 3) + 8 * (r >> 2) + 4 * lhi;
    if (row < Tt) ob[(int64_t)row * Ts + x] = acc0[r] + colc;
    if (row + 128 < Tt) ob[(int64_t)(row + 128) * Ts + x] = acc1[r] + colc;
  }
}

}  // namespace

extern "C" int vits_neg_cent(const float* z_p, const float* m_p, const float* logs_p,
                             float* neg_cent, int batch, int channels, int t_t, int t_s,
                             void* stream) {
  VITS_CHECK_ARG(z_p && m_p && logs_p && neg_cent);
  VITS_CHECK_ARG(batch > 0 && channels > 0 && t_t > 0 && t_s > 0);
  const size_t lds = sizeof(float) * (2 * (size_t)channels * 32 + 256);
  if (nc3_lds_bytes(channels) <= 80 * 1024) {  // (two workgroups per CU)
    // one 1-D grid; the kernel decodes (column tile, row block, utterance)
    const int nx = (t_s + 31) / 32, nq = (t_t + 255) / 256 * batch;
    hipLaunchKernelGGL(neg_cent_kernel3, dim3(nx * 8 * ((nq + 7) / 8)), dim3(256),
                       nc3_lds_bytes(channels), as_stream(stream), z_p, m_p, logs_p, neg_cent,
                       channels, t_t, t_s, batch);
  } else if (lds <= 64 * 1024) {
    dim3 grid((t_s + 31) / 32, (t_t + 255) / 256, batch);
    hipLaunchKernelGGL(neg_cent_kernel2, grid, dim3(256), lds, as_stream(stream), z_p, m_p, logs_p,
                       neg_cent, channels, t_t, t_s);
  } else {  // very wide channel counts: the LDS-free v1
    dim3 grid((t_s + 31) / 32, (t_t + 31) / 32, batch);
    hipLaunchKernelGGL(neg_cent_kernel, grid, dim3(64), 0, as_stream(stream), z_p, m_p, logs_p,
                       neg_cent, channels, t_t, t_s);
  }
  return vits_launch_status();
}
