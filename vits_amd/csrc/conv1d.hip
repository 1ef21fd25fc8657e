// conv1d.hip — implicit-GEMM dilated 1-D convolution on gfx950 fp32 MFMA
// (v_mfma_f32_32x32x2_f32), with the elementwise tails of the VITS blocks
// fused into the prologue/epilogue.
//
// GEMM view (one utterance b):
//   Y[m][n] = sum_{c<cin, j<k} W[m][c][j] * X[c][n - pad_left + j*dil]
// rows m = output channels (gate pairs interleaved / polyphase phases
// stacked, see vits_amd/engine.py), columns n = time positions.
//
// Layout in HBM: activations stay [B][C][T] (time contiguous, as the
// reference keeps them), packed weights are [cin_pad][k][m_pad] so a
// K-chunk of `kc` input channels is one contiguous slab whose rows the
// workgroup streams with 16-byte loads.
//
// One workgroup = 4 waves = one BM x BN output tile of one utterance.  Per
// K-chunk the workgroup stages W[kc][k][BM] and the input window
// X[kc][BN + (k-1)*dil] (leaky-relu prologue applied on the way in) into
// LDS once; every tap j then reads the same X rows shifted by j*dil, so the
// input is fetched once per chunk regardless of the kernel width.
//
// vits_conv1d_forward_groups runs independent convs of one kind (the three
// ResBlock2 branches of a Generator stage) as one grid: blockIdx.z selects
// the member descriptor and the utterance.
//
// Reference call sites: modules.py:136,148 (WN in/res_skip convs),
// modules.py:252,257 (ResBlock2 convs1/convs2), models.py:307,310
// (conv_pre, ups), modules.py:363,366 (coupling pre/post).
#include <cstdlib>

#include "conv1d_impl.h"

namespace {

int check_desc(const vits_conv1d_desc& d, int batch) {
  VITS_CHECK_ARG(d.x && d.w && d.out0.y);
  VITS_CHECK_ARG(batch > 0 && d.cin > 0 && d.m > 0 && d.k > 0 && d.dil > 0 && d.n_out > 0);
  VITS_CHECK_SHAPE(d.kc >= 2 && (d.kc % 2) == 0 && d.cin_pad % d.kc == 0 && d.cin_pad >= d.cin);
  VITS_CHECK_SHAPE(d.m_pad % 128 == 0 && d.m_pad >= d.m);
  VITS_CHECK_SHAPE(d.tin >= 0 && d.x_tstride >= 1);
  VITS_CHECK_SHAPE(d.x_tstride != 1 || d.x_cstride >= d.tin);
  if (d.epi == VITS_EPI_GATE) VITS_CHECK_SHAPE((d.m % 2) == 0);
  // (the epilogue's fp32 row / u is exact for rows < 2^14, u <= 64)
  if (d.epi == VITS_EPI_UPSAMPLE)
    VITS_CHECK_SHAPE(d.up_u > 0 && d.up_u <= 64 && d.m < (1 << 14) && d.m % d.up_u == 0 &&
                     d.t_out > 0);
  if (d.epi == VITS_EPI_STORE && d.split < d.m) VITS_CHECK_ARG(d.out1.y != nullptr);
  if ((reinterpret_cast<uintptr_t>(d.w) & 15) != 0) return VITS_E_SHAPE;
  VITS_CHECK_ARG(d.wdtype == VITS_WDT_F32 || d.wdtype == VITS_WDT_BF16 ||
                 d.wdtype == VITS_WDT_F16 || d.wdtype == VITS_WDT_F32S ||
                 d.wdtype == VITS_WDT_F32P);
  if (d.wdtype == VITS_WDT_F32P) VITS_CHECK_SHAPE(d.kc == 16 || d.kc == 32);
  if (d.wdtype != VITS_WDT_F32) VITS_CHECK_SHAPE((d.kc % 16) == 0);
  if (d.gmask) VITS_CHECK_ARG(d.epi == VITS_EPI_STORE && d.split >= d.m);
  if (d.io16) VITS_CHECK_ARG(d.wdtype == VITS_WDT_BF16 || d.wdtype == VITS_WDT_F16);
  // row-joined 2-D layers: 4-column blocks within one row, single-output
  // STORE, K-chunks inside one frequency tap
  return VITS_OK;
}

// 16-bit operand types read their weight fragments from global memory
// (conv1d_impl.h GA) for fp32-activation (inference) groups with a >= 5-tap
// member; tools/conv_bench.py BF=1 on MI355X (B=16, Ty=500): k = 7 / 11
// +3..20 %, k = 3 -3..-15 % and the 2-tap upsampler -11 % against the
// LDS-staged weights, and the fp16-I/O training convs (kc up to 64, io16 = 1)
// lose ~3 % of the train step; the 16-bit-activation inference decoder
// (io16 = 2) takes it for every group (C5, B=4 Ty=2500 bf16: conv time 12.9
// -> 12.2 ms/step, its k=3 and 2-tap upsampler groups included).
bool ga16(const vits_conv1d_desc* d, int n) {
  int kmax = 0;
  for (int i = 0; i < n; ++i) {
    if (d[i].io16 == 1) return false;
    if (d[i].io16 == 2) return true;
    kmax = d[i].k > kmax ? d[i].k : kmax;
  }
  return kmax >= 5;
}

int conv1d_group(const vits_conv1d_desc* d, int n, int batch, hipStream_t s) {
  vits_conv::ConvGroup g;
  g.n = n;
  g.batch = batch;
  for (int i = 0; i < n; ++i) {
    int rc = check_desc(d[i], batch);
    if (rc) return rc;
    g.d[i] = d[i];
  }
  int rc, which;
  switch (d[0].wdtype) {
    case VITS_WDT_BF16:
      rc = ga16(d, n) ? vits_conv1d_dispatch_bf16g(g, s) : vits_conv1d_dispatch_bf16(g, s);
      which = VITS_CNT_CONV_16;
      break;
    case VITS_WDT_F16:
      rc = ga16(d, n) ? vits_conv1d_dispatch_f16g(g, s) : vits_conv1d_dispatch_f16(g, s);
      which = VITS_CNT_CONV_16;
      break;
    case VITS_WDT_F32S:
      rc = vits_conv1d_dispatch_f32s(g, s);
      which = VITS_CNT_CONV_SPLIT;
      break;
    case VITS_WDT_F32P:
      rc = vits_conv1d_dispatch_f32p(g, s);
      which = VITS_CNT_CONV_SPLIT;
      break;
    default:
      rc = vits_conv1d_dispatch_f32(g, s);
      which = VITS_CNT_CONV_F32;
  }
  if (rc == VITS_OK) vits_count(which);
  return rc;
}

// a group that cannot share one grid (different tiles / epilogues / staging
// kinds) runs as separate launches, in order
int conv1d_group_or_seq(const vits_conv1d_desc* d, int n, int batch, hipStream_t s) {
  if (n > 1 && n <= vits_conv::VITS_CONV_GROUP) {
    int rc = conv1d_group(d, n, batch, s);
    if (rc != VITS_E_UNSUP) return rc;
  }
  for (int i = 0; i < n; ++i) {
    int rc = conv1d_group(d + i, 1, batch, s);
    if (rc) return rc;
  }
  return VITS_OK;
}

}  // namespace

extern "C" int vits_conv1d_forward(const vits_conv1d_desc* d, int batch, void* stream) {
  if (!d) return VITS_E_ARG;
  return conv1d_group(d, 1, batch, as_stream(stream));
}

extern "C" int vits_conv1d_forward_seq(const vits_conv1d_desc* d, int n, int batch, void* stream) {
  if (!d || n < 0) return VITS_E_ARG;
  for (int i = 0; i < n; ++i) {
    int rc = conv1d_group(d + i, 1, batch, as_stream(stream));
    if (rc) return rc;
  }
  return VITS_OK;
}

extern "C" int vits_conv1d_forward_groups(const vits_conv1d_desc* d, const int32_t* sizes,
                                          int ngroups, int batch, void* stream) {
  if (!d || !sizes || ngroups < 0) return VITS_E_ARG;
  int off = 0;
  for (int i = 0; i < ngroups; ++i) {
    VITS_CHECK_ARG(sizes[i] >= 1);
    int rc = conv1d_group_or_seq(d + off, sizes[i], batch, as_stream(stream));
    if (rc) return rc;
    off += sizes[i];
  }
  return VITS_OK;
}
