/*
 * vits_amd.h — C-ABI of the MI355X (gfx950) VITS hot path.
 *
 * Every entry point takes plain device pointers, sizes and a hipStream_t
 * passed as `void*` (NULL = default stream).  No torch types cross this
 * boundary; ownership of every buffer stays with the caller (the PyTorch
 * caching allocator on the Python side).  All calls are asynchronous on the
 * given stream, never synchronise the host, and return 0 on success or a
 * negative VITS_E* code on a shape/argument error (checked on the host
 * before anything is launched) or a hipError_t (positive) from the launch.
 *
 * Reference interfaces replaced (paths relative to emotional-vits/):
 *   vits_maximum_path        monotonic_align.maximum_path, call site
 *                            models.py:498 (external Cython package
 *                            `monotonic-align`, not vendored)
 *   vits_neg_cent            the alignment scores of SynthesizerTrn.forward
 *                            (models.py:483-490: exp, 2 matmuls, 2 sums)
 *   vits_conv1d_forward      nn.Conv1d / ConvTranspose1d forward of
 *                            modules.WN (modules.py:130-182),
 *                            modules.ResBlock2 (modules.py:250-260),
 *                            models.Generator (models.py:306-318),
 *                            ResidualCouplingLayer.infer (modules.py:362-375)
 *                            with their elementwise tails fused in
 *   vits_linear_forward      per-utterance nn.Linear conditioning of
 *                            WN.cond_layer (modules.py:109-110,139),
 *                            ResBlock2.conds (modules.py:243-245,253),
 *                            FFN2.cond (attentions.py:143,152)
 *   vits_expand_prior        the prior-expansion matmuls + noise of
 *                            SynthesizerTrn.infer_p2 (models.py:569-571)
 *   vits_conv_post_tanh      Generator tail: leaky_relu(0.01) -> conv_post
 *                            -> tanh (models.py:315-317)
 *   vits_stft_mag_forward /  TorchSTFT.stft + STFTLoss.spec2mag
 *   vits_stft_mag_backward   (modules.py:386-392, stft_loss.py:22-23);
 *   (_multi)                 all resolutions of MultiResolutionSTFTLoss
 *                            (stft_loss.py:47-95) in one launch
 *   vits_layer_norm_channels modules.LayerNorm (modules.py:41-44)
 *   vits_attention_forward   MultiHeadAttention.attention core
 *                            (attentions.py:85-100)
 */
#ifndef VITS_AMD_H
#define VITS_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VITS_OK 0
#define VITS_E_ARG (-1)     /* bad pointer / non-positive size */
#define VITS_E_SHAPE (-2)   /* inconsistent shapes / strides */
#define VITS_E_UNSUP (-3)   /* configuration outside the compiled kernels */

/* ---------------------------------------------------------------------- */
/* conv1d: implicit-GEMM dilated 1-D convolution on fp32 MFMA             */
/* ---------------------------------------------------------------------- */

/* epilogue kinds */
#define VITS_EPI_STORE 0     /* y = act(acc + bias + cond) [+res] [accumulate] */
#define VITS_EPI_GATE 1      /* y[p] = tanh(v[2p]) * sigmoid(v[2p+1])           */
                             /* (+ out1.y set: the pre-activation acc + bias,   */
                             /* no cond, to out1 channels p and m/2 + p - the   */
                             /* training gate's saved input)                    */
#define VITS_EPI_UPSAMPLE 2  /* polyphase ConvTranspose1d output scatter        */

/* activations applied to v before residual/accumulate (STORE epilogue) */
#define VITS_ACT_NONE 0
#define VITS_ACT_RELU 1
#define VITS_ACT_TANH 2
#define VITS_ACT_EXP 3

/* tile configurations (rows x cols of one workgroup) */
#define VITS_TILE_128x128 0
#define VITS_TILE_64x256 1
#define VITS_TILE_32x256 2
#define VITS_TILE_64x128 3  /* chosen by the library for small grids of 128x128 layers */

typedef struct vits_conv_out {
  float* y;               /* output [B][*][y_cstride]                        */
  int64_t y_bstride;      /* elements between utterances                     */
  int32_t y_cstride;      /* elements between channels                       */
  int32_t act;            /* VITS_ACT_*                                      */
  const float* res;       /* optional residual (may alias y)                 */
  int64_t res_bstride;
  int32_t res_cstride;
  float res_scale;        /* y = res + res_scale * v                         */
  int32_t accumulate;     /* y = y_old + (...)                               */
  float post_div;         /* y /= post_div when != 1                         */
} vits_conv_out;

typedef struct vits_conv1d_desc {
  /* input x: element (b, c, t) at b*x_bstride + c*x_cstride + t*x_tstride   */
  /* ([B][C][T] activations: x_tstride = 1; time-major [B][T][C]: x_cstride */
  /* = 1, x_tstride = C, used for the text-embedding Linear)                */
  const float* x;
  int64_t x_bstride;
  int32_t x_cstride;
  int32_t x_tstride;
  int32_t cin;
  int32_t tin;            /* valid input positions; outside reads as 0        */
  float in_slope;         /* prologue leaky-relu slope on x; 1.0 = identity   */
  /* packed weights: [cin_pad][k][m_pad] fp32, see vits_amd/engine.py       */
  const float* w;
  int32_t m;              /* GEMM rows actually produced                      */
  int32_t m_pad;          /* row stride of the packed weights                 */
  int32_t cin_pad;        /* multiple of kc                                    */
  int32_t kc;             /* input channels staged per K-chunk (even)         */
  int32_t k;              /* taps                                             */
  int32_t dil;            /* tap dilation                                      */
  int32_t pad_left;       /* input position of column n, tap j: n-pad+j*dil   */
  int32_t n_out;          /* GEMM columns (output positions)                  */
  int32_t tile;           /* VITS_TILE_*                                      */
  /* epilogue */
  int32_t epi;            /* VITS_EPI_*                                       */
  const float* bias;      /* logical-order bias or NULL                       */
  const float* cond;      /* [B][cond_bstride] logical-order add, or NULL     */
  int64_t cond_bstride;
  int32_t split;          /* STORE: rows [0,split)->out0, [split,m)->out1     */
  int32_t up_u;           /* UPSAMPLE: stride u                               */
  int32_t up_pad;         /* UPSAMPLE: ConvTranspose padding                  */
  int32_t t_out;          /* UPSAMPLE: output length                          */
  const int32_t* lengths; /* [B]: zero output columns t >= lengths[b]; NULL   */
  vits_conv_out out0;
  vits_conv_out out1;
  /* weight / MFMA type: VITS_WDT_F32 (w as above, exact-f32 MFMA) or      */
  /* VITS_WDT_BF16 / VITS_WDT_F16 (w = 16-bit [cin_pad/kc][k][kc/8][m_pad]  */
  /* [8], kc % 16 == 0; activations stay fp32 in HBM and are rounded to the */
  /* 16-bit type when staged; fp32 accumulation:                           */
  /* v_mfma_f32_32x32x16_bf16 / _f16), or VITS_WDT_F32S (w = the fp32     */
  /* [cin_pad/16][k][2][m_pad][8] slab image, kc % 16 == 0: fp32 operands  */
  /* split exactly into three bf16 terms in registers, six bf16 MFMAs per  */
  /* 16-deep k-step (hi*hi, hi*mid, mid*hi, mid*mid, hi*lo, lo*hi), fp32   */
  /* accumulation; error vs fp64 at the exact-fp32 kernel's level)         */
  int32_t wdtype;
  /* single-output STORE only (the input gradient of a conv whose forward   */
  /* fused a leaky-relu prologue): v *= gmask[b][row][n] > 0 ? 1 : slope    */
  /* before residual / accumulate; gmask = the forward's input, NULL = off  */
  const float* gmask;
  int64_t gmask_bstride;
  int32_t gmask_cstride;
  float gmask_slope;
  /* io16 != 0 (16-bit wdtype only): x, out0/out1 y and res, and gmask are  */
  /* tensors of the 16-bit operand type (strides in elements); fp32 I/O    */
  /* otherwise.  The fp16-autocast training convs keep fp16 activations   */
  /* (io16 = 1); io16 = 2 marks the 16-bit inference decoder, whose groups */
  /* with a >= 5-tap member read weight fragments from global memory.    */
  int32_t io16;
  /* with lengths: > 0 = workgroups whose first output position is at or    */
  /* past lengths[b] + len_skip exit without computing or writing (the      */
  /* bucketed whole-utterance infer: work follows the utterance, not the     */
  /* bucket; consumers never read past lengths[b] + halo, halo < len_skip,  */
  /* and [lengths[b], lengths[b] + len_skip) is written as zeros); 0 = off  */
  int32_t len_skip;
} vits_conv1d_desc;

#define VITS_WDT_F32 0
#define VITS_WDT_BF16 1
#define VITS_WDT_F16 2
#define VITS_WDT_F32S 3
/* VITS_WDT_F32P: the F32S arithmetic with w = the host-split bf16 planes   */
/* [cin_pad/16][k][2][3][m_pad][8] (plane 0 = hi, 1 = mid, 2 = lo of each   */
/* fp32 weight, x == hi + mid + lo exactly), kc 16 or 32; A fragments are  */
/* read from global memory, so only the input window is staged in LDS.     */
#define VITS_WDT_F32P 4

int vits_conv1d_forward(const vits_conv1d_desc* d, int batch, void* stream);

/* Run `n` conv descriptors back to back on one stream (one host call). */
int vits_conv1d_forward_seq(const vits_conv1d_desc* d, int n, int batch, void* stream);

/* Run `ngroups` groups of consecutive descriptors (sizes[i] each, <= 3):  */
/* the members of a group are independent convs (no member reads another's */
/* output; the three ResBlock2 branches of one Generator stage,            */
/* models.py:311-313 / modules.py:250-260) and share ONE launch when they  */
/* have the same tile, epilogue and staging kind, else run in order.       */
/* Groups run in order.                                                    */
int vits_conv1d_forward_groups(const vits_conv1d_desc* d, const int32_t* sizes, int ngroups,
                               int batch, void* stream);

/* ---------------------------------------------------------------------- */
/* per-utterance conditioning GEMV: y[b][n] = W[n][:] . g[b][:] + bias[n] */
/* ---------------------------------------------------------------------- */
int vits_linear_forward(const float* g, int64_t g_bstride, const float* w, const float* bias,
                        float* y, int64_t y_bstride, int batch, int n_out, int n_in,
                        void* stream);

/* ---------------------------------------------------------------------- */
/* prior expansion: z[b][c][t] = sum_x attn[b][t][x] m[b][c][x]           */
/*                    + noise[b][c][t] * sum_x attn[b][t][x] s[b][c][x]   */
/* ---------------------------------------------------------------------- */
int vits_expand_prior(const float* attn, const float* m, const float* s, const float* noise,
                      float* z, int batch, int channels, int t_y, int t_x, int exp_s,
                      float noise_scale, void* stream);
/* exp_s = 0: z = A.m + noise * (A.s)                 (infer_p2, models.py:569-571) */
/* exp_s = 1: z = A.m + noise * exp(A.s) * noise_scale  (inference, models.py:529-532) */

/* ---------------------------------------------------------------------- */
/* Generator tail: y[b][t] = tanh(sum_{c,j} w[c][j] lrelu(x[b][c][t-3+j], 0.01)) */
/* w: [channels][7] (conv_post, no bias)                                  */
/* ---------------------------------------------------------------------- */
/* ---------------------------------------------------------------------- */
/* durations -> lengths + expanded prior, on the device (replaces the       */
/* w = exp(logw)*rate -> ceil -> y_len .item() -> infer_path -> attn @ m /  */
/* attn @ s -> z_p sequence of models.py:544-553, infer.py:169-176 and     */
/* commons.py:143-155 without a host sync, over a static bucket t_y):       */
/*   w_ceil[x] = ceil(exp(logw[b][x]) * rate) (x < x_len[b], else 0;        */
/*   half_round: fp16 roundings of the half model), y_len = max(sum, 1),   */
/*   z[b][c][t] = m[b][c][x(t)] + noise(c,t) * s[b][c][x(t)] * noise_scale  */
/*   for t < y_len (x(t): cum[x-1] <= t < cum[x]), 0 for y_len <= t < t_y;  */
/*   lens[i][b] = y_len * stage_mult[i].  noise_mode 0: noise [B][C][t_y];  */
/*   1: element (c, t) at noise[s + c*y_len + t] (EmoVITS's buffer slice,   */
/*   infer.py:172-175), s = np.random.randint(noise_len - C*y_len) drawn on */
/*   the device exactly as numpy's legacy RandomState does (masked         */
/*   rejection) from noise_start = [B][VITS_ED_DRAWS] raw MT19937 uint32    */
/*   words; lens must then have n_stage + 1 rows: lens[n_stage][b] = words  */
/*   consumed (the host re-advances its generator by that many), -1 when   */
/*   the slice does not fit (the reference's randint raises), -2 when all  */
/*   VITS_ED_DRAWS words were rejected (the host advances by the pool and  */
/*   calls again with the next words); z = 0 and no noise read for both.  */
/*   t_x <= 4096, n_stage <= 8.                                             */
#define VITS_ED_DRAWS 32
/* ---------------------------------------------------------------------- */
int vits_expand_durations(const float* logw, int64_t logw_bstride, const int32_t* x_len, int t_x,
                          float rate, int half_round, const float* m, const float* s,
                          int64_t ms_bstride, int32_t ms_cstride, const float* noise,
                          int noise_mode, const int32_t* noise_start, int64_t noise_len,
                          float noise_scale, float* z,
                          int batch, int channels, int t_y, int32_t* lens,
                          const int32_t* stage_mult, int n_stage, void* stream);

int vits_conv_post_tanh(const float* x, int64_t x_bstride, int32_t x_cstride, const float* w,
                        float* y, int batch, int channels, int t_len, int ksize, void* stream);
/* Same on a 16-bit last-stage activation (xdtype VITS_WDT_BF16 / _F16; the
 * 16-bit model's decoder with 16-bit activations, as the reference's .half()
 * model holds them); VITS_WDT_F32 = vits_conv_post_tanh. */
int vits_conv_post_tanh_lowp(const void* x, int64_t x_bstride, int32_t x_cstride, const float* w,
                             float* y, int batch, int channels, int t_len, int ksize, int xdtype,
                             void* stream);

/* ---------------------------------------------------------------------- */
/* Monotonic alignment search (VITS DP + backtrack), bit-exact vs the     */
/* Cython core.  neg_cent [B][t_t][t_s] fp32 (the reference casts to fp32 */
/* before the DP); mask [B][t_t][t_s] of mask_dtype: lengths are taken as */
/* t_t[b] = sum_y mask[b][y][0], t_s[b] = sum_x mask[b][0][x] exactly as  */
/* monotonic_align/__init__.py does.  path [B][t_t][t_s] of path_dtype is */
/* written in full (1 on the path, 0 elsewhere).                          */
/* dtype codes: VITS_DT_*.                                                */
/* ---------------------------------------------------------------------- */
#define VITS_DT_F32 0
#define VITS_DT_F16 1
#define VITS_DT_BF16 2
#define VITS_DT_I32 3
int vits_maximum_path(const float* neg_cent, const void* mask, int mask_dtype, void* path,
                      int path_dtype, int batch, int t_t, int t_s, void* workspace,
                      int64_t workspace_bytes, void* stream);
/* same, with explicit per-utterance lengths (int32 [B] each, on device) */
int vits_maximum_path_lengths(const float* neg_cent, const int32_t* t_t_len,
                              const int32_t* t_s_len, void* path, int path_dtype, int batch,
                              int t_t, int t_s, void* workspace, int64_t workspace_bytes,
                              void* stream);
/* bytes of workspace the two calls above need (0 when the backtrack bits */
/* fit in LDS)                                                            */
int64_t vits_maximum_path_workspace(int batch, int t_t, int t_s);

/* ---------------------------------------------------------------------- */
/* MAS scores (models.py:483-490): neg_cent[b][y][x] = sum_d(-0.5 log 2pi */
/* - logs_p - 0.5 z_p^2 s + z_p m_p s - 0.5 m_p^2 s), s = exp(-2 logs_p). */
/* z_p [B][C][t_t], m_p / logs_p [B][C][t_s], neg_cent [B][t_t][t_s], all */
/* contiguous fp32.  Computed in fp32 over every (padded) position, as    */
/* the reference does before its mask.                                    */
/* ---------------------------------------------------------------------- */
int vits_neg_cent(const float* z_p, const float* m_p, const float* logs_p, float* neg_cent,
                  int batch, int channels, int t_t, int t_s, void* stream);

/* ---------------------------------------------------------------------- */
/* STFT magnitude and its adjoint.  x [B][L] fp32; the signal is reflect- */
/* padded by `pad` samples on both sides (pad = n_fft/2 reproduces        */
/* torch.stft(center=True, pad_mode='reflect'); mel_processing pads       */
/* (n_fft-hop)/2 itself and calls center=False), then framed with `hop`,  */
/* windowed by `window` (length win, centred in n_fft as torch.stft does) */
/* and transformed: frames = (L + 2 pad - n_fft)/hop + 1.                 */
/* mag [B][n_fft/2+1][frames] = sqrt(re^2 + im^2 + eps); re/im (optional, */
/* needed by the backward) same layout.                                   */
/* ---------------------------------------------------------------------- */
int vits_stft_mag_forward(const float* x, int batch, int length, const float* window,
                          int n_fft, int hop, int win, int pad, float eps, float* mag,
                          float* re, float* im, void* stream);
/* grad_x [B][L] = d(sum grad_mag * mag)/dx.  workspace: frames*n_fft*B   */
/* floats (vits_stft_workspace).                                          */
int vits_stft_mag_backward(const float* grad_mag, const float* mag, const float* re,
                           const float* im, const float* window, int batch, int length,
                           int n_fft, int hop, int win, int pad, float* grad_x,
                           float* workspace, int64_t workspace_floats, void* stream);
int64_t vits_stft_workspace(int batch, int length, int n_fft, int hop, int pad);

/* Several transforms in one launch (the 2 signals x 5 resolutions of the */
/* MR-STFT loss, stft_loss.py:47-95): up to 16 jobs, each with its own    */
/* signal batch, resolution and outputs.  Forward uses x, window, sizes,  */
/* eps, mag, re, im; backward uses grad_mag, mag, re, im, window, sizes,  */
/* grad_x and a workspace of vits_stft_workspace_multi floats.  layout 1: */
/* mag / re / im / grad_mag are [B][frames][n_fft/2+1] (frame-major: a    */
/* workgroup's frames are one contiguous run - coalesced stores); 0: the  */
/* torch.stft layout [B][n_fft/2+1][frames].                              */
typedef struct vits_stft_job {
  const float* x;
  const float* window;
  const float* grad_mag;
  float* mag;
  float* re;
  float* im;
  float* grad_x;
  int32_t batch;
  int32_t length;
  int32_t n_fft;
  int32_t hop;
  int32_t win;
  int32_t pad;
  float eps;
  int32_t layout;
} vits_stft_job;
int vits_stft_mag_forward_multi(const vits_stft_job* jobs, int njobs, void* stream);
int vits_stft_mag_backward_multi(const vits_stft_job* jobs, int njobs, float* workspace,
                                 int64_t workspace_floats, void* stream);
int64_t vits_stft_workspace_multi(const vits_stft_job* jobs, int njobs);

/* ---------------------------------------------------------------------- */
/* channel LayerNorm over dim 1 of [B][C][T]:                             */
/*   v = LN(x + r) * gamma + beta                (r, gamma, beta optional) */
/*   v = (v + post_add[b][c]) * scale + pos[t][c] * (*pos_alpha)           */
/*   y = (t < lengths[b]) ? v : 0                (lengths optional)        */
/* post_add / pos / pos_alpha optional (NULL); pos is [T][C] (sin table);  */
/* pos_alpha is a device scalar (the learnable TextEncoder.alpha).        */
/* ---------------------------------------------------------------------- */
int vits_layer_norm_channels(const float* x, const float* r, const float* gamma,
                             const float* beta, float* y, int batch, int channels, int t_len,
                             float eps, const int32_t* lengths, const float* post_add,
                             int64_t post_add_bstride, float scale, const float* pos,
                             const float* pos_alpha, void* stream);

/* ---------------------------------------------------------------------- */
/* scaled-dot-product attention over [B][H*D][T] channel-major q/k/v      */
/* (batch stride qkv_bstride, e.g. slices of one fused q|k|v buffer), key */
/* mask from lengths (fill -1e4), out [B][H*D][T] with out_bstride;        */
/* head_dim in {16, 32, 48, 64, 96, 128}, else VITS_E_UNSUP              */
/* ---------------------------------------------------------------------- */
int vits_attention_forward(const float* q, const float* k, const float* v, float* out,
                           int batch, int heads, int head_dim, int t_len,
                           int64_t qkv_bstride, int64_t out_bstride, const int32_t* lengths,
                           void* stream);

/* ---------------------------------------------------------------------- */
/* Training-step convs (backward of every stride-1 nn.Conv1d the          */
/* train_stft.py step runs under fp16 autocast, train_stft.py:165-236:    */
/* WN modules.py:130-182, ResBlock2 modules.py:250-260, couplings         */
/* modules.py:357-375, PosteriorEncoder models.py:268-279, Generator      */
/* models.py:306-318, WaveDiscriminator mrd.py:15-55).  The forward and   */
/* the input gradient run through vits_conv1d_forward on a 16-bit image   */
/* of the weight; the weight gradient has its own kernel.                 */
/* ---------------------------------------------------------------------- */
/* fp32 W [cout][cin][k] -> 16-bit image [cin_pad/16][k][2][m_pad][8] of   */
/* wdtype (VITS_WDT_F16 / _BF16).  transpose = 0: rows = co, channels =   */
/* ci (forward).  transpose = 1: rows = ci, channels = co, taps reversed  */
/* (input gradient: dX = conv(dY, W', pad_left = (k-1)*dil - pad)).       */
/* zero / zero_n: optional fp32 buffer the same launch clears (the weight- */
/* gradient accumulator of the backward that follows; NULL / 0 = none).   */
int vits_conv1d_pack16(const float* w, int cout, int cin, int k, int transpose, void* out,
                       int m_pad, int cin_pad, int wdtype, float* zero, int64_t zero_n,
                       void* stream);
/* Both images in one launch: `out` as transpose = 0 ([cin_pad/16][k][2]   */
/* [m_pad][8], rows cout) and `out_t` as transpose = 1 (rows cin, channels  */
/* cout) -- the training forward packs its backward's image with it.       */
int vits_conv1d_pack16_pair(const float* w, int cout, int cin, int k, void* out, int m_pad,
                            int cin_pad, void* out_t, int m_pad_t, int cin_pad_t, int wdtype,
                            void* stream);
/* Both images of many layers in few launches (48 layers per launch): the  */
/* training step packs every HIP conv of a network once per forward, right  */
/* after the weight / spectral norm launch that produced the weights,       */
/* instead of one vits_conv1d_pack16_pair launch per conv call.             */
typedef struct vits_pack16_layer {
  const float* w;   /* fp32 [cout][cin][k] */
  int32_t cout, cin, k;
  void* img;        /* [cin_pad/16][k][2][m_pad][8], rows cout */
  int32_t m_pad, cin_pad;
  void* img_t;      /* [cin_pad_t/16][k][2][m_pad_t][8], rows cin, taps reversed */
  int32_t m_pad_t, cin_pad_t;
  int32_t gate;     /* 1: img rows gate-interleaved (row 2q = output q, row 2q+1 = */
                    /* output cout/2 + q: VITS_EPI_GATE); img_t stays natural      */
} vits_pack16_layer;
int vits_conv1d_pack16_pairs(const vits_pack16_layer* layers, int n, int wdtype, void* stream);

typedef struct vits_conv1d_wgrad_desc {
  const float* dy;        /* output gradient [B][cout][n_out], t contiguous  */
  int64_t dy_bstride;
  int32_t dy_cstride;
  int32_t cout;
  const float* x;         /* forward input [B][cin][tin], t contiguous       */
  int64_t x_bstride;
  int32_t x_cstride;
  int32_t cin;
  int32_t tin;
  int32_t n_out;
  int32_t k;
  int32_t dil;
  int32_t pad_left;       /* forward: output t reads x[t - pad_left + j*dil] */
  float in_slope;         /* forward's leaky-relu prologue slope (1 = none)  */
  float* dw_t;            /* += dW as [k][cout][cin] fp32 (caller zeroes)    */
  float* dbias;           /* += sum_{b,t} dY [cout] fp32, or NULL            */
  int32_t wdtype;         /* MFMA operand type: VITS_WDT_F16 / VITS_WDT_BF16, */
                          /* or VITS_WDT_F32 (fp32 dy / x, exact-fp32 MFMA,  */
                          /* split mode only; the fp32 training step)        */
  int32_t reserved;       /* > 0: (b, t)-chunks of 64 steps per workgroup    */
                          /* (tuning override), 0 = automatic                */
  int32_t io16;           /* dy / x are tensors of the 16-bit operand type   */
                          /* (strides in elements)                           */
  int32_t reserved2;
} vits_conv1d_wgrad_desc;
/* dW[co][ci][j] = sum_{b,t} dY[b][co][t] * act(x[b][ci][t - pad_left + j*dil]) */
/* (operands rounded to wdtype, fp32 accumulation; VITS_E_UNSUP when       */
/* 64 + (k-1)*dil > 128 or k not in {1,2,3,4,5,7,9,11})                  */
int vits_conv1d_wgrad(const vits_conv1d_wgrad_desc* d, int batch, void* stream);
/* Same weight gradient without atomics (deterministic): every (b, t)-split */
/* workgroup stores its partial tile into `workspace`, a second launch sums */
/* the splits and WRITES d->dw_t in the parameter layout [cout][cin][k]    */
/* and d->dbias [cout] (no zeroing needed).  workspace_floats >=           */
/* vits_conv1d_wgrad_workspace(d, batch).  Replaces the weight-gradient    */
/* half of torch's conv backward under autocast (train_stft.py:206,232).   */
int64_t vits_conv1d_wgrad_workspace(const vits_conv1d_wgrad_desc* d, int batch);
int vits_conv1d_wgrad_split(const vits_conv1d_wgrad_desc* d, int batch, float* workspace,
                            int64_t workspace_floats, void* stream);

/* WaveNet gate of WN (modules.py:139-146) / ResBlock2 (modules.py:253-255) */
/* in training: y[b][p][t] = tanh(x[b][p][t] + g[b][p]) *                 */
/*                           sigmoid(x[b][H+p][t] + g[b][H+p]),  p < H     */
/* g optional ([B][>= 2H] with g_bstride).  Backward: dx [B][2H][T] and   */
/* (optional) dg[b][c] = sum_t dx[b][c][t] as a dense [B][2H].            */
int vits_gate_forward(const float* x, int64_t x_bstride, int32_t x_cstride, const float* g,
                      int64_t g_bstride, float* y, int64_t y_bstride, int32_t y_cstride,
                      int batch, int half_channels, int t_len, void* stream);
int vits_gate_backward(const float* dy, int64_t dy_bstride, int32_t dy_cstride, const float* x,
                       int64_t x_bstride, int32_t x_cstride, const float* g, int64_t g_bstride,
                       float* dx, int64_t dx_bstride, int32_t dx_cstride, float* dg, int batch,
                       int half_channels, int t_len, void* stream);
/* The same with x / g / y (and dy / x / g / dx) of the 16-bit type wdtype */
/* (VITS_WDT_F16 / _BF16: the fp16 activations of the autocast training    */
/* step), fp32 math, dg fp32.                                              */
int vits_gate_forward_io16(const void* x, int64_t x_bstride, int32_t x_cstride, const void* g,
                           int64_t g_bstride, void* y, int64_t y_bstride, int32_t y_cstride,
                           int batch, int half_channels, int t_len, int wdtype, void* stream);
int vits_gate_backward_io16(const void* dy, int64_t dy_bstride, int32_t dy_cstride, const void* x,
                            int64_t x_bstride, int32_t x_cstride, const void* g,
                            int64_t g_bstride, void* dx, int64_t dx_bstride, int32_t dx_cstride,
                            float* dg, int batch, int half_channels, int t_len, int wdtype,
                            void* stream);

/* Up to 4 independent vits_gate_backward_io16 jobs of one batch and length */
/* as ONE launch (the three ResBlock2 branches of a Generator stage,         */
/* modules.py:253-255 under train_stft.py:165's autocast); dg of job i at    */
/* dg[b * dg_bstride + c] (a column slice of the stage's cond gradient).     */
typedef struct vits_gate_bwd_job {
  const void* dy;
  int64_t dy_bstride;
  int64_t dy_cstride;
  const void* x;
  int64_t x_bstride;
  int64_t x_cstride;
  const void* g;         /* 16-bit cond [B][g_bstride], or NULL */
  int64_t g_bstride;
  void* dx;
  int64_t dx_bstride;
  int64_t dx_cstride;
  float* dg;             /* fp32, or NULL */
  int64_t dg_bstride;
  int32_t half_channels;
  int32_t reserved;
} vits_gate_bwd_job;
int vits_gate_backward_io16_multi(const vits_gate_bwd_job* jobs, int n, int batch, int t_len,
                                  int wdtype, void* stream);

/* ---------------------------------------------------------------------- */
/* One ResBlock2 dilation pair of the Generator as ONE kernel              */
/* (modules.py:250-260, fp32):                                             */
/*   y = x + c2(tanh(a + sa) * sigmoid(b + sb)),  (a|b) = c1(lrelu(x,.1)) */
/* c1 = Conv1d(C, C, k, dil) packed as vits_conv1d_forward's GATE layout  */
/* ([cin_pad1][k][m_pad1], rows (a_p, b_p) interleaved), c2 = Conv1d(C/2, */
/* C, k, dil 1, pad (k-1)/2) packed [cin_pad2][k][m_pad2]; b1 / cond are  */
/* in logical order ([a | b], cond already offset to this pair), b2 [C].  */
/* accumulate: y += result (then / post_div) - the branch mean of a stage.*/
/* x: [B][C][T] fp32, T % 4 == 0, 16-byte aligned; y must not alias x.    */
/* C in {32, 64} (the 64- and 32-channel Generator stages).  Up to 3      */
/* independent pairs (same C) run as one launch.  kc1 / kc2 from          */
/* vits_resblock_pair_kc.                                                 */
/* ---------------------------------------------------------------------- */
typedef struct vits_resblock_pair_desc {
  const float* x;
  int64_t x_bstride;
  int32_t x_cstride;
  int32_t t_len;
  int32_t channels;
  float in_slope;
  const float* w1;
  int32_t m_pad1;
  int32_t cin_pad1;
  int32_t kc1;
  int32_t k;
  int32_t dil;
  int32_t kc2;
  const float* b1;
  const float* cond;
  int64_t cond_bstride;
  const float* w2;
  int32_t m_pad2;
  int32_t cin_pad2;
  const float* b2;
  float* y;
  int64_t y_bstride;
  int32_t y_cstride;
  int32_t accumulate;
  float post_div;
  int32_t len_skip;      /* as vits_conv1d_desc.len_skip                     */
  /* [B] valid lengths or NULL: the gated tensor is zero and the output 0  */
  /* at t >= lengths[b] (the utterance ends there, as the convs' masks)    */
  const int32_t* lengths;
} vits_resblock_pair_desc;
int vits_resblock_pair_forward(const vits_resblock_pair_desc* d, int n, int batch, void* stream);
int vits_resblock_pair_kc(int channels, int k, int dil, int* kc1, int* kc2);
/* The same pair for 16-bit models (csrc/resblock16.hip; modules.py:250-  */
/* 260 of a model.half() / bf16 Generator): wdtype VITS_WDT_BF16 / F16;   */
/* x and y are [B][C][T] tensors of that type (the float pointers of the  */
/* descriptor reinterpreted), w1 / w2 the 16-bit images                   */
/* [cin_pad/16][k][2][m_pad][8] of vits_conv1d_desc (w1's rows gate-      */
/* interleaved); kc1 / kc2 are ignored.  C = 32, 64, 128 or 256 (the    */
/* 256-channel pairs run csrc/resblock_f32p.hip's streamed-K tile in its  */
/* 16-bit mode; not for the _mean variant), odd k, (k - 1) * dil <= 96,  */
/* T % 4 == 0.                                                            */
int vits_resblock_pair16_forward(const vits_resblock_pair_desc* d, int n, int batch, int wdtype,
                                 void* stream);
/* The last pairs of a stage's n branches as ONE launch: d[0].y receives  */
/* (sum_i pair_i(d[i].x)) / n (models.py:311-313's branch mean; each      */
/* workgroup runs every member on its time tile and sums in registers);   */
/* the members share t_len and lengths; accumulate / post_div ignored.    */
int vits_resblock_pair16_mean_forward(const vits_resblock_pair_desc* d, int n, int batch,
                                      int wdtype, void* stream);
/* The same pair for the split-fp32 (VITS_WDT_F32P) 64-, 128- and 256-  */
/* channel stages of an fp32 Generator (csrc/resblock_f32p.hip;           */
/* modules.py:250-260): x / y fp32 [B][C][T], w1 / w2 the pre-split       */
/* images [cin_pad/16][k][2][3][m_pad][8] bf16 of vits_conv1d_desc (w1's  */
/* rows gate-interleaved); kc1 / kc2 ignored.  Bitwise the two-conv path  */
/* (c1 with the gate epilogue, c2 with the residual one).  Odd k,         */
/* (k - 1) * dil <= 96, T % 4 == 0, 16-byte aligned x rows.               */
int vits_resblock_pair_f32p_forward(const vits_resblock_pair_desc* d, int n, int batch,
                                    void* stream);

/* Fused RAdam step (radam.py:35-99, the D optimizer of train_stft.py:97) */
/* over a list of fp32 tensors, one launch per VITS_RADAM_MAX tensors.     */
/* scal: device float[8] state (scal[0] = step count, the rest scratch);  */
/* found_inf: device flag of GradScaler's unscale (NULL = never skip);    */
/* when set, nothing is updated (GradScaler's skip rule, no host sync).   */
/* grad_scale: device scalar the grads are still multiplied by (NULL =    */
/* already unscaled).  lr_dev: optional device double read at run time   */
/* instead of lr (an lr scheduler's in-place update then reaches a        */
/* captured hipGraph, train_stft.py:127-139 ExponentialLR).               */
#define VITS_RADAM_MAX 96
typedef struct vits_radam_tensor {
  float* param;
  const float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  int64_t numel;
} vits_radam_tensor;
int vits_radam_step(const vits_radam_tensor* tensors, int n, float* scal, const float* found_inf,
                    const float* grad_scale, double lr, const double* lr_dev, double beta1,
                    double beta2, double eps, double weight_decay, void* stream);

/* ---------------------------------------------------------------------- */
/* Weight normalisation of many layers in one launch (legacy             */
/* torch.nn.utils.weight_norm, dim 0: the generator's convs, upsamplers   */
/* and conditioning Linears, modules.py:58-109, models.py:233; replaces   */
/* the per-layer torch._weight_norm / its backward of every forward).     */
/* Each layer is [rows][cols] (rows = size of dim 0), fp32, contiguous.  */
/* forward: w = v * (g / ||v_row||), norms[row] written (global row      */
/* index over all layers of the call, in order); backward (same layers,  */
/* same norms): dg = <dw,v>/n, dv = (g/n)(dw - v <dw,v>/n^2).            */
/* ---------------------------------------------------------------------- */
#define VITS_WNORM_MAX 56
typedef struct vits_wnorm_layer {
  const float* v;
  const float* g;
  float* w;        /* forward output */
  const float* dw; /* backward input */
  float* dv;       /* backward outputs */
  float* dg;
  int32_t rows;
  int32_t cols;
} vits_wnorm_layer;
int vits_weight_norm_forward(const vits_wnorm_layer* layers, int n, float* norms, void* stream);
int vits_weight_norm_backward(const vits_wnorm_layer* layers, int n, const float* norms,
                              void* stream);

/* ---------------------------------------------------------------------- */
/* Spectral normalisation of many layers at once (torch.nn.utils.        */
/* spectral_norm, dim 0, one power iteration per training forward, the   */
/* discriminators of mrd.py; replaces the per-layer forward pre-hooks).  */
/* forward (5 launches for all layers): training: v = normalize(W^T u),  */
/* u = normalize(W v), u / v updated in place; sigma = u . (W v);        */
/* w_sn = W / sigma; saved = [sigma, u (rows), v (cols)] of this call.   */
/* backward (2 launches): dw = dw_sn / sigma - (<dw_sn, W> / sigma^2)    */
/* u v^T, with a workspace of vits_spectral_norm_workspace floats.       */
/* emu16 = 1: the hook inside an fp16 autocast region (mv operands and   */
/* result rounded to fp16, as the reference's autocast mv).              */
/* ---------------------------------------------------------------------- */
#define VITS_SNORM_MAX 48
typedef struct vits_snorm_layer {
  const float* w;     /* weight_orig viewed [rows][cols] */
  float* u;           /* [rows] buffer */
  float* v;           /* [cols] buffer */
  float* w_sn;        /* forward output */
  const float* dw_sn; /* backward input */
  float* dw;          /* backward output */
  float* saved;       /* [1 + rows + cols] */
  int32_t rows;
  int32_t cols;
  float eps;
  int32_t cl_channels; /* 0: w_sn / dw_sn fp32 like w; C > 0: fp16 channels-  */
                       /* last [O][kh][kw][C] images of a Conv2d weight       */
                       /* [O][C][kh][kw] (the autocast MIOpen conv's operand) */
} vits_snorm_layer;
int vits_spectral_norm_supported(int rows, int cols);
int vits_spectral_norm_forward(const vits_snorm_layer* layers, int n, int training, int emu16,
                               void* stream);
int64_t vits_spectral_norm_workspace(const vits_snorm_layer* layers, int n);
int vits_spectral_norm_backward(const vits_snorm_layer* layers, int n, int emu16,
                                float* workspace, int64_t ws_floats, void* stream);

/* ---------------------------------------------------------------------- */
/* The residual / skip update between two WN layers of the fp16-autocast  */
/* training step (modules.py:93-182): x' = (x + rs[:, :H]) * mask (fp32), */
/* x16' = x' rounded to the 16-bit type (the next conv's input), out' =   */
/* out + rs[:, H:] (out NULL = 0); rs [B][2H][T] of the 16-bit type, x /  */
/* out / x' / out' [B][H][T] fp32, mask [B][1][T] fp32, all contiguous.   */
/* backward: G = dx' + dx16' (either NULL = 0), dx = G * mask, drs =      */
/* [G * mask ; dout'] rounded to the 16-bit type (dout' NULL = 0).        */
/* ---------------------------------------------------------------------- */
int vits_wn_update_forward(const float* x, const void* rs, const float* mask, const float* out,
                           float* x_new, void* x16_new, float* out_new, int batch, int H, int T,
                           int wdtype, void* stream);
int vits_wn_update_backward(const float* gx, const void* gx16, const float* gout,
                            const float* mask, float* dx, void* drs, int batch, int H, int T,
                            int wdtype, void* stream);

/* ---------------------------------------------------------------------- */
/* Mean-only coupling layer glue of the fp16-autocast training step       */
/* (ResidualCouplingLayer.forward modules.py:314-360, WN output           */
/* modules.py:182, Flip folded in: ResidualCouplingBlock models.py:219-235).*/
/* mask_cast: h = y * mask (fp32) and h16 = h in the 16-bit type;          */
/*   backward: dy = 16-bit((gh + gh16) * mask) (either NULL = 0).         */
/* wn_final: o16 = 16-bit((out + rs) * mask) (out NULL = 0); backward:    */
/*   d = g16 * mask, dout = d (fp32, NULL = skip), drs = 16-bit(d).       */
/* coupling: x [B][2h][T] fp32, p = post conv output [B][h][T] 16-bit,    */
/*   m = p * mask; out = cat(x0, reverse ? (x1 - m) * mask :              */
/*   m + x1 * mask), channel-reversed when flip; backward: gx0 = g0, gx1 = */
/*   g1 * mask, gp = 16-bit(+-g1 * mask) (g read through the same flip).  */
/* ---------------------------------------------------------------------- */
int vits_mask_cast_forward(const void* y, const float* mask, float* h, void* h16, int batch,
                           int C, int T, int wdtype, void* stream);
int vits_mask_cast_backward(const float* gh, const void* gh16, const float* mask, void* dy,
                            int batch, int C, int T, int wdtype, void* stream);
int vits_wn_final_forward(const float* out, const void* rs, const float* mask, void* o16,
                          int batch, int C, int T, int wdtype, void* stream);
int vits_wn_final_backward(const void* g16, const float* mask, float* dout, void* drs, int batch,
                           int C, int T, int wdtype, void* stream);
int vits_coupling_forward(const float* x, const void* p, const float* mask, float* out,
                          int batch, int half, int T, int reverse, int flip, int wdtype,
                          void* stream);
int vits_coupling_backward(const float* g, const float* mask, float* gx, void* gp, int batch,
                           int half, int T, int reverse, int flip, int wdtype, void* stream);

/* ---------------------------------------------------------------------- */
/* STFT-discriminator glue of the fp16-autocast training step             */
/* (mrd.py:94-156, STFTDiscriminator.forward: Conv2d -> LeakyReLU ...).   */
/* join_to_cl: the first layer's joined-row conv output y [B][C][F_out*L] */
/* (row f's T outputs at columns f*L + p1 ..) -> out [B][F_out][T][C]     */
/* (NHWC) = leaky_relu(y, slope); backward: dy [B][C][F_out*L] =          */
/* lrelu'(out) * g at output columns, 0 at pad columns.                   */
/* bias_lrelu: out = leaky_relu(y + fp16(bias), slope) on NHWC rows of C  */
/* channels (the MIOpen conv runs without bias); backward: dy = lrelu'(out)*g */
/* and db[c] = fp16-rounded fp32 sum of dy (deterministic: per-workgroup  */
/* partials in `workspace`, added in workgroup order by a second launch; */
/* db NULL: the data gradient only, one launch, no workspace).           */
/* 16-bit tensors of `wdtype`; C % 8 == 0, C <= 512 (bias_lrelu backward: */
/* 256 % (C/8) == 0).                                                      */
/* ---------------------------------------------------------------------- */
int vits_stftd_join_to_cl_forward(const void* y, void* out, int batch, int C, int F_out, int L,
                                  int p1, int T, float slope, int wdtype, void* stream);
int vits_stftd_join_to_cl_backward(const void* g, const void* out, void* dy, int batch, int C,
                                   int F_out, int L, int p1, int T, float slope, int wdtype,
                                   void* stream);
int vits_bias_lrelu_forward(const void* y, const float* bias, void* out, int64_t rows, int C,
                            float slope, int wdtype, void* stream);
int vits_bias_lrelu_workspace(int64_t rows, int C);
int vits_bias_lrelu_backward(const void* g, const void* out, void* dy, float* db,
                             float* workspace, int ws_floats, int64_t rows, int C, float slope,
                             int wdtype, void* stream);

/* library introspection */
const char* vits_amd_version(void);
int vits_amd_device_arch(char* buf, int len);

/* Dispatch counters: how many kernel launches each family of entry points */
/* has issued since the last reset (host-side counts, one per launched     */
/* kernel, incremented only when the launch was accepted).  Tests use them */
/* to prove that a step ran on this library's kernels (not a torch path).  */
#define VITS_CNT_CONV_F32 0      /* vits_conv1d_forward*: exact fp32 MFMA    */
#define VITS_CNT_CONV_SPLIT 1    /*   split fp32 (VITS_WDT_F32S / F32P)     */
#define VITS_CNT_CONV_16 2       /*   bf16 / fp16 operands                  */
#define VITS_CNT_WGRAD_F32 3     /* vits_conv1d_wgrad(_split), fp32 operands */
#define VITS_CNT_WGRAD_16 4      /*   16-bit operands                       */
#define VITS_CNT_GATE_F32 5      /* vits_gate_forward / _backward           */
#define VITS_CNT_GATE_16 6       /* vits_gate_*_io16                        */
#define VITS_CNT_RESBLOCK 7      /* vits_resblock_pair*_forward             */
#define VITS_CNT_PACK 8          /* vits_conv1d_pack*                       */
#define VITS_CNT_N 9
int64_t vits_dispatch_count(int which);
void vits_dispatch_count_reset(void);

#ifdef __cplusplus
}
#endif
#endif /* VITS_AMD_H */
