"""Tensor-level wrappers over the C-ABI (libvits_amd.so).

Every function here requires CUDA(ROCm) tensors and launches HIP kernels on
the current torch stream; there is no CPU path (a CPU tensor raises).
Weight packing helpers turn reference-layout conv weights into the
``[cin_pad][k][m_pad]`` slabs the MFMA conv kernel streams.
"""
from __future__ import annotations

import contextlib
import ctypes as C
import threading
from dataclasses import dataclass, field
from typing import Optional

import numpy as np
import torch

from . import _lib
from ._lib import (ACT_NONE, WDT_BF16, WDT_F16, WDT_F32, WDT_F32P, WDT_F32S, ConvDesc, ConvOut, EPI_GATE, EPI_STORE,
                   ResblockPairDesc,
                   EPI_UPSAMPLE, TILE_128x128, TILE_32x256, TILE_64x128, TILE_64x256, TILE_ROWS,
                   check)

# ---------------------------------------------------------------------------
# plumbing
# ---------------------------------------------------------------------------


def _stream_ptr(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def require_device(*tensors: torch.Tensor):
    for t in tensors:
        if t is None:
            continue
        if t.device.type != "cuda":
            raise _lib.VitsAmdError(
                "vits_amd HIP ops need tensors on a ROCm GPU (device 'cuda'); "
                f"got {t.device}. There is no CPU path.")


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


_WEIGHT_CACHE: dict = {}


def set_weight_cache(cache: dict) -> dict:
    """Install ``{module: effective weight}`` (wnorm.WeightNormCache.active:
    every weight-normed layer of a network computed in one launch); returns
    the previous mapping."""
    global _WEIGHT_CACHE
    prev, _WEIGHT_CACHE = _WEIGHT_CACHE, cache
    return prev


def cached_weight(module: torch.nn.Module):
    return _WEIGHT_CACHE.get(module)


def weight_norm_effective(module: torch.nn.Module, name: str = "weight") -> torch.Tensor:
    """Effective weight of a (legacy) weight-normed or plain layer."""
    w = _WEIGHT_CACHE.get(module) if name == "weight" else None
    if w is not None:
        return w
    g = getattr(module, name + "_g", None)
    v = getattr(module, name + "_v", None)
    if g is not None and v is not None:
        return torch._weight_norm(v, g, 0)
    return getattr(module, name)


# ---------------------------------------------------------------------------
# conv layer packing
# ---------------------------------------------------------------------------


def _pick_tile(m: int, k: int) -> int:
    """fp32 workgroup tile by GEMM rows and taps, from the per-shape sweep of
    tools/conv_bench.py on MI355X (B=16, Ty=500 decoder/flow shapes, 16-byte
    X staging): 32 rows -> 32x256; the 2-tap polyphase ups and 1x1 convs ->
    64x128; everything else -> 64x256 (k=3: +3..5 %, k=7: +6 %, k=11: +5 %
    over 128x128 / 64x128).  Grids too small to fill the chip twice fall back
    to 64x128 at launch (conv1d.hip)."""
    if m <= 32:
        return TILE_32x256
    if k <= 2:
        return TILE_64x128
    return TILE_64x256


def _pick_tile_bf16(m: int, k: int) -> int:
    """bf16-MFMA tile (same sweep, BF=1): short kernels on >= 128 rows are
    fastest as 128x128 (k=3: 430 vs 340 TF/s), long ones as 64x256
    (k=11: 730 vs 555), 64-row k<=7 as 64x128, 32 rows as 32x256."""
    if m <= 32:
        return TILE_32x256
    if k <= 3:
        return TILE_128x128 if m >= 128 else TILE_64x128
    if m >= 128 or k >= 9:
        return TILE_64x256
    return TILE_64x128


TILE_COLS = {TILE_128x128: 128, TILE_64x256: 256, TILE_32x256: 256, TILE_64x128: 128}
W_TILE_FLOATS = 4096                                   # conv1d.hip VITS_W_TILE
X_TILE_FLOATS = {128: 2048, 256: 4096}                  # conv1d.hip XTile<BN>::floats


# workgroups per CU each tile reaches by its VGPR count (ISA dump of
# conv1d.hip: 128x128 154 VGPRs -> 3 waves/SIMD, 64x256 / 32x256 ~122 -> 4,
# 64x128 89 -> 5; 64x256 is budgeted at 3: its k=7 convs run faster with the
# bigger chunk); the K-chunk is sized so that LDS does not cut this further
TILE_OCCUPANCY = {TILE_128x128: 3, TILE_64x256: 3, TILE_32x256: 4, TILE_64x128: 5}
LDS_BYTES_PER_CU = 160 * 1024


def _pick_kc(cin: int, k: int, dil: int, tile: int) -> int:
    """Input channels per K-chunk: the largest even kc within the kernel's
    per-stage LDS/register budgets (W chunk kc*k*BM floats, X chunk
    kc*xw_pad floats) AND within the LDS share that keeps the tile's VGPR
    occupancy (the conv is latency-bound at small K: on MI355X a 64x128 k=3
    conv runs 86 TF/s at kc=10 / 5 WGs per CU but 77 TF/s at kc=14 / 4)."""
    bm, bn = TILE_ROWS[tile], TILE_COLS[tile]
    # + 4: the 16-byte staging path aligns the window start down to 4 columns
    xw_pad = (bn + (k - 1) * dil + 3) // 4 * 4 + 4
    lds_fixed = 4 * (2 * k * bm + 2 * xw_pad + 64)
    lds_floats = (LDS_BYTES_PER_CU // TILE_OCCUPANCY[tile] - lds_fixed) // 8  # per stage, W+X
    occ_kc = lds_floats // (k * bm + xw_pad)
    occ_kc = max(occ_kc, 2 * -(-12 // k))  # but keep >= ~24 taps x channels per chunk
    budget = min(32, W_TILE_FLOATS // (k * bm), X_TILE_FLOATS[bn] // xw_pad, occ_kc,
                 cin + (cin & 1))
    budget = max(2, budget - (budget & 1))
    # zero-padded channels cost MFMA work, each chunk costs a fixed overhead
    # (~2 channels' worth): minimise ceil(cin/kc) * (kc + 2)
    kc = min(range(2, budget + 1, 2), key=lambda c: (-(-cin // c) * (c + 2), -(-cin // c) * c, -c))
    assert kc * k * bm <= W_TILE_FLOATS and kc * xw_pad <= X_TILE_FLOATS[bn], (cin, k, dil, tile)
    return kc


@dataclass
class PackedConv:
    """A conv (or polyphase conv-transpose) lowered for vits_conv1d_forward."""

    w: torch.Tensor            # [cin_pad, k, m_pad] fp32 contiguous
    bias: Optional[torch.Tensor]
    cin: int
    m: int                     # GEMM rows
    k: int
    dil: int
    pad_left: int
    epi: int
    tile: int
    kc: int
    up_u: int = 1
    up_pad: int = 0
    out_channels: int = 0      # channels of the produced tensor
    extra: dict = field(default_factory=dict)
    wdtype: int = WDT_F32      # WDT_BF16 / WDT_F16: w is [cin_pad/16][k][2][m_pad][8] 16-bit
                               # (16-channel slabs; a K-chunk of kc channels = kc/16 slabs)

    @property
    def m_pad(self) -> int:
        if self.wdtype == WDT_F32P:
            return self.w.shape[4]
        return self.w.shape[3] if self.wdtype != WDT_F32 else self.w.shape[2]

    @property
    def cin_pad(self) -> int:
        return self.w.shape[0] * 16 if self.wdtype != WDT_F32 else self.w.shape[0]


def _finish_pack(rows_w: torch.Tensor, k: int, tile: int, dil: int = 1) -> tuple[torch.Tensor, int]:
    """rows_w: [m, cin, k] -> packed [cin_pad, k, m_pad]."""
    m, cin, _ = rows_w.shape
    kc = _pick_kc(cin, k, dil, tile)
    cin_pad = (cin + kc - 1) // kc * kc
    m_pad = (m + 127) // 128 * 128
    packed = rows_w.new_zeros(cin_pad, k, m_pad, dtype=torch.float32)
    packed[:cin, :, :m] = rows_w.permute(1, 2, 0).to(torch.float32)
    return packed.contiguous(), kc


class _PackPrecision(threading.local):
    wdtype = WDT_F32


PACK_PRECISION = _PackPrecision()
_WDT_TORCH = {WDT_BF16: torch.bfloat16, WDT_F16: torch.float16}


@contextlib.contextmanager
def pack_lowp(wdtype: int = WDT_BF16):
    """While active, pack_conv / pack_conv_transpose return 16-bit-MFMA layers
    (WDT_BF16 or WDT_F16; WDT_F32 = exact fp32).  Engine plans of a bf16 /
    fp16 model are built under it."""
    old = PACK_PRECISION.wdtype
    PACK_PRECISION.wdtype = int(wdtype)
    try:
        yield
    finally:
        PACK_PRECISION.wdtype = old


def pack_bf16(enabled: bool = True):
    return pack_lowp(WDT_BF16 if enabled else WDT_F32)


def _pick_tile_f32s(m: int, k: int) -> int:
    """Split-fp32 tile (VITS_WDT_F32S), from the per-shape sweep of
    tools/conv_bench.py (WDT=3 TILES=0,1,2,3) on MI355X at B=16, Ty=500
    (profiles/r02_split_conv_sweep.txt): k = 3 on >= 128 rows -> 128x128
    (W pre-split too, 131-140 TF/s), k <= 8 otherwise -> 64x128 (k=7
    147-159, the polyphase upsamplers 111-117, conv_pre 135, flow k=5 133),
    k >= 9 -> 64x256 (k=11 145-158)."""
    if k == 3 and m >= 128:
        return TILE_128x128
    if k <= 8:
        return TILE_64x128
    return TILE_64x256


def _pick_tile_f32p(m: int, k: int) -> int:
    """Tile of the pre-split-weight kernel (VITS_WDT_F32P): W is read from
    global memory, so the LDS holds only the double-buffered window and
    128x128 (2x2 waves of 64x64: two A and two B fragment triples feed 24
    MFMAs per k-step) fits every decoder shape; grids too small to fill the
    chip twice fall back to 64x128 in the dispatcher."""
    return TILE_128x128 if m >= 128 else TILE_64x128


# channels per K-chunk of the pre-split kernel: 32 (two slabs, half the
# chunk barriers) when the window of a 32-channel chunk fits the staging
# budget (conv1d_impl.h XTile<BN, true, true>: 6144 / 10240 elements for 128
# / 256 columns), else 16; F32P_MAX_KC = 16 forces single slabs
F32P_MAX_KC = 32


def _kc_f32p(cin_pad: int, k: int, dil: int, tile: int) -> int:
    if tile == TILE_64x128:
        # 64-row layers (the 64-channel decoder stage): 16-channel chunks halve
        # the double-buffered window (3 instead of 2 workgroups per CU);
        # measured on MI355X (tools/conv_bench.py WDT=3, r03): c1 k=3/7/11
        # +15/+8/+3 %, c2 +12..17 % over 32-channel chunks.  A 1x1 layer's
        # window is one tile wide, and its chunks are latency-bound: 32
        # channels (the flow's 96-row post conv: 29.5 -> 21.6 us, r06; the
        # k-steps and so the accumulation order are the same either way)
        return 32 if (k == 1 and cin_pad % 32 == 0) else 16
    bn = TILE_COLS[tile]
    xrs = (bn + (k - 1) * dil + 3 + 3) // 4 * 4  # window row incl. the 16-byte alignment shift
    budget = 6144 if bn <= 128 else 10240
    if F32P_MAX_KC >= 32 and cin_pad % 32 == 0 and 32 * xrs <= budget:
        return 32
    return 16


# pre-split weights for split fp32 (False: the F32S kernel, which
# splits the fp32 weight slabs per fragment in registers)
SPLIT_W = True


def split_planes(w: torch.Tensor) -> torch.Tensor:
    """Exact three-term bf16 split of an fp32 tensor, stacked on a new
    dimension -4 as (hi, mid, lo) planes: hi = x truncated to bf16, mid =
    (x - hi) truncated, lo = x - hi - mid (<= 8 significant bits), so
    hi + mid + lo == x bit for bit - conv1d_impl.h split3_bf16 on the host."""
    w = w.to(torch.float32).contiguous()
    mask = -65536  # (a Python scalar: no host-to-device copy, graph-capture safe)
    h = (w.view(torch.int32) & mask).view(torch.float32)
    # (a non-finite weight keeps mid = lo = 0: inf - inf would make them NaN;
    # a NaN stays NaN in hi even when its payload sits in the truncated bits)
    h = torch.where(torch.isnan(w), w, h)
    r = torch.where(torch.isfinite(w), w - h, torch.zeros_like(w))
    m = (r.view(torch.int32) & mask).view(torch.float32)
    lo = r - m
    return torch.stack([h, m, lo], dim=-3).to(torch.bfloat16)


# Split-fp32 layers need >= this many GEMM rows: the r02 sweep measured the
# per-fragment split (F32S) ahead of the exact-f32 kernel on every 128- /
# 256-channel decoder conv (+8..35 %), the upsamplers, conv_pre and the flow,
# but behind it on the 32- / 64-channel stages.  With pre-split weights
# (F32P, tools/conv_bench.py on MI355X, r03) the 64-channel stage gains too
# (k=11 c1 180 vs 122 TF/s exact, c2 138 vs 107, k=7 c1 154 vs 104; k=3 c2
# 56 vs 60), the 32-channel one still does not (k=11 92 vs 108): 64 rows.
F32S_MIN_ROWS = 0


def _f32s_min_rows() -> int:
    return F32S_MIN_ROWS or (64 if SPLIT_W else 128)


def to_lowp(layer: PackedConv, wdtype: int = WDT_BF16, min_rows: Optional[int] = None) -> PackedConv:
    """Re-pack an fp32 layer for the 16-bit-MFMA kernel variant (bf16 or
    fp16 operands, fp32 accumulation): K-chunks of 16 channels, W as
    [cin_pad/16][k][2][m_pad][8] (one 16-byte A fragment per row and 8
    channels), tile by _pick_tile_bf16.  WDT_F32S keeps that slab image in
    fp32 (split into three exact bf16 terms inside the kernel)."""
    if layer.wdtype != WDT_F32 or wdtype == WDT_F32:
        return layer
    if wdtype == WDT_F32S:
        # (min_rows: the fused split-fp32 pairs take the 32-row convs too)
        if layer.m < (_f32s_min_rows() if min_rows is None else min_rows):
            return layer
        kc = 16
        w32 = layer.w[:layer.cin]
        cin_pad = (layer.cin + kc - 1) // kc * kc
        k, m_pad = w32.shape[1], w32.shape[2]
        w = w32.new_zeros(cin_pad, k, m_pad)
        w[:layer.cin] = w32
        w = w.view(cin_pad // kc, kc // 8, 8, k, m_pad).permute(0, 3, 1, 4, 2).contiguous()
        if SPLIT_W:
            # [cin_pad/16][k][2][3][m_pad][8] bf16: planes next to the lane half
            tile = _pick_tile_f32p(layer.m, layer.k)
            return PackedConv(split_planes(w), layer.bias, layer.cin, layer.m, layer.k,
                              layer.dil, layer.pad_left, layer.epi, tile,
                              _kc_f32p(cin_pad, layer.k, layer.dil, tile), up_u=layer.up_u,
                              up_pad=layer.up_pad, out_channels=layer.out_channels,
                              extra=layer.extra, wdtype=WDT_F32P)
        return PackedConv(w, layer.bias, layer.cin, layer.m, layer.k, layer.dil,
                          layer.pad_left, layer.epi, _pick_tile_f32s(layer.m, layer.k), kc,
                          up_u=layer.up_u, up_pad=layer.up_pad,
                          out_channels=layer.out_channels, extra=layer.extra, wdtype=wdtype)
    kc = 16
    w32 = layer.w[:layer.cin]                          # [cin, k, m_pad]
    cin_pad = (layer.cin + kc - 1) // kc * kc
    k, m_pad = w32.shape[1], w32.shape[2]
    w = w32.new_zeros(cin_pad, k, m_pad)
    w[:layer.cin] = w32
    w = w.view(cin_pad // kc, kc // 8, 8, k, m_pad).permute(0, 3, 1, 4, 2).contiguous()
    tile = _pick_tile_bf16(layer.m, layer.k)
    return PackedConv(w.to(_WDT_TORCH[wdtype]), layer.bias, layer.cin, layer.m, layer.k,
                      layer.dil, layer.pad_left, layer.epi, tile, kc, up_u=layer.up_u,
                      up_pad=layer.up_pad, out_channels=layer.out_channels, extra=layer.extra,
                      wdtype=wdtype)


# K-chunk of 16-bit inference layers whose activations are 16-bit too
# (engine.ACT16): the X window of a chunk stages at 2 bytes per element, so a
# chunk can hold 32-64 channels instead of 16 (fewer barriers per tile).
# VITS_LOWP_KCK caps kc * k (16: keep kc = 16, for A/B).
LOWP_KCK = 512


def io16_kc(layer: PackedConv) -> int:
    """Largest kc in (64, 48, 32, 16) dividing cin_pad that fits the kernel's
    W stage (kc*k*BM/2 <= 6144 slots, for the LDS-weight groups) and the
    16-bit X budget (conv1d_impl.h XTile<BN, BF, true>: 6144 / 10240
    elements for BN 128 / 256)."""
    bm, bn = TILE_ROWS[layer.tile], TILE_COLS[layer.tile]
    xrs = bn + (layer.k - 1) * layer.dil + 8
    xbudget = 6144 if bn <= 128 else 10240
    for kc in (64, 48, 32):
        if (kc * layer.k <= LOWP_KCK and layer.cin_pad % kc == 0
                and kc * layer.k * bm // 2 <= 6144 and kc * xrs <= xbudget):
            return kc
    return 16


def to_bf16(layer: PackedConv) -> PackedConv:
    return to_lowp(layer, WDT_BF16)


def pack_conv(weight: torch.Tensor, bias: Optional[torch.Tensor], *, dilation: int = 1,
              padding: Optional[int] = None, gate: bool = False) -> PackedConv:
    """nn.Conv1d weight [Cout, Cin, k].  ``gate``: rows (a_p, b_p) interleaved
    so the tanh/sigmoid pair of output p lands in one lane (EPI_GATE)."""
    w = weight.detach().to(torch.float32)
    cout, cin, k = w.shape
    if padding is None:
        padding = (k * dilation - dilation) // 2
    if gate:
        assert cout % 2 == 0
        h = cout // 2
        rows = torch.stack([w[:h], w[h:]], dim=1).reshape(cout, cin, k)
        epi, outc = EPI_GATE, h
    else:
        rows, epi, outc = w, EPI_STORE, cout
    tile = _pick_tile(cout, k)
    packed, kc = _finish_pack(rows, k, tile, dilation)
    b = None if bias is None else bias.detach().to(torch.float32).contiguous()
    layer = PackedConv(packed, b, cin, cout, k, dilation, padding, epi, tile, kc,
                       out_channels=outc)
    return to_lowp(layer, PACK_PRECISION.wdtype)


def pack_conv_transpose(weight: torch.Tensor, bias: Optional[torch.Tensor], stride: int,
                        padding: int) -> PackedConv:
    """nn.ConvTranspose1d weight [Cin, Cout, K] (K % stride == 0) as one
    polyphase conv: GEMM row (o*u + r) holds phase r of output channel o,
    tap j' reads x[q - (K/u - 1) + j'] with W'[(o,r)][c][j'] = W[c][o][(K/u-1-j')u + r]."""
    w = weight.detach().to(torch.float32)
    cin, cout, K = w.shape
    u = stride
    assert K % u == 0, "polyphase lowering needs kernel_size % stride == 0"
    kp = K // u
    # W[c][o][i*u + r] -> [c][o][i][r]
    w4 = w.reshape(cin, cout, kp, u)
    # rows (o, r), taps j' = kp-1-i
    rows = w4.flip(2).permute(1, 3, 0, 2).reshape(cout * u, cin, kp)
    tile = _pick_tile(cout * u, kp)
    packed, kc = _finish_pack(rows, kp, tile)
    b = None if bias is None else bias.detach().to(torch.float32).contiguous()
    layer = PackedConv(packed, b, cin, cout * u, kp, 1, kp - 1, EPI_UPSAMPLE, tile, kc,
                       up_u=u, up_pad=padding, out_channels=cout)
    return to_lowp(layer, PACK_PRECISION.wdtype)


# ---------------------------------------------------------------------------
# conv descriptor construction / launch
# ---------------------------------------------------------------------------


def make_out(y: torch.Tensor, *, act: int = ACT_NONE, res: Optional[torch.Tensor] = None,
             res_scale: float = 1.0, accumulate: bool = False, post_div: float = 1.0,
             channel_offset: int = 0) -> ConvOut:
    o = ConvOut()
    o.y = y.data_ptr() + y.element_size() * channel_offset * y.stride(1)
    o.y_bstride = y.stride(0)
    o.y_cstride = y.stride(1)
    o.act = act
    if res is not None:
        o.res = res.data_ptr() + res.element_size() * channel_offset * res.stride(1)
        o.res_bstride = res.stride(0)
        o.res_cstride = res.stride(1)
    else:
        o.res = None
        o.res_bstride = 0
        o.res_cstride = 0
    o.res_scale = res_scale
    o.accumulate = 1 if accumulate else 0
    o.post_div = post_div
    return o


_LOWP_TORCH = {WDT_F16: torch.float16, WDT_BF16: torch.bfloat16}


class _LenSkip(threading.local):
    margin = 0


LEN_SKIP = _LenSkip()


@contextlib.contextmanager
def length_skip(margin: int = 64):
    """While active, descriptors built with ``lengths`` skip every tile that
    starts ``margin`` or more positions past lengths[b] (no compute, no
    write; vits_conv1d_desc.len_skip): the bucketed whole-utterance infer
    then costs what the utterance needs, not what the bucket holds.
    ``margin`` must exceed every consumer's input halo ((k - 1) * dil / 2 <=
    25 in the decoder)."""
    old = LEN_SKIP.margin
    LEN_SKIP.margin = int(margin)
    try:
        yield
    finally:
        LEN_SKIP.margin = old


def make_desc(layer: PackedConv, x: torch.Tensor, out0: ConvOut, *, out1: Optional[ConvOut] = None,
              split: Optional[int] = None, tin: Optional[int] = None, n_out: Optional[int] = None,
              in_slope: float = 1.0, cond: Optional[torch.Tensor] = None, cond_offset: int = 0,
              lengths: Optional[torch.Tensor] = None, t_out: int = 0,
              x_channel_offset: int = 0, io16: bool = False) -> ConvDesc:
    """io16: x / outputs / residuals / gmask are tensors of the layer's
    16-bit operand type - 1 (True) the fp16 training convs, 2 the 16-bit
    inference decoder (csrc/conv1d.hip ga16); fp32 otherwise."""
    if io16:
        assert layer.wdtype != WDT_F32 and x.dtype == _LOWP_TORCH[layer.wdtype]
    else:
        assert x.dtype == torch.float32
    d = ConvDesc()
    d.x = x.data_ptr() + x.element_size() * x_channel_offset * x.stride(1)
    d.io16 = int(io16)
    d.x_bstride = x.stride(0)
    d.x_cstride = x.stride(1)
    d.x_tstride = x.stride(2)
    d.cin = layer.cin
    d.tin = x.shape[2] if tin is None else tin
    d.in_slope = in_slope
    d.w = layer.w.data_ptr()
    d.m = layer.m
    d.m_pad = layer.m_pad
    d.cin_pad = layer.cin_pad
    d.kc = layer.kc
    d.k = layer.k
    d.dil = layer.dil
    d.pad_left = layer.pad_left
    if n_out is None:
        if layer.epi == EPI_UPSAMPLE:
            # phases q = 0 .. Tin + ceil(pad/u) - 1 cover every t in [0, Tin*u)
            n_out = d.tin + (layer.up_pad + layer.up_u - 1) // layer.up_u
        else:
            n_out = d.tin
    d.n_out = n_out
    d.tile = layer.tile
    d.epi = layer.epi
    d.bias = _ptr(layer.bias)
    if cond is not None:
        d.cond = cond.data_ptr() + 4 * cond_offset
        d.cond_bstride = cond.stride(0)
    else:
        d.cond = None
        d.cond_bstride = 0
    d.split = layer.m if split is None else split
    d.up_u = layer.up_u
    d.up_pad = layer.up_pad
    d.t_out = t_out
    d.lengths = _ptr(lengths)
    d.len_skip = LEN_SKIP.margin if lengths is not None else 0
    d.out0 = out0
    if out1 is not None:
        d.out1 = out1
    d.wdtype = layer.wdtype
    return d


def conv_flops(desc: ConvDesc, batch: int) -> int:
    """Algorithmic FLOPs of one conv launch (2 * MACs of the convolution it
    implements; for the polyphase conv-transpose: Cout * Tout * Cin * K/u)."""
    cols = desc.tin if desc.epi == EPI_UPSAMPLE else desc.n_out
    return 2 * batch * desc.m * cols * desc.cin * desc.k


# Dense MFMA peaks (MI355X_MICROARCH.md) of the arithmetic each weight type
# runs: exact fp32 on v_mfma_f32_32x32x2_f32 (157.3 TF/s); bf16 / fp16 ~2.5
# PF/s; split fp32 = six bf16 MFMAs per fp32 product, 2.5 PF / 6.
BF16_DENSE_PEAK_TFLOPS = 2500.0
MFMA_PEAK_TFLOPS = {WDT_F32: 157.3, WDT_BF16: BF16_DENSE_PEAK_TFLOPS,
                    WDT_F16: BF16_DENSE_PEAK_TFLOPS, WDT_F32S: BF16_DENSE_PEAK_TFLOPS / 6,
                    WDT_F32P: BF16_DENSE_PEAK_TFLOPS / 6}


class ConvTimer:
    """Optional per-launch timing of the conv kernel with HIP events on the
    launch stream (used by bench.py for the roofline of the dominant kernel).
    While active, batched launches are issued one descriptor at a time."""

    active = None

    def __init__(self):
        self.records = []  # (start_event, end_event, flops)
        self.shapes = []   # one label per record (tools/infer_breakdown.py)
        self.peaks = []    # MFMA-bound TFLOP/s of each record's arithmetic (MFMA_PEAK)

    def __enter__(self):
        ConvTimer.active = self
        return self

    def __exit__(self, *exc):
        ConvTimer.active = None
        return False

    def launch(self, lib, desc, batch, device):
        """One launch: a ConvDesc, or a tuple of ConvDescs run as one grid."""
        group = tuple(desc) if isinstance(desc, (tuple, list)) else (desc,)
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        stream = torch.cuda.current_stream(device)
        s.record(stream)
        arr = (ConvDesc * len(group))(*group)
        sizes = (C.c_int32 * 1)(len(group))
        check(lib.vits_conv1d_forward_groups(arr, sizes, 1, batch, stream.cuda_stream),
              "vits_conv1d_forward_groups")
        e.record(stream)
        self.records.append((s, e, sum(conv_flops(d, batch) for d in group)))
        self.peaks.append(MFMA_PEAK_TFLOPS[group[0].wdtype])
        self.shapes.append("conv " + "+".join(
            f"m{d.m}c{d.cin}k{d.k}d{d.dil}T{d.n_out}e{d.epi}t{d.tile}" for d in group))

    def launch_pairs(self, lib, group, batch, device, wdtype=None, mean=False):
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        stream = torch.cuda.current_stream(device)
        s.record(stream)
        arr = (ResblockPairDesc * len(group))(*group)
        if wdtype is None:
            check(lib.vits_resblock_pair_forward(arr, len(group), batch, stream.cuda_stream),
                  "vits_resblock_pair_forward")
        elif wdtype == WDT_F32P:
            check(lib.vits_resblock_pair_f32p_forward(arr, len(group), batch, stream.cuda_stream),
                  "vits_resblock_pair_f32p_forward")
        else:
            fn = lib.vits_resblock_pair16_mean_forward if mean else lib.vits_resblock_pair16_forward
            check(fn(arr, len(group), batch, int(wdtype), stream.cuda_stream),
                  "vits_resblock_pair16_forward")
        e.record(stream)
        self.records.append((s, e, sum(resblock_pair_flops(d, batch) for d in group)))
        self.peaks.append(MFMA_PEAK_TFLOPS[WDT_F32 if wdtype is None else
                                           WDT_F32S if wdtype == WDT_F32P else wdtype])
        self.shapes.append("pair " + "+".join(
            f"C{d.channels}k{d.k}d{d.dil}T{d.t_len}" for d in group))

    def summary(self):
        torch.cuda.synchronize()
        ms = [s.elapsed_time(e) for s, e, _ in self.records]
        fl = [f for _, _, f in self.records]
        # the MFMA-bound minimum time of the same launches (each at the peak
        # of the MFMA form its arithmetic runs on)
        min_ms = sum(f / (pk * 1e9) for f, pk in zip(fl, self.peaks))
        return dict(launches=len(ms), total_ms=float(sum(ms)), total_flops=int(sum(fl)),
                    avg_ms=float(sum(ms) / max(1, len(ms))), mfma_bound_ms=float(min_ms),
                    f32s_flops=int(sum(f for f, pk in zip(fl, self.peaks)
                                       if pk == MFMA_PEAK_TFLOPS[WDT_F32S])))

    def per_launch(self):
        """[(label, ms, flops)] in launch order."""
        torch.cuda.synchronize()
        return [(lab, s.elapsed_time(e), f)
                for lab, (s, e, f) in zip(self.shapes, self.records)]


# ---------------------------------------------------------------------------
# fused ResBlock2 pair (csrc/resblock.hip)
# ---------------------------------------------------------------------------
_RB_KC = {}


RESBLOCK_PAIR_MAX_K = 7


def resblock_pair_supported(c1: PackedConv, c2: PackedConv, T: int) -> bool:
    """Pairs that run fused (csrc/resblock.hip): the fp32 32- and 64-channel
    stages (C' = C, 16-byte aligned time rows) with k <= 7.  tools/rb_bench.py
    on MI355X (B=16, Ty=500): fused vs the two-conv path k=3 +6..11 %, k=7
    +0..10 %, k=11 -4..-8 % (the c1 phase recomputes the c2 halo and the
    workgroup holds the gated tile in LDS: two workgroups per CU instead of
    three) - so k=11 pairs keep the two-conv path."""
    C = c2.out_channels
    return (c1.wdtype == WDT_F32 and c2.wdtype == WDT_F32 and C in (32, 64)
            and c1.m == C and c1.cin == C and c2.cin == C // 2 and c1.k == c2.k
            and c1.k <= RESBLOCK_PAIR_MAX_K and c2.dil == 1 and T % 4 == 0
            and _resblock_kc(C, c1.k, c1.dil) is not None)


# split-fp32 fused pairs (csrc/resblock_f32p.hip): channels -> largest k that
# runs fused.  tools/rbp_bench.py on MI355X (B=16, Ty=500, each branch alone,
# profiles/r05_rbp_bench*.txt): C=64 fused vs two-conv k=3 -23 %, k=7 -12 %,
# k=11 -2 %; C=128 k=3 -25 %, k=7 -4..-8 %, k=11 +-0 (the c1 phase
# recomputes c2's halo: 10 of 128 columns at k=11); C=256 (one 512-thread
# workgroup per CU, 543 tiles per utterance batch: 2.1 rounds of the chip)
# k=3 -17 %, k=7 / k=11 +30..40 %.  The 32-channel stage's convs stay exact
# fp32 as single convs (32 rows), but its pairs run split fused too
# (engine.GeneratorPlan keeps split images beside them): vs the shipped exact
# pair / two-conv path k=3 -2..-5 %, k=7 -25..-33 %, k=11 -34..-35 %
F32P_PAIR_MAX_K = {32: 11, 64: 11, 128: 7, 256: 3}


def resblock_pair_f32p_supported(c1: PackedConv, c2: PackedConv, x: torch.Tensor) -> bool:
    """Pairs of an fp32 Generator's split-fp32 stages (pre-split images,
    VITS_WDT_F32P) that run fused (csrc/resblock_f32p.hip): odd k, 'same'
    padding, (k - 1) * dil <= 96, 16-byte aligned fp32 time rows."""
    C_ = c2.out_channels
    return (c1.wdtype == WDT_F32P and c2.wdtype == WDT_F32P and c1.k <= F32P_PAIR_MAX_K.get(C_, 0)
            and x.dtype == torch.float32 and c1.m == C_ and c1.cin == C_ and c2.cin == C_ // 2
            and c2.m == C_ and c1.k == c2.k and c1.k % 2 == 1 and (c1.k - 1) * c1.dil <= 96
            and c2.dil == 1 and c1.epi == EPI_GATE and c2.epi == EPI_STORE
            and (C_ != 256 or (c1.k - 1) * c1.dil <= 56)  # (its 64-channel X chunks' LDS)
            and c1.pad_left == (c1.k - 1) * c1.dil // 2 and c2.pad_left == (c2.k - 1) // 2
            and x.shape[2] % 4 == 0 and x.stride(2) == 1 and x.stride(1) % 4 == 0
            and x.stride(0) % 4 == 0 and x.data_ptr() % 16 == 0)


def _resblock_kc(ch: int, k: int, dil: int):
    key = (ch, k, dil)
    if key not in _RB_KC:
        kc1, kc2 = C.c_int(), C.c_int()
        rc = _lib.load().vits_resblock_pair_kc(ch, k, dil, kc1, kc2)
        _RB_KC[key] = (kc1.value, kc2.value) if rc == 0 else None
    return _RB_KC[key]


def resblock_pair_desc(c1: PackedConv, c2: PackedConv, x: torch.Tensor, y: torch.Tensor, *,
                       cond: Optional[torch.Tensor] = None, cond_offset: int = 0,
                       in_slope: float = 0.1, accumulate: bool = False,
                       post_div: float = 1.0,
                       lengths: Optional[torch.Tensor] = None) -> ResblockPairDesc:
    """y = x + c2(gate(c1(lrelu(x)) + cond)) in one launch (modules.py:250-260);
    ``lengths`` (int32 [B], device): the utterance ends there (zero past)."""
    assert x.dtype == torch.float32 and y.dtype == torch.float32 and x.stride(2) == 1
    C_, T = x.shape[1], x.shape[2]
    # (the split-fp32 kernel stages 16-channel slabs: no kc choice)
    kc1, kc2 = (16, 16) if c1.wdtype == WDT_F32P else _resblock_kc(C_, c1.k, c1.dil)
    d = ResblockPairDesc()
    d.x, d.x_bstride, d.x_cstride, d.t_len = x.data_ptr(), x.stride(0), x.stride(1), T
    d.channels, d.in_slope = C_, in_slope
    d.w1, d.m_pad1, d.cin_pad1, d.kc1 = c1.w.data_ptr(), c1.m_pad, c1.cin_pad, kc1
    d.k, d.dil, d.kc2 = c1.k, c1.dil, kc2
    d.b1 = _ptr(c1.bias)
    if cond is not None:
        d.cond, d.cond_bstride = cond.data_ptr() + 4 * cond_offset, cond.stride(0)
    d.w2, d.m_pad2, d.cin_pad2 = c2.w.data_ptr(), c2.m_pad, c2.cin_pad
    d.b2 = _ptr(c2.bias)
    d.y, d.y_bstride, d.y_cstride = y.data_ptr(), y.stride(0), y.stride(1)
    d.accumulate, d.post_div = int(accumulate), float(post_div)
    d.lengths = _ptr(lengths)
    d.len_skip = LEN_SKIP.margin if lengths is not None else 0
    return d


# fused pairs of 16-bit models (csrc/resblock16.hip): False keeps their
# two-conv path
FUSED_PAIRS16 = True
# largest k fused on the 256-channel stage (resblock_f32p.hip's 16-bit mode;
# 0 = none, the two-conv path)
PAIR16_256_MAX_K = 15


def resblock_pair16_supported(c1: PackedConv, c2: PackedConv, x: torch.Tensor) -> bool:
    """Pairs of a 16-bit model with 16-bit activations that run fused
    (csrc/resblock16.hip; the 256-channel stage csrc/resblock_f32p.hip),
    any odd k with (k - 1) * dil <= 96, 8-byte aligned time rows
    (T % 4 == 0)."""
    C_ = c2.out_channels
    if C_ == 256 and c1.k > PAIR16_256_MAX_K:
        return False
    return (FUSED_PAIRS16 and c1.wdtype in (WDT_BF16, WDT_F16) and c2.wdtype == c1.wdtype
            and x.dtype == _WDT_TORCH[c1.wdtype] and C_ in (32, 64, 128, 256) and c1.m == C_
            and c1.cin == C_ and c2.cin == C_ // 2 and c2.m == C_ and c1.k == c2.k
            and c1.k % 2 == 1 and (c1.k - 1) * c1.dil <= 96 and c2.dil == 1
            and c1.epi == EPI_GATE and x.shape[2] % 4 == 0 and x.stride(2) == 1
            and x.stride(1) % 4 == 0 and x.stride(0) % 4 == 0)


def resblock_pair16_desc(c1: PackedConv, c2: PackedConv, x: torch.Tensor, y: torch.Tensor, *,
                         cond: Optional[torch.Tensor] = None, cond_offset: int = 0,
                         in_slope: float = 0.1, accumulate: bool = False, post_div: float = 1.0,
                         lengths: Optional[torch.Tensor] = None) -> ResblockPairDesc:
    """resblock_pair_desc for resblock16 (16-bit x / y, 16-bit images)."""
    assert x.dtype == y.dtype == _WDT_TORCH[c1.wdtype] and x.stride(2) == 1 and y.stride(2) == 1
    C_, T = x.shape[1], x.shape[2]
    d = ResblockPairDesc()
    d.x, d.x_bstride, d.x_cstride, d.t_len = x.data_ptr(), x.stride(0), x.stride(1), T
    d.channels, d.in_slope = C_, in_slope
    d.w1, d.m_pad1, d.cin_pad1, d.kc1 = c1.w.data_ptr(), c1.m_pad, c1.cin_pad, 16
    d.k, d.dil, d.kc2 = c1.k, c1.dil, 16
    d.b1 = _ptr(c1.bias)
    if cond is not None:
        d.cond, d.cond_bstride = cond.data_ptr() + 4 * cond_offset, cond.stride(0)
    d.w2, d.m_pad2, d.cin_pad2 = c2.w.data_ptr(), c2.m_pad, c2.cin_pad
    d.b2 = _ptr(c2.bias)
    d.y, d.y_bstride, d.y_cstride = y.data_ptr(), y.stride(0), y.stride(1)
    d.accumulate, d.post_div = int(accumulate), float(post_div)
    d.lengths = _ptr(lengths)
    d.len_skip = LEN_SKIP.margin if lengths is not None else 0
    return d


def resblock_pair16_launch(descs, batch: int, device: torch.device, wdtype: int,
                           mean: bool = False):
    """One launch of up to 3 independent 16-bit pairs (tuple) or one pair;
    mean=True: the members' mean into descs[0]'s output
    (vits_resblock_pair16_mean_forward)."""
    group = tuple(descs) if isinstance(descs, (tuple, list)) else (descs,)
    lib = _lib.load()
    if ConvTimer.active is not None:
        return ConvTimer.active.launch_pairs(lib, group, batch, device, wdtype, mean=mean)
    arr = (ResblockPairDesc * len(group))(*group)
    fn = lib.vits_resblock_pair16_mean_forward if mean else lib.vits_resblock_pair16_forward
    check(fn(arr, len(group), batch, int(wdtype), _stream_ptr(device)),
          "vits_resblock_pair16_forward")


def resblock_pair_flops(d: ResblockPairDesc, batch: int) -> int:
    """Algorithmic FLOPs of the pair (c1 + c2 as the reference computes
    them; the kernel's recomputed halo columns are not counted)."""
    C_, k, T = d.channels, d.k, d.t_len
    return 2 * batch * T * (C_ * C_ * k + (C_ // 2) * C_ * k)


def resblock_pair_launch(descs, batch: int, device: torch.device, wdtype: int = WDT_F32):
    """One launch of up to 3 independent pairs (tuple) or one pair; wdtype
    WDT_F32 (exact fp32, csrc/resblock.hip) or WDT_F32P (split fp32,
    csrc/resblock_f32p.hip)."""
    group = tuple(descs) if isinstance(descs, (tuple, list)) else (descs,)
    lib = _lib.load()
    if ConvTimer.active is not None:
        return ConvTimer.active.launch_pairs(lib, group, batch, device,
                                             wdtype=WDT_F32P if wdtype == WDT_F32P else None)
    arr = (ResblockPairDesc * len(group))(*group)
    if wdtype == WDT_F32P:
        check(lib.vits_resblock_pair_f32p_forward(arr, len(group), batch, _stream_ptr(device)),
              "vits_resblock_pair_f32p_forward")
        return
    check(lib.vits_resblock_pair_forward(arr, len(group), batch, _stream_ptr(device)),
          "vits_resblock_pair_forward")


def conv1d_launch(desc: ConvDesc, batch: int, device: torch.device):
    lib = _lib.load()
    if ConvTimer.active is not None:
        return ConvTimer.active.launch(lib, desc, batch, device)
    check(lib.vits_conv1d_forward(C.byref(desc), batch, _stream_ptr(device)), "vits_conv1d_forward")


def conv1d_launch_seq(descs, batch: int, device: torch.device):
    """Run descriptors in order, one host call.  An item may be a tuple of
    independent ConvDescs (the ResBlock2 branches of one Generator stage):
    they share one launch (vits_conv1d_forward_groups)."""
    lib = _lib.load()
    if ConvTimer.active is not None:
        for d in descs:
            ConvTimer.active.launch(lib, d, batch, device)
        return
    flat, sizes = [], []
    for d in descs:
        group = tuple(d) if isinstance(d, (tuple, list)) else (d,)
        flat.extend(group)
        sizes.append(len(group))
    arr = (ConvDesc * len(flat))(*flat)
    sz = (C.c_int32 * len(sizes))(*sizes)
    check(lib.vits_conv1d_forward_groups(arr, sz, len(sizes), batch, _stream_ptr(device)),
          "vits_conv1d_forward_groups")


def conv1d(x: torch.Tensor, layer: PackedConv, *, in_slope: float = 1.0, act: int = ACT_NONE,
           cond: Optional[torch.Tensor] = None, residual: Optional[torch.Tensor] = None,
           res_scale: float = 1.0, lengths: Optional[torch.Tensor] = None,
           out: Optional[torch.Tensor] = None, accumulate: bool = False,
           post_div: float = 1.0, t_out: Optional[int] = None) -> torch.Tensor:
    """Run one packed conv on [B, cin, T] (device) and return [B, out_channels,
    T_out].  x fp32, or of the layer's 16-bit type (io16: output, residual
    and accumulator of that type too)."""
    require_device(x, cond, residual, lengths)
    B, _, T = x.shape
    io16 = x.dtype != torch.float32
    if layer.epi == EPI_UPSAMPLE:
        T_out = T * layer.up_u if t_out is None else t_out
    else:
        T_out = T
    if out is None:
        out = torch.empty(B, layer.out_channels, T_out, device=x.device, dtype=x.dtype)
    o0 = make_out(out, act=act, res=residual, res_scale=res_scale, accumulate=accumulate,
                  post_div=post_div)
    if lengths is not None:
        lengths = lengths.to(device=x.device, dtype=torch.int32).contiguous()
    d = make_desc(layer, x, o0, in_slope=in_slope, cond=cond, lengths=lengths, t_out=T_out,
                  io16=2 if io16 else 0)
    conv1d_launch(d, B, x.device)
    return out


# ---------------------------------------------------------------------------
# small kernels
# ---------------------------------------------------------------------------


def linear_rows(g: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor],
                out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y[b] = weight @ g[b] + bias (per-utterance conditioning)."""
    require_device(g, weight, bias)
    g = g.contiguous().float()
    B, n_in = g.shape
    n_out = weight.shape[0]
    if out is None:
        out = torch.empty(B, n_out, device=g.device, dtype=torch.float32)
    lib = _lib.load()
    check(lib.vits_linear_forward(g.data_ptr(), g.stride(0), weight.data_ptr(), _ptr(bias),
                                  out.data_ptr(), out.stride(0), B, n_out, n_in,
                                  _stream_ptr(g.device)), "vits_linear_forward")
    return out


def expand_prior(attn: torch.Tensor, m_p: torch.Tensor, s_p: torch.Tensor, noise: torch.Tensor,
                 out: Optional[torch.Tensor] = None, exp_s: bool = False,
                 noise_scale: float = 1.0) -> torch.Tensor:
    require_device(attn, m_p, s_p, noise)
    attn = attn.contiguous().float()
    m_p = m_p.contiguous().float()
    s_p = s_p.contiguous().float()
    noise = noise.contiguous().float()
    B, Ty, Tx = attn.shape
    Cc = m_p.shape[1]
    if out is None:
        out = torch.empty(B, Cc, Ty, device=attn.device, dtype=torch.float32)
    lib = _lib.load()
    check(lib.vits_expand_prior(attn.data_ptr(), m_p.data_ptr(), s_p.data_ptr(), noise.data_ptr(),
                                out.data_ptr(), B, Cc, Ty, Tx, 1 if exp_s else 0, noise_scale,
                                _stream_ptr(attn.device)),
          "vits_expand_prior")
    return out


ED_DRAWS = 32  # VITS_ED_DRAWS (include/vits_amd.h)


def numpy_draw_pool(n: int = ED_DRAWS):
    """The next ``n`` raw 32-bit MT19937 words of numpy's global legacy
    generator (RandomState.randint over the full uint32 range returns them
    unmasked, one word each) and the generator state before them.  The
    device consumes k of them the way ``np.random.randint(high)`` would;
    ``numpy_draw_commit`` then leaves the generator exactly where that
    randint call would have left it."""
    state = np.random.get_state()
    words = np.random.randint(0, 2 ** 32, size=n, dtype=np.uint32)
    return words.view(np.int32).copy(), state


def numpy_draw_commit(state, used: int) -> None:
    """Rewind numpy's global generator to ``state`` and advance it by the
    ``used`` words the device consumed (see numpy_draw_pool)."""
    np.random.set_state(state)
    if used > 0:
        np.random.randint(0, 2 ** 32, size=used, dtype=np.uint32)


def expand_durations(logw: torch.Tensor, m_p: torch.Tensor, s_p: torch.Tensor,
                     noise: torch.Tensor, t_y: int, *, rate: float = 1.0,
                     noise_scale: float = 1.0, x_len: Optional[torch.Tensor] = None,
                     noise_start: Optional[torch.Tensor] = None, half_round: bool = False,
                     stage_mult=(1,), out: Optional[torch.Tensor] = None,
                     lens: Optional[torch.Tensor] = None):
    """Durations -> (z [B, C, t_y], lens int32 [n_stage, B]) on the device,
    without the host sync of models.py:547 / infer.py:171: w_ceil =
    ceil(exp(logw) * rate), y_len = max(sum, 1), z = the one-hot expansion of
    m_p + noise * s_p * noise_scale over the static bucket t_y (0 past
    y_len), lens[i] = y_len * stage_mult[i].  ``noise`` is [B, C, t_y], or
    with ``noise_start`` (int32 [B]) a flat buffer read as EmoVITS slices it
    (element (c, t) at s + c * y_len + t): ``noise_start`` is then an int32
    [B, ED_DRAWS] pool of raw MT19937 words (``numpy_draw_pool``) from which the
    device draws s = np.random.randint(numel - C * y_len) exactly as numpy's
    legacy RandomState would, and ``lens`` gets one more row: the words
    consumed per utterance (-1: the slice does not fit; -2: every word of the
    pool was rejected, the caller advances by the pool and calls again; z is
    zero for both)."""
    require_device(logw, m_p, s_p, noise)
    B, C_, t_x = m_p.shape
    logw = logw.reshape(B, t_x).float().contiguous()
    m_p = m_p.float().contiguous()
    s_p = s_p.float().contiguous()
    noise = noise.float().contiguous()
    if out is None:
        out = torch.empty(B, C_, t_y, device=m_p.device, dtype=torch.float32)
    n_stage = len(stage_mult)
    rows = n_stage + (0 if noise_start is None else 1)
    if lens is None:
        lens = torch.empty(rows, B, device=m_p.device, dtype=torch.int32)
    if tuple(lens.shape) != (rows, B) or lens.dtype != torch.int32 or not lens.is_contiguous():
        raise _lib.VitsAmdError(f"expand_durations: lens must be int32 [{rows}, {B}]")
    mult = (C.c_int32 * n_stage)(*[int(v) for v in stage_mult])
    if noise_start is None:
        assert tuple(noise.shape) == (B, C_, t_y), noise.shape
    elif (tuple(noise_start.shape) != (B, ED_DRAWS) or noise_start.dtype != torch.int32
          or not noise_start.is_contiguous()):
        raise _lib.VitsAmdError(f"expand_durations: noise_start must be int32 [{B}, {ED_DRAWS}]")
    check(_lib.load().vits_expand_durations(
        logw.data_ptr(), logw.stride(0), _ptr(x_len), t_x, float(rate), int(half_round),
        m_p.data_ptr(), s_p.data_ptr(), m_p.stride(0), m_p.stride(1), noise.data_ptr(),
        0 if noise_start is None else 1, _ptr(noise_start), noise.numel(), float(noise_scale),
        out.data_ptr(),
        B, C_, t_y, lens.data_ptr(), mult, n_stage, _stream_ptr(m_p.device)),
        "vits_expand_durations")
    return out, lens


def conv_post_tanh(x: torch.Tensor, weight: torch.Tensor, out: Optional[torch.Tensor] = None):
    require_device(x, weight)
    B, Cc, T = x.shape
    k = weight.shape[-1]
    w = weight.reshape(Cc, k).contiguous().float()
    if out is None:
        out = torch.empty(B, 1, T, device=x.device, dtype=torch.float32)
    xdt = {torch.float32: WDT_F32, torch.bfloat16: WDT_BF16, torch.float16: WDT_F16}[x.dtype]
    lib = _lib.load()
    check(lib.vits_conv_post_tanh_lowp(x.data_ptr(), x.stride(0), x.stride(1), w.data_ptr(),
                                       out.data_ptr(), B, Cc, T, k, xdt, _stream_ptr(x.device)),
          "vits_conv_post_tanh_lowp")
    return out


def layer_norm_channels(x: torch.Tensor, gamma: Optional[torch.Tensor], beta: Optional[torch.Tensor],
                        eps: float = 1e-5, residual: Optional[torch.Tensor] = None,
                        out: Optional[torch.Tensor] = None,
                        lengths: Optional[torch.Tensor] = None,
                        post_add: Optional[torch.Tensor] = None, scale: float = 1.0,
                        pos: Optional[torch.Tensor] = None,
                        pos_alpha: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y = ((LN(x + residual) * gamma + beta) + post_add[b]) * scale + pos[t] * alpha,
    zeroed at t >= lengths[b]; x, residual, out are [B, C, T] contiguous."""
    require_device(x, residual, lengths, post_add, pos, pos_alpha)
    assert x.is_contiguous() and (residual is None or residual.is_contiguous())
    B, Cc, T = x.shape
    if out is None:
        out = torch.empty_like(x)
    if pos is not None:
        assert pos.is_contiguous() and pos.shape[-1] == Cc and pos.numel() >= T * Cc
    lib = _lib.load()
    check(lib.vits_layer_norm_channels(x.data_ptr(), _ptr(residual), _ptr(gamma), _ptr(beta),
                                       out.data_ptr(), B, Cc, T, eps, _ptr(lengths),
                                       _ptr(post_add), 0 if post_add is None else post_add.stride(0),
                                       scale, _ptr(pos), _ptr(pos_alpha),
                                       _stream_ptr(x.device)), "vits_layer_norm_channels")
    return out


def attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, n_heads: int,
              lengths: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None):
    """softmax((q/sqrt(d)) k^T, masked -1e4) v on [B, H*D, T] channel-major tensors."""
    require_device(q, k, v, lengths)
    B, Cc, T = q.shape
    D = Cc // n_heads
    assert q.stride() == k.stride() == v.stride() and q.stride(2) == 1 and q.stride(1) == T
    if out is None:
        out = torch.empty(B, Cc, T, device=q.device, dtype=torch.float32)
    assert out.stride(2) == 1 and out.stride(1) == T
    lib = _lib.load()
    check(lib.vits_attention_forward(q.data_ptr(), k.data_ptr(), v.data_ptr(), out.data_ptr(), B,
                                     n_heads, D, T, q.stride(0), out.stride(0), _ptr(lengths),
                                     _stream_ptr(q.device)), "vits_attention_forward")
    return out


_DT = {torch.float32: _lib.DT_F32, torch.float16: _lib.DT_F16, torch.bfloat16: _lib.DT_BF16,
       torch.int32: _lib.DT_I32}


def neg_cent(z_p: torch.Tensor, m_p: torch.Tensor, logs_p: torch.Tensor) -> torch.Tensor:
    """MAS scores [B, t_t, t_s] of models.py:483-490 in one fp32 MFMA kernel
    (no autograd: the reference computes them under torch.no_grad)."""
    require_device(z_p, m_p, logs_p)
    z = z_p.detach().to(torch.float32).contiguous()
    m = m_p.detach().to(torch.float32).contiguous()
    lg = logs_p.detach().to(torch.float32).contiguous()
    B, C, Tt = z.shape
    if m.shape != lg.shape or m.shape[0] != B or m.shape[1] != C:
        raise _lib.VitsAmdError(f"neg_cent: z_p {tuple(z.shape)} m_p {tuple(m.shape)} "
                                f"logs_p {tuple(lg.shape)}")
    Ts = m.shape[2]
    out = torch.empty(B, Tt, Ts, device=z.device, dtype=torch.float32)
    check(_lib.load().vits_neg_cent(z.data_ptr(), m.data_ptr(), lg.data_ptr(), out.data_ptr(),
                                    B, C, Tt, Ts, _stream_ptr(z.device)), "vits_neg_cent")
    return out


def maximum_path(neg_cent: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    """monotonic_align.maximum_path on the GPU (models.py:498 call contract)."""
    require_device(neg_cent, mask)
    dtype = neg_cent.dtype
    if dtype not in _DT:
        raise _lib.VitsAmdError(f"maximum_path: unsupported dtype {dtype}")
    nc = neg_cent.detach().to(torch.float32).contiguous()
    mk = mask.detach()
    if mk.dtype not in _DT:
        mk = mk.to(torch.float32)
    mk = mk.contiguous()
    B, Tt, Ts = nc.shape
    if mk.shape != nc.shape:
        raise _lib.VitsAmdError(f"maximum_path: mask {tuple(mk.shape)} vs neg_cent {tuple(nc.shape)}")
    path = torch.empty(B, Tt, Ts, device=nc.device, dtype=dtype)
    lib = _lib.load()
    wsb = int(lib.vits_maximum_path_workspace(B, Tt, Ts))
    ws = torch.empty(max(wsb, 16), device=nc.device, dtype=torch.uint8)
    check(lib.vits_maximum_path(nc.data_ptr(), mk.data_ptr(), _DT[mk.dtype], path.data_ptr(),
                                _DT[dtype], B, Tt, Ts, ws.data_ptr(), ws.numel(),
                                _stream_ptr(nc.device)), "vits_maximum_path")
    return path


def maximum_path_lengths(neg_cent: torch.Tensor, t_t: torch.Tensor, t_s: torch.Tensor,
                         dtype: torch.dtype = torch.float32) -> torch.Tensor:
    require_device(neg_cent, t_t, t_s)
    nc = neg_cent.detach().to(torch.float32).contiguous()
    B, Tt, Ts = nc.shape
    tt = t_t.to(torch.int32).contiguous()
    ts = t_s.to(torch.int32).contiguous()
    path = torch.empty(B, Tt, Ts, device=nc.device, dtype=dtype)
    lib = _lib.load()
    wsb = int(lib.vits_maximum_path_workspace(B, Tt, Ts))
    ws = torch.empty(max(wsb, 16), device=nc.device, dtype=torch.uint8)
    check(lib.vits_maximum_path_lengths(nc.data_ptr(), tt.data_ptr(), ts.data_ptr(),
                                        path.data_ptr(), _DT[dtype], B, Tt, Ts, ws.data_ptr(),
                                        ws.numel(), _stream_ptr(nc.device)),
          "vits_maximum_path_lengths")
    return path


# ---------------------------------------------------------------------------
# STFT magnitude with autograd
# ---------------------------------------------------------------------------


class _StftMag(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, window, n_fft, hop, win, pad, eps):
        require_device(x, window)
        x = x.contiguous().float()
        window = window.contiguous().float()
        B, L = x.shape
        frames = (L + 2 * pad - n_fft) // hop + 1
        nb = n_fft // 2 + 1
        mag = torch.empty(B, nb, frames, device=x.device, dtype=torch.float32)
        need_grad = ctx.needs_input_grad[0]
        re = torch.empty_like(mag) if need_grad else None
        im = torch.empty_like(mag) if need_grad else None
        lib = _lib.load()
        check(lib.vits_stft_mag_forward(x.data_ptr(), B, L, window.data_ptr(), n_fft, hop, win, pad,
                                        eps, mag.data_ptr(), _ptr(re), _ptr(im),
                                        _stream_ptr(x.device)), "vits_stft_mag_forward")
        if need_grad:
            ctx.save_for_backward(mag, re, im, window)
        ctx.cfg = (B, L, n_fft, hop, win, pad)
        return mag

    @staticmethod
    def backward(ctx, gmag):
        mag, re, im, window = ctx.saved_tensors
        B, L, n_fft, hop, win, pad = ctx.cfg
        gmag = gmag.contiguous().float()
        gx = torch.empty(B, L, device=gmag.device, dtype=torch.float32)
        lib = _lib.load()
        nws = int(lib.vits_stft_workspace(B, L, n_fft, hop, pad))
        ws = torch.empty(max(nws, 1), device=gmag.device, dtype=torch.float32)
        check(lib.vits_stft_mag_backward(gmag.data_ptr(), mag.data_ptr(), re.data_ptr(),
                                         im.data_ptr(), window.data_ptr(), B, L, n_fft, hop, win,
                                         pad, gx.data_ptr(), ws.data_ptr(), ws.numel(),
                                         _stream_ptr(gmag.device)), "vits_stft_mag_backward")
        return gx, None, None, None, None, None, None


class _StftMagMulti(torch.autograd.Function):
    """Magnitudes of several (signal, resolution) jobs in one launch each way
    (vits_stft_mag_{forward,backward}_multi); gradients flow to every input
    signal that requires them."""

    @staticmethod
    def forward(ctx, specs, *xs):
        # specs: tuple of (window, n_fft, hop, win, pad, eps) per job
        require_device(*xs)
        jobs = (_lib.StftJob * len(xs))()
        keep, mags, saved = [], [], []
        for i, (x, (window, n_fft, hop, win, pad, eps)) in enumerate(zip(xs, specs)):
            x = x.contiguous().float()
            window = window.contiguous().float()
            B, L = x.shape
            frames = (L + 2 * pad - n_fft) // hop + 1
            # frame-major storage (coalesced kernel stores, layout 1); the
            # caller gets the [B, n_fft/2+1, frames] view torch.stft returns
            mag = torch.empty(B, frames, n_fft // 2 + 1, device=x.device, dtype=torch.float32)
            need = ctx.needs_input_grad[i + 1]
            re = torch.empty_like(mag) if need else None
            im = torch.empty_like(mag) if need else None
            j = jobs[i]
            j.x, j.window, j.mag, j.re, j.im = x.data_ptr(), window.data_ptr(), mag.data_ptr(), \
                _ptr(re), _ptr(im)
            j.batch, j.length, j.n_fft, j.hop, j.win, j.pad, j.eps = B, L, n_fft, hop, win, pad, eps
            j.layout = 1
            keep += [x, window]
            mags.append(mag.transpose(1, 2))
            saved.append((mag, re, im, window, B, L, n_fft, hop, win, pad) if need else None)
        check(_lib.load().vits_stft_mag_forward_multi(jobs, len(xs), _stream_ptr(xs[0].device)),
              "vits_stft_mag_forward_multi")
        ctx.saved = saved
        ctx.dev = xs[0].device
        # magnitudes of signals that need no gradient (the MR-STFT target y)
        # stay plain tensors, as torch.stft of such a signal would be
        nd = [m for m, sv in zip(mags, saved) if sv is None]
        if nd:
            ctx.mark_non_differentiable(*nd)
        return tuple(mags)

    @staticmethod
    def backward(ctx, *gmags):
        idx = [i for i, sv in enumerate(ctx.saved) if sv is not None]
        grads = [None] * len(ctx.saved)
        if not idx:
            return (None,) + tuple(grads)
        jobs = (_lib.StftJob * len(idx))()
        keep = []
        for q, i in enumerate(idx):
            mag, re, im, window, B, L, n_fft, hop, win, pad = ctx.saved[i]
            g = gmags[i]
            # frame-major like the saved forward outputs (free when the
            # gradient is itself a transposed view of frame-major storage)
            g = torch.zeros_like(mag) if g is None else g.transpose(1, 2).contiguous().float()
            gx = torch.empty(B, L, device=ctx.dev, dtype=torch.float32)
            j = jobs[q]
            j.grad_mag, j.mag, j.re, j.im, j.window, j.grad_x = g.data_ptr(), mag.data_ptr(), \
                re.data_ptr(), im.data_ptr(), window.data_ptr(), gx.data_ptr()
            j.batch, j.length, j.n_fft, j.hop, j.win, j.pad = B, L, n_fft, hop, win, pad
            j.layout = 1
            keep.append(g)
            grads[i] = gx
        lib = _lib.load()
        nws = int(lib.vits_stft_workspace_multi(jobs, len(idx)))
        ws = torch.empty(max(nws, 1), device=ctx.dev, dtype=torch.float32)
        check(lib.vits_stft_mag_backward_multi(jobs, len(idx), ws.data_ptr(), ws.numel(),
                                               _stream_ptr(ctx.dev)), "vits_stft_mag_backward_multi")
        return (None,) + tuple(grads)


def stft_mag_multi(xs, specs):
    """[sqrt(|STFT(x_i)|^2 + eps_i)] for jobs (x_i, window_i, n_fft_i, hop_i,
    win_i, pad_i, eps_i) in one launch (at most 16 jobs); differentiable in
    every x_i.  specs: sequence of (window, n_fft, hop, win, pad, eps)."""
    if len(xs) > 16:
        raise _lib.VitsAmdError("stft_mag_multi: at most 16 jobs per launch")
    specs = tuple((w, int(n), int(h), int(wl), int(n) // 2 if p is None else int(p), float(e))
                  for (w, n, h, wl, p, e) in specs)
    # cast outside the Function so autograd returns gradients in each x's dtype
    return list(_StftMagMulti.apply(specs, *[x.float() for x in xs]))


def stft_mag(x: torch.Tensor, window: torch.Tensor, n_fft: int, hop: int, win: int,
             pad: Optional[int] = None, eps: float = 1e-7) -> torch.Tensor:
    """sqrt(|STFT(x)|^2 + eps), [B, n_fft//2+1, frames]; differentiable in x."""
    if pad is None:
        pad = n_fft // 2
    # cast outside the Function so autograd returns the gradient in x's dtype
    # (fp16 under autocast, as y_hat is in train_stft.py)
    return _StftMag.apply(x.float(), window, n_fft, hop, win, pad, eps)
