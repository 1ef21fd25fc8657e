"""Training-step convs on the HIP kernels (forward, input gradient, weight
gradient), as autograd functions.

The train_stft.py step (train_stft.py:162-236) runs every nn.Conv1d of the
generator (WN modules.py:130-182, ResBlock2 modules.py:250-260, couplings
modules.py:357-375, PosteriorEncoder models.py:268-279, Generator
models.py:306-318) and of the MWSD wave discriminators (mrd.py:15-55) under
fp16 autocast.  Here each such conv is one ``Conv1dHip`` call:

* forward: ``vits_conv1d_forward`` on a 16-bit image of the fp32 weight
  (``vits_conv1d_pack16``), activations fp32 in HBM, rounded to fp16 when
  staged, fp32 accumulation; an optional leaky-relu on the input (the
  ``F.leaky_relu`` / ``nn.LeakyReLU`` that precedes the conv in the
  reference) is fused into the staging, so the activated tensor is never
  materialised;
* input gradient: the same forward kernel on the transposed, tap-reversed
  weight image (dX = conv(dY, W'), pad' = (k-1)*dil - pad), times the
  leaky-relu derivative of the saved input;
* weight / bias gradient: ``vits_conv1d_wgrad`` (MFMA over the (b, t)
  reduction, bias sum fused).

Autocast: inputs are cast to fp32 and autocast is disabled inside
(``custom_fwd(cast_inputs=float32)``); outputs are fp32.  The reference's
autocast convs round inputs/weights to fp16 and return fp16; here operands
are rounded the same way but results stay fp32 (GradScaler overflow
semantics are the same: an fp16-overflowing gradient becomes inf).

``conv1d`` selects the path (``train_wdtype``): on a ROCm device it is
always a HIP path and raises if the library is missing - inside a 16-bit
autocast region (the reference's ``fp16_run``) the 16-bit kernels with fp16
activations, in fp32 training (autocast off, ``fp16_run: false``) the fp32
kernels (``Conv1dHip32``: forward / input gradient on the split- or exact-
fp32 MFMA conv of the inference path, weight gradient on the exact-fp32
MFMA ``wgrad_f32_kernel``; fp32 activations, the reference's fp32
precision).  On CPU, and with ``HIP_TRAIN = False`` (a test switch: the
reference's own torch arithmetic on the same device), it is the torch conv.
"""
from __future__ import annotations

import collections
import contextlib
import os
import sys

import torch
import torch.nn.functional as F
from torch import nn

from . import _lib
from ._lib import (EPI_GATE, EPI_STORE, TILE_32x256, TILE_64x128, TILE_64x256, TILE_128x128,
                   WDT_BF16, WDT_F16, WDT_F32, ConvWgradDesc, check)
from . import engine
from .ops import (PackedConv, _pick_tile_bf16, _stream_ptr, cached_weight, conv1d_launch,
                  conv1d_launch_seq,
                  make_desc, make_out,
                  pack_conv, to_lowp, weight_norm_effective)

_TORCH_16 = {WDT_F16: torch.float16, WDT_BF16: torch.bfloat16}
TRAIN_WDTYPE = WDT_F16  # the reference's autocast dtype (train_stft.py:165)


def _pick_tile_train(m: int, k: int, n_out: int | None) -> int:
    """16-bit tile for the training convs (tools/train_tile_sweep.py on
    MI355X): the inference rule (_pick_tile_bf16, tuned on long outputs)
    except short outputs on >= 128 rows with k <= 5 run as 128x128 (the
    FFN2 conv at T=100: 193 -> 266 TF/s; a 256-column tile is mostly
    padding there) and 128-row k <= 7 convs as 64x128 (ResBlock stage 2,
    k7: 307 -> 377 TF/s)."""
    if m > 32 and n_out is not None and n_out <= 128:
        return TILE_128x128 if (m >= 128 and k <= 5) else TILE_64x128
    if 64 < m <= 128 and 3 < k <= 7:
        return TILE_64x128
    return _pick_tile_bf16(m, k)


# K-chunk of the 16-bit training convs: kc channels (a multiple of 16) with
# kc * k <= TRAIN_KCK.  A chunk is one barrier-separated step of the
# kernel's two-stage global->LDS pipeline; at kc = 16 a 1x1 conv has one
# MFMA k-step per chunk and waits on every chunk's loads.
TRAIN_KCK = 64
_TILE_BM = {TILE_128x128: 128, TILE_64x128: 64, TILE_64x256: 64, TILE_32x256: 32}
_TILE_BN = {TILE_128x128: 128, TILE_64x128: 128, TILE_64x256: 256, TILE_32x256: 256}


def _train_kc(cin_pad: int, k: int, dil: int, tile: int, io16: bool) -> int:
    """Largest kc in (64, 48, 32, 16) that divides cin_pad and fits the
    kernel's W (kc*k*BM/2 <= 6144 slots) and X staging budgets
    (conv1d_impl.h XTile: 6144 / 10240 16-bit elements for BN 128 / 256 with
    16-bit activations, 3072 / 5120 otherwise)."""
    bm, bn = _TILE_BM[tile], _TILE_BN[tile]
    xrs = bn + (k - 1) * dil + 8
    xbudget = (6144 if bn <= 128 else 10240) if io16 else (3072 if bn <= 128 else 5120)
    for kc in (64, 48, 32):
        if (kc * k <= TRAIN_KCK and cin_pad % kc == 0
                and kc * k * bm // 2 <= 6144
                and kc * xrs <= xbudget):
            return kc
    return 16


# per-call weight packs by call site (tools/pack_census.py sets it)
PACK_TRACE = None  # tools/pack_census.py sets a collections.Counter()


def _trace_pack(kind, shape):
    if PACK_TRACE is not None:
        import traceback

        fr = [f for f in traceback.extract_stack(limit=8)[:-2]
              if not f.filename.endswith(("train_ops.py", "function.py"))]
        site = fr[-1] if fr else traceback.extract_stack(limit=3)[0]
        PACK_TRACE[(kind, tuple(shape), f"{os.path.basename(site.filename)}:{site.lineno}")] += 1


def _pack16(w32: torch.Tensor, transpose: bool, dil: int, pad_left: int, wdtype: int,
            bias: torch.Tensor | None = None, zero: torch.Tensor | None = None,
            n_out: int | None = None, io16: bool = False) -> PackedConv:
    """16-bit weight image (and, in the same launch, clear ``zero``)."""
    _trace_pack("pack16", w32.shape)
    cout, cin, k = w32.shape
    rows, chans = (cin, cout) if transpose else (cout, cin)
    m_pad = (rows + 127) // 128 * 128
    cin_pad = (chans + 15) // 16 * 16
    img = torch.empty(cin_pad // 16, k, 2, m_pad, 8, dtype=_TORCH_16[wdtype], device=w32.device)
    check(_lib.load().vits_conv1d_pack16(
        w32.data_ptr(), cout, cin, k, int(transpose), img.data_ptr(), m_pad, cin_pad, wdtype,
        None if zero is None else zero.data_ptr(), 0 if zero is None else zero.numel(),
        _stream_ptr(w32.device)), "vits_conv1d_pack16")
    tile = _pick_tile_train(rows, k, n_out)
    return PackedConv(img, bias, chans, rows, k, dil, pad_left, EPI_STORE, tile,
                      _train_kc(cin_pad, k, dil, tile, io16), out_channels=rows, wdtype=wdtype)


def _pack16_pair(w32: torch.Tensor, dil: int, pad_left: int, wdtype: int,
                 bias: torch.Tensor | None, n_out: int | None = None, n_in: int | None = None,
                 io16: bool = False):
    """The forward image and the input-gradient (transposed, tap-reversed)
    image of one weight in ONE launch: (forward PackedConv, backward
    PackedConv)."""
    _trace_pack("pair", w32.shape)
    cout, cin, k = w32.shape
    dt = _TORCH_16[wdtype]
    m_pad, cin_pad = (cout + 127) // 128 * 128, (cin + 15) // 16 * 16
    m_pad_t, cin_pad_t = (cin + 127) // 128 * 128, (cout + 15) // 16 * 16
    img = torch.empty(cin_pad // 16, k, 2, m_pad, 8, dtype=dt, device=w32.device)
    img_t = torch.empty(cin_pad_t // 16, k, 2, m_pad_t, 8, dtype=dt, device=w32.device)
    check(_lib.load().vits_conv1d_pack16_pair(
        w32.data_ptr(), cout, cin, k, img.data_ptr(), m_pad, cin_pad, img_t.data_ptr(), m_pad_t,
        cin_pad_t, wdtype, _stream_ptr(w32.device)), "vits_conv1d_pack16_pair")
    tf, tb = _pick_tile_train(cout, k, n_out), _pick_tile_train(cin, k, n_in)
    fwd = PackedConv(img, bias, cin, cout, k, dil, pad_left, EPI_STORE, tf,
                     _train_kc(cin_pad, k, dil, tf, io16), out_channels=cout, wdtype=wdtype)
    bwd = PackedConv(img_t, None, cout, cin, k, dil, (k - 1) * dil - pad_left, EPI_STORE, tb,
                     _train_kc(cin_pad_t, k, dil, tb, io16), out_channels=cin, wdtype=wdtype)
    return fwd, bwd


def _layers16(pre, shape, dil: int, pad_left: int, wdtype: int, bias, n_out: int, n_in: int):
    """(forward PackedConv, input-gradient PackedConv) around prepacked
    images (img, img_t) of a [cout, cin, k] weight (the 16-bit activation
    path, io16)."""
    img, img_t = pre
    cout, cin, k = shape
    tf, tb = _pick_tile_train(cout, k, n_out), _pick_tile_train(cin, k, n_in)
    fwd = PackedConv(img, bias, cin, cout, k, dil, pad_left, EPI_STORE, tf,
                     _train_kc(img.shape[0] * 16, k, dil, tf, True), out_channels=cout,
                     wdtype=wdtype)
    bwd = PackedConv(img_t, None, cout, cin, k, dil, (k - 1) * dil - pad_left, EPI_STORE, tb,
                     _train_kc(img_t.shape[0] * 16, k, dil, tb, True), out_channels=cin,
                     wdtype=wdtype)
    return fwd, bwd


# module -> (weight tensor, (img, img_t), wdtype): the images of every HIP
# conv of a network packed in one launch per 48 layers (prepacked) and used
# by conv1d() while the same weight tensor is served
_PREPACK: dict = {}


PREPACK = True


@contextlib.contextmanager
def prepacked(net: nn.Module):
    """Inside a 16-bit autocast region on the GPU: pack the 16-bit forward
    and input-gradient images of every Conv1d of ``net`` that ``conv1d``
    runs on the HIP kernels, from the weights it will be served (the active
    weight-norm cache's or the module's own), with ONE
    ``vits_conv1d_pack16_pairs`` launch per 48 layers instead of one
    ``vits_conv1d_pack16_pair`` launch per conv call.  The images are valid
    for this scope only (the weights change at the next optimizer step)."""
    wdt = autocast_wdtype("cuda") if HIP_TRAIN else None
    mods = []
    if PREPACK and wdt is not None and _io16(wdt):
        # (q / k / v projections come concatenated from conv1d_cat: QKV_CAT)
        skip_cat = getattr(sys.modules.get(__package__ + ".attentions"), "QKV_CAT", False)
        mods = [m for m in net.modules() if supported(m)
                and not (skip_cat and getattr(m, "_vits_cat", False))
                and any(p.is_cuda for p in m.parameters(recurse=False))]
    gates = [bool(GATE_FUSED and getattr(m, "_vits_gate", False)) for m in mods]
    if not mods:
        yield
        return
    items, arr = [], (_lib.Pack16Layer * len(mods))()
    dt = _TORCH_16[wdt]
    for i, m in enumerate(mods):
        w = weight_norm_effective(m)
        w32 = w.detach()
        if w32.dtype != torch.float32 or not w32.is_contiguous():
            w32 = w32.float().contiguous()
        cout, cin, k = w32.shape
        m_pad, cin_pad = (cout + 127) // 128 * 128, (cin + 15) // 16 * 16
        m_pad_t, cin_pad_t = (cin + 127) // 128 * 128, (cout + 15) // 16 * 16
        img = torch.empty(cin_pad // 16, k, 2, m_pad, 8, dtype=dt, device=w32.device)
        img_t = torch.empty(cin_pad_t // 16, k, 2, m_pad_t, 8, dtype=dt, device=w32.device)
        e = arr[i]
        e.w, e.cout, e.cin, e.k = w32.data_ptr(), cout, cin, k
        e.img, e.m_pad, e.cin_pad = img.data_ptr(), m_pad, cin_pad
        e.img_t, e.m_pad_t, e.cin_pad_t = img_t.data_ptr(), m_pad_t, cin_pad_t
        e.gate = int(gates[i])  # (the forward image of a fused gate conv: interleaved rows)
        items.append((m, (w, (img, img_t), wdt, gates[i]), w32))
    check(_lib.load().vits_conv1d_pack16_pairs(arr, len(mods), wdt, _stream_ptr(items[0][2].device)),
          "vits_conv1d_pack16_pairs")
    prev = {m: _PREPACK.get(m) for m, _, _ in items}
    for m, ent, _ in items:
        _PREPACK[m] = ent
    try:
        yield
    finally:
        for m, old in prev.items():
            if old is None:
                _PREPACK.pop(m, None)
            else:
                _PREPACK[m] = old


def _run(x: torch.Tensor, layer: PackedConv, n_out: int, in_slope: float = 1.0,
         gmask: torch.Tensor | None = None, gmask_slope: float = 1.0,
         io16: bool = False, res: torch.Tensor | None = None) -> torch.Tensor:
    B = x.shape[0]
    y = torch.empty(B, layer.m, n_out, device=x.device,
                    dtype=_TORCH_16[layer.wdtype] if io16 else torch.float32)
    d = make_desc(layer, x, make_out(y, res=res), in_slope=in_slope, tin=x.shape[2], n_out=n_out,
                  io16=io16)
    if gmask is not None:
        # leaky-relu derivative of the forward input, fused into the epilogue
        d.gmask, d.gmask_bstride, d.gmask_cstride = gmask.data_ptr(), gmask.stride(0), gmask.stride(1)
        d.gmask_slope = gmask_slope
    conv1d_launch(d, B, x.device)
    return y


def wgrad_buffer(cout: int, cin: int, k: int, with_bias: bool, device, zeroed: bool = True):
    """One fp32 accumulator for [k][cout][cin] dW (+ [cout] dbias)."""
    n = k * cout * cin + (cout if with_bias else 0)
    alloc = torch.zeros if zeroed else torch.empty
    return alloc(n, device=device, dtype=torch.float32)


def use_split_wgrad(cout: int, cin: int, k: int) -> bool:
    """Split-K weight gradient (partial tiles + one reduce launch, no atomics,
    deterministic, written straight into the parameter layout): faster than
    the atomic mode on every training shape measured with
    tools/wgrad_split_bench.py (8-36 %), so it is the default; the atomic
    mode stays for callers that accumulate into a buffer."""
    return k * cout * cin <= SPLIT_WGRAD_MAX


SPLIT_WGRAD_MAX = 1 << 40


def _wgrad_io16_ok(dy: torch.Tensor, x: torch.Tensor) -> bool:
    """dy and x of one 16-bit type: read as such by the weight-gradient
    kernel (8-byte block loads when aligned, element loads otherwise)."""
    return dy.dtype == x.dtype and dy.dtype in (torch.float16, torch.bfloat16)


def wgrad(dy: torch.Tensor, x: torch.Tensor, k: int, dil: int, pad_left: int,
          in_slope: float = 1.0, with_bias: bool = True, wdtype: int = TRAIN_WDTYPE,
          buf: torch.Tensor | None = None, split: bool | None = None):
    """dW [Cout, Cin, k] and dbias [Cout] (fp32) of y = conv1d(act(x), W) + b.
    ``buf``: a zeroed wgrad_buffer (atomic mode; else one is allocated).
    ``split``: split-K mode (default: ``use_split_wgrad``).  dy / x: fp32, or
    both of the 16-bit operand type (read as such when aligned, else cast)."""
    io16 = dy.dtype != torch.float32
    if io16 and not _wgrad_io16_ok(dy, x):
        dy, x, io16 = dy.float().contiguous(), x.float().contiguous(), False
    B, cout, n_out = dy.shape
    _, cin, tin = x.shape
    assert dy.stride(2) == 1 and x.stride(2) == 1 and dy.dtype == x.dtype
    assert io16 or dy.dtype == torch.float32
    if split is None:
        split = buf is None and use_split_wgrad(cout, cin, k)
    if split:
        dw = torch.empty(cout, cin, k, device=dy.device, dtype=torch.float32)
        db = torch.empty(cout, device=dy.device, dtype=torch.float32) if with_bias else None
        d = _wgrad_desc(dy, x, k, dil, pad_left, in_slope, dw, db, wdtype)
        d.io16 = int(io16)
        lib = _lib.load()
        nws = int(lib.vits_conv1d_wgrad_workspace(d, B))
        ws = torch.empty(max(nws, 1), device=dy.device, dtype=torch.float32)
        check(lib.vits_conv1d_wgrad_split(d, B, ws.data_ptr(), nws, _stream_ptr(dy.device)),
              "vits_conv1d_wgrad_split")
        return dw, db
    if buf is None:
        buf = wgrad_buffer(cout, cin, k, with_bias, dy.device)
    dw_t = buf[:k * cout * cin].view(k, cout, cin)
    db = buf[k * cout * cin:] if with_bias else None
    d = _wgrad_desc(dy, x, k, dil, pad_left, in_slope, dw_t, db, wdtype)
    d.io16 = int(io16)
    check(_lib.load().vits_conv1d_wgrad(d, B, _stream_ptr(dy.device)), "vits_conv1d_wgrad")
    if k == 1:  # [1][cout][cin] is already the parameter layout
        return dw_t.view(cout, cin, 1), db
    return dw_t.permute(1, 2, 0).contiguous(), db


def _wgrad_desc(dy, x, k, dil, pad_left, in_slope, dw, db, wdtype):
    cout, n_out = dy.shape[1], dy.shape[2]
    cin, tin = x.shape[1], x.shape[2]
    d = ConvWgradDesc()
    d.dy, d.dy_bstride, d.dy_cstride, d.cout = dy.data_ptr(), dy.stride(0), dy.stride(1), cout
    d.x, d.x_bstride, d.x_cstride, d.cin = x.data_ptr(), x.stride(0), x.stride(1), cin
    d.tin, d.n_out, d.k, d.dil, d.pad_left = tin, n_out, k, dil, pad_left
    d.in_slope = in_slope
    d.dw_t = dw.data_ptr()
    d.dbias = None if db is None else db.data_ptr()
    d.wdtype = wdtype
    return d


class Conv1dHip(torch.autograd.Function):
    """y = conv1d(leaky_relu(x, in_slope), weight, bias, dilation, padding),
    stride 1, zero padding, fp32 in/out, 16-bit MFMA operands."""

    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda", cast_inputs=torch.float32)
    def forward(ctx, x, weight, bias, dilation: int, padding: int, in_slope: float, wdtype: int):
        x = x.contiguous()
        w32 = weight.detach().contiguous()
        k = w32.shape[2]
        n_out = x.shape[2] + 2 * padding - (k - 1) * dilation
        b32 = None if bias is None else bias.detach().contiguous()
        if ctx.needs_input_grad[0]:
            # the backward's input-gradient image is packed in the same launch
            layer, layer_t = _pack16_pair(w32, dilation, padding, wdtype, b32, n_out, x.shape[2])
            ctx.layer_t = layer_t
        else:
            layer = _pack16(w32, False, dilation, padding, wdtype, b32, n_out=n_out)
            ctx.layer_t = None
        y = _run(x, layer, n_out, in_slope)
        ctx.save_for_backward(x, w32)
        ctx.conf = (dilation, padding, in_slope, wdtype, bias is not None)
        return y

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, dy):
        x, w32 = ctx.saved_tensors
        dil, pad, slope, wdtype, has_bias = ctx.conf
        k = w32.shape[2]
        dy = dy.to(torch.float32).contiguous()
        dx = dw = db = buf = None
        cout, cin = w32.shape[0], w32.shape[1]
        want_w = ctx.needs_input_grad[1] or (has_bias and ctx.needs_input_grad[2])
        split = use_split_wgrad(cout, cin, k)
        if ctx.needs_input_grad[0]:
            # the atomic weight-gradient accumulator is cleared by the packing launch
            if want_w and not split:
                buf = wgrad_buffer(cout, cin, k, has_bias, dy.device, zeroed=False)
            layer_t = ctx.layer_t
            if layer_t is None or buf is not None:
                layer_t = _pack16(w32, True, dil, (k - 1) * dil - pad, wdtype, zero=buf,
                                  n_out=x.shape[2])
            ctx.layer_t = None
            dx = _run(dy, layer_t, x.shape[2], gmask=x if slope != 1.0 else None,
                      gmask_slope=slope)
        if want_w:
            dw, db = wgrad(dy, x, k, dil, pad, slope, with_bias=has_bias, wdtype=wdtype, buf=buf,
                           split=split)
        return dx, dw, db, None, None, None, None


class GateHip(torch.autograd.Function):
    """tanh(x[:, :H] + g[:, :H, None]) * sigmoid(x[:, H:] + g[:, H:, None])
    (WN modules.py:139-146, ResBlock2 modules.py:253-255); g optional."""

    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda", cast_inputs=torch.float32)
    def forward(ctx, x, g):
        B, C2, T = x.shape
        H = C2 // 2
        if x.stride(2) != 1:
            x = x.contiguous()
        if g is not None and g.stride(1) != 1:
            g = g.contiguous()
        y = torch.empty(B, H, T, device=x.device, dtype=torch.float32)
        check(_lib.load().vits_gate_forward(
            x.data_ptr(), x.stride(0), x.stride(1), None if g is None else g.data_ptr(),
            0 if g is None else g.stride(0), y.data_ptr(), y.stride(0), y.stride(1), B, H, T,
            _stream_ptr(x.device)), "vits_gate_forward")
        ctx.save_for_backward(x, g)
        return y

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, dy):
        x, g = ctx.saved_tensors
        B, C2, T = x.shape
        H = C2 // 2
        dy = dy.to(torch.float32)
        if dy.stride(2) != 1:
            dy = dy.contiguous()
        dx = torch.empty(B, C2, T, device=x.device, dtype=torch.float32)
        want_dg = g is not None and ctx.needs_input_grad[1]
        dg = torch.empty(B, C2, device=x.device, dtype=torch.float32) if want_dg else None
        check(_lib.load().vits_gate_backward(
            dy.data_ptr(), dy.stride(0), dy.stride(1), x.data_ptr(), x.stride(0), x.stride(1),
            None if g is None else g.data_ptr(), 0 if g is None else g.stride(0), dx.data_ptr(),
            dx.stride(0), dx.stride(1), None if dg is None else dg.data_ptr(), B, H, T,
            _stream_ptr(x.device)), "vits_gate_backward")
        return dx, dg


def _pack32(w32: torch.Tensor, dil: int, pad_left: int, bias=None, gate: bool = False,
            transpose: bool = False) -> PackedConv:
    """fp32 image of a [cout, cin, k] weight for the fp32 training convs: the
    inference packing (ops.pack_conv) in the engine's fp32 arithmetic
    (engine.FP32_WDTYPE: split fp32 - three exact bf16 planes - on >= 64-row
    layers, exact fp32 otherwise).  transpose: the input-gradient image (rows
    cin, channels cout, taps reversed, pad' = (k-1)*dil - pad)."""
    _trace_pack("pack32", w32.shape)
    k = w32.shape[2]
    if transpose:
        w32 = w32.transpose(0, 1).flip(2)
        pad_left = (k - 1) * dil - pad_left
    layer = pack_conv(w32, bias, dilation=dil, padding=pad_left, gate=gate)
    return to_lowp(layer, engine.FP32_WDTYPE)


class Conv1dHip32(torch.autograd.Function):
    """y = conv1d(leaky_relu(x, in_slope), weight, bias, dilation, padding)
    (+ res) in fp32 training (autocast off): fp32 activations and weights,
    fp32 arithmetic throughout.  Forward and input gradient run the
    inference path's fp32 conv (split fp32 / exact fp32 MFMA, leaky-relu
    prologue and its derivative fused as in Conv1dHip16), the weight / bias
    gradient the exact-fp32 MFMA split-K kernel (vits_conv1d_wgrad_split,
    VITS_WDT_F32)."""

    @staticmethod
    def forward(ctx, x, weight, bias, dilation: int, padding: int, in_slope: float, res=None):
        if x.stride(2) != 1:
            x = x.contiguous()
        w32 = weight.detach().float().contiguous()
        k = w32.shape[2]
        n_out = x.shape[2] + 2 * padding - (k - 1) * dilation
        b32 = None if bias is None else bias.detach().float().contiguous()
        layer = _pack32(w32, dilation, padding, b32)
        ctx.layer_t = (_pack32(w32, dilation, padding, transpose=True)
                       if ctx.needs_input_grad[0] else None)
        if res is not None:
            assert res.dtype == torch.float32 and res.shape == (x.shape[0], w32.shape[0], n_out)
            if res.stride(2) != 1:
                res = res.contiguous()
        y = _run(x, layer, n_out, in_slope, res=res)
        ctx.save_for_backward(x, w32)
        ctx.conf = (dilation, padding, in_slope, bias is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w32 = ctx.saved_tensors
        dil, pad, slope, has_bias = ctx.conf
        k = w32.shape[2]
        dy = dy.float()
        if dy.stride(2) != 1:
            dy = dy.contiguous()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = _run(dy, ctx.layer_t, x.shape[2], gmask=x if slope != 1.0 else None,
                      gmask_slope=slope)
        ctx.layer_t = None
        if ctx.needs_input_grad[1] or (has_bias and ctx.needs_input_grad[2]):
            dw, db = wgrad(dy, x, k, dil, pad, slope, with_bias=has_bias, wdtype=WDT_F32,
                           split=True)
        dres = dy if (len(ctx.needs_input_grad) > 6 and ctx.needs_input_grad[6]) else None
        return dx, dw, db, None, None, None, dres


class ConvGateHip32(torch.autograd.Function):
    """ConvGateHip16 in fp32 training: acts = tanh(xin_a + g_a) *
    sigmoid(xin_b + g_b), xin = conv1d(leaky_relu(x, in_slope), W) + b, one
    conv launch (GATE epilogue on gate-interleaved rows, the pre-activation
    xin written for the backward); backward: the fp32 gate backward kernel
    (dxin, the cond gradient summed over time), then Conv1dHip32's input /
    weight gradient kernels.  All fp32."""

    @staticmethod
    def forward(ctx, x, weight, bias, g, dilation: int, padding: int, in_slope: float):
        if x.stride(2) != 1:
            x = x.contiguous()
        B, _, T = x.shape
        w32 = weight.detach().float().contiguous()
        cout, cin, k = w32.shape
        H = cout // 2
        n_out = T + 2 * padding - (k - 1) * dilation
        b32 = None if bias is None else bias.detach().float().contiguous()
        layer = _pack32(w32, dilation, padding, b32, gate=True)
        ctx.layer_t = (_pack32(w32, dilation, padding, transpose=True)
                       if ctx.needs_input_grad[0] else None)
        acts = torch.empty(B, H, n_out, device=x.device, dtype=torch.float32)
        xin = torch.empty(B, cout, n_out, device=x.device, dtype=torch.float32)
        cond = None
        if g is not None:
            cond = g.detach()
            if cond.dim() == 3:
                cond = cond[:, :, 0]
            if cond.stride(1) != 1:
                cond = cond.contiguous()
        d = make_desc(layer, x, make_out(acts), out1=make_out(xin), in_slope=in_slope, tin=T,
                      n_out=n_out, cond=cond)
        conv1d_launch(d, B, x.device)
        ctx.g_shape = None if g is None else tuple(g.shape)
        ctx.save_for_backward(x, w32, xin, cond)
        ctx.conf = (dilation, padding, in_slope, bias is not None)
        return acts

    @staticmethod
    def backward(ctx, dacts):
        x, w32, xin, g = ctx.saved_tensors
        dil, pad, slope, has_bias = ctx.conf
        B, C2, T = xin.shape
        H = C2 // 2
        k = w32.shape[2]
        dacts = dacts.float()
        if dacts.stride(2) != 1:
            dacts = dacts.contiguous()
        dxin = torch.empty(B, C2, T, device=xin.device, dtype=torch.float32)
        want_dg = g is not None and ctx.needs_input_grad[3]
        dg = torch.empty(B, C2, device=xin.device, dtype=torch.float32) if want_dg else None
        check(_lib.load().vits_gate_backward(
            dacts.data_ptr(), dacts.stride(0), dacts.stride(1), xin.data_ptr(), xin.stride(0),
            xin.stride(1), None if g is None else g.data_ptr(), 0 if g is None else g.stride(0),
            dxin.data_ptr(), dxin.stride(0), dxin.stride(1), None if dg is None else dg.data_ptr(),
            B, H, T, _stream_ptr(xin.device)), "vits_gate_backward")
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = _run(dxin, ctx.layer_t, x.shape[2], gmask=x if slope != 1.0 else None,
                      gmask_slope=slope)
        ctx.layer_t = None
        if ctx.needs_input_grad[1] or (has_bias and ctx.needs_input_grad[2]):
            dw, db = wgrad(dxin, x, k, dil, pad, slope, with_bias=has_bias, wdtype=WDT_F32,
                           split=True)
        if dg is not None and len(ctx.g_shape) == 3:
            dg = dg.unsqueeze(-1)
        return dx, dw, db, dg, None, None, None


class Conv1dHip16(torch.autograd.Function):
    """Conv1dHip with 16-bit activations: x, y, dY and dX are tensors of the
    operand type (fp16 under the reference's fp16 autocast, whose convs
    return fp16), read and written as such by the kernels (io16); W and b
    stay fp32 masters (packed to 16 bits per call), dW / db fp32."""

    @staticmethod
    def forward(ctx, x, weight, bias, dilation: int, padding: int, in_slope: float, wdtype: int,
                res=None, pre=None):
        """res (optional, fp16 [B, Cout, n_out]): y = res + conv, the
        residual add of ResBlock2 (modules.py:258-259) in the epilogue.
        pre (optional): (img, img_t) of ``weight`` already packed by
        ``prepacked`` (one launch for the whole network)."""
        if x.stride(2) != 1:
            x = x.contiguous()
        w32 = weight.detach().float().contiguous()
        k = w32.shape[2]
        n_out = x.shape[2] + 2 * padding - (k - 1) * dilation
        b32 = None if bias is None else bias.detach().float().contiguous()
        if pre is not None:
            layer, layer_t = _layers16(pre, w32.shape, dilation, padding, wdtype, b32, n_out,
                                       x.shape[2])
            ctx.layer_t = layer_t
        elif ctx.needs_input_grad[0]:
            layer, layer_t = _pack16_pair(w32, dilation, padding, wdtype, b32, n_out, x.shape[2],
                                          io16=True)
            ctx.layer_t = layer_t
        else:
            layer = _pack16(w32, False, dilation, padding, wdtype, b32, n_out=n_out, io16=True)
            ctx.layer_t = None
        if res is not None:
            assert res.dtype == x.dtype and res.shape == (x.shape[0], layer.m, n_out)
            if res.stride(2) != 1:
                res = res.contiguous()
        y = _run(x, layer, n_out, in_slope, io16=True, res=res)
        ctx.save_for_backward(x, w32)
        ctx.conf = (dilation, padding, in_slope, wdtype, bias is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w32 = ctx.saved_tensors
        dil, pad, slope, wdtype, has_bias = ctx.conf
        k = w32.shape[2]
        dy = dy.to(x.dtype)
        if dy.stride(2) != 1:
            dy = dy.contiguous()
        dx = dw = db = None
        want_w = ctx.needs_input_grad[1] or (has_bias and ctx.needs_input_grad[2])
        if ctx.needs_input_grad[0]:
            layer_t = ctx.layer_t
            if layer_t is None:
                layer_t = _pack16(w32, True, dil, (k - 1) * dil - pad, wdtype, n_out=x.shape[2],
                                  io16=True)
            ctx.layer_t = None
            dx = _run(dy, layer_t, x.shape[2], gmask=x if slope != 1.0 else None,
                      gmask_slope=slope, io16=True)
        if want_w:
            dw, db = wgrad(dy, x, k, dil, pad, slope, with_bias=has_bias, wdtype=wdtype,
                           split=True)
        grads = [dx, dw, db, None, None, None, None]
        if len(ctx.needs_input_grad) > 7:  # the residual argument
            grads.append(dy if ctx.needs_input_grad[7] else None)
        grads += [None] * (len(ctx.needs_input_grad) - len(grads))
        return tuple(grads)


class GateHip16(torch.autograd.Function):
    """GateHip on 16-bit activations (x, g, y, dY, dX of the operand type;
    the cond gradient is summed in fp32 and returned in g's type)."""

    @staticmethod
    def forward(ctx, x, g, wdtype: int):
        B, C2, T = x.shape
        H = C2 // 2
        if x.stride(2) != 1:
            x = x.contiguous()
        if g is not None and g.stride(1) != 1:
            g = g.contiguous()
        y = torch.empty(B, H, T, device=x.device, dtype=x.dtype)
        check(_lib.load().vits_gate_forward_io16(
            x.data_ptr(), x.stride(0), x.stride(1), None if g is None else g.data_ptr(),
            0 if g is None else g.stride(0), y.data_ptr(), y.stride(0), y.stride(1), B, H, T,
            wdtype, _stream_ptr(x.device)), "vits_gate_forward_io16")
        ctx.save_for_backward(x, g)
        ctx.wdtype = wdtype
        return y

    @staticmethod
    def backward(ctx, dy):
        x, g = ctx.saved_tensors
        B, C2, T = x.shape
        H = C2 // 2
        dy = dy.to(x.dtype)
        if dy.stride(2) != 1:
            dy = dy.contiguous()
        dx = torch.empty(B, C2, T, device=x.device, dtype=x.dtype)
        want_dg = g is not None and ctx.needs_input_grad[1]
        dg = torch.empty(B, C2, device=x.device, dtype=torch.float32) if want_dg else None
        check(_lib.load().vits_gate_backward_io16(
            dy.data_ptr(), dy.stride(0), dy.stride(1), x.data_ptr(), x.stride(0), x.stride(1),
            None if g is None else g.data_ptr(), 0 if g is None else g.stride(0), dx.data_ptr(),
            dx.stride(0), dx.stride(1), None if dg is None else dg.data_ptr(), B, H, T,
            ctx.wdtype, _stream_ptr(x.device)), "vits_gate_backward_io16")
        return dx, (None if dg is None else dg.to(g.dtype)), None


class WNUpdate16(torch.autograd.Function):
    """x' = (x + rs[:, :H]) * mask, x16' = x' in the 16-bit type, out' = out +
    rs[:, H:] (modules.WN between two layers, modules.py:93-182) - one
    kernel each way (csrc/wnres.hip).  out may be None (= 0)."""

    @staticmethod
    def forward(ctx, x, rs, mask, out, wdtype: int):
        B, H, T = x.shape
        assert rs.shape == (B, 2 * H, T) and mask.shape == (B, 1, T)
        xn = torch.empty_like(x)
        x16 = torch.empty(B, H, T, device=x.device, dtype=rs.dtype)
        outn = torch.empty_like(x)
        check(_lib.load().vits_wn_update_forward(
            x.data_ptr(), rs.data_ptr(), mask.data_ptr(), None if out is None else out.data_ptr(),
            xn.data_ptr(), x16.data_ptr(), outn.data_ptr(), B, H, T, wdtype,
            _stream_ptr(x.device)), "vits_wn_update_forward")
        ctx.save_for_backward(mask)
        ctx.conf = (B, H, T, wdtype, rs.dtype, out is not None)
        ctx.set_materialize_grads(False)
        return xn, x16, outn

    @staticmethod
    def backward(ctx, gxn, gx16, gout):
        (mask,) = ctx.saved_tensors
        B, H, T, wdtype, dt, has_out = ctx.conf
        dx = torch.empty(B, H, T, device=mask.device, dtype=torch.float32)
        drs = torch.empty(B, 2 * H, T, device=mask.device, dtype=dt)
        gxn = None if gxn is None else gxn.contiguous()
        gx16 = None if gx16 is None else gx16.to(dt).contiguous()
        gout = None if gout is None else gout.float().contiguous()
        check(_lib.load().vits_wn_update_backward(
            None if gxn is None else gxn.data_ptr(), None if gx16 is None else gx16.data_ptr(),
            None if gout is None else gout.data_ptr(), mask.data_ptr(), dx.data_ptr(),
            drs.data_ptr(), B, H, T, wdtype, _stream_ptr(mask.device)), "vits_wn_update_backward")
        return dx, drs, None, (gout if has_out else None), None


def wn_update(x: torch.Tensor, rs: torch.Tensor, mask: torch.Tensor, out):
    """(x', x16', out') of WN's residual / skip update (WNUpdate16) when it
    applies: an fp16-autocast training step on the GPU, fp32 contiguous x /
    out / mask and a 16-bit rs; None otherwise (the caller runs torch)."""
    wdt = train_wdtype(x)
    if (wdt is None or not _io16(wdt) or rs.dtype != _TORCH_16[wdt] or x.dtype != torch.float32
            or mask.dtype != torch.float32 or (out is not None and out.dtype != torch.float32)):
        return None
    # (a strided x - the PosteriorEncoder's pre-conv output - is copied once
    # here; the fused update's outputs are contiguous from then on)
    return WNUpdate16.apply(x.contiguous(), rs.contiguous(), mask.contiguous(),
                            None if out is None else out.contiguous(), wdt)


def _coupling_ok(wdt, *tensors16) -> bool:
    return (wdt is not None and _io16(wdt) and COUPLING_FUSED
            and all(t.dtype == _TORCH_16[wdt] for t in tensors16))


# the coupling layers' element-wise glue on wnres.hip (mask_cast, wn_final,
# coupling); False: the reference's torch ops
COUPLING_FUSED = True


def _mask_ok(mask: torch.Tensor, B: int, T: int) -> bool:
    return (mask.dtype == torch.float32 and mask.is_contiguous()
            and tuple(mask.shape) == (B, 1, T))


class MaskCast16(torch.autograd.Function):
    """(y * mask, the same rounded to the 16-bit type) for a 16-bit conv
    output y and an fp32 mask - the coupling's ``pre(x0) * x_mask`` and the
    WN's first in_layer input (csrc/wnres.hip mask_cast)."""

    @staticmethod
    def forward(ctx, y, mask, wdtype: int):
        B, C, T = y.shape
        y = y.contiguous()
        h = torch.empty(B, C, T, device=y.device, dtype=torch.float32)
        h16 = torch.empty_like(y)
        check(_lib.load().vits_mask_cast_forward(
            y.data_ptr(), mask.data_ptr(), h.data_ptr(), h16.data_ptr(), B, C, T, wdtype,
            _stream_ptr(y.device)), "vits_mask_cast_forward")
        ctx.save_for_backward(mask)
        ctx.conf = (B, C, T, wdtype, y.dtype)
        ctx.set_materialize_grads(False)
        return h, h16

    @staticmethod
    def backward(ctx, gh, gh16):
        (mask,) = ctx.saved_tensors
        B, C, T, wdtype, dt = ctx.conf
        dy = torch.empty(B, C, T, device=mask.device, dtype=dt)
        gh = None if gh is None else gh.float().contiguous()
        gh16 = None if gh16 is None else gh16.to(dt).contiguous()
        check(_lib.load().vits_mask_cast_backward(
            None if gh is None else gh.data_ptr(), None if gh16 is None else gh16.data_ptr(),
            mask.data_ptr(), dy.data_ptr(), B, C, T, wdtype, _stream_ptr(mask.device)),
            "vits_mask_cast_backward")
        return dy, None, None


def mask_cast(y: torch.Tensor, mask: torch.Tensor):
    """(y * mask fp32, its 16-bit copy) on the fused path, else None."""
    wdt = train_wdtype(y)
    if not (_coupling_ok(wdt, y) and _mask_ok(mask, y.shape[0], y.shape[2])):
        return None
    return MaskCast16.apply(y, mask, wdt)


class WNFinal16(torch.autograd.Function):
    """16-bit((out + rs) * mask): the WN output (modules.py:182) for a
    consumer that feeds it to an autocast conv (csrc/wnres.hip wn_final)."""

    @staticmethod
    def forward(ctx, out, rs, mask, wdtype: int):
        B, C, T = rs.shape
        rs = rs.contiguous()
        o16 = torch.empty_like(rs)
        check(_lib.load().vits_wn_final_forward(
            None if out is None else out.data_ptr(), rs.data_ptr(), mask.data_ptr(),
            o16.data_ptr(), B, C, T, wdtype, _stream_ptr(rs.device)), "vits_wn_final_forward")
        ctx.save_for_backward(mask)
        ctx.conf = (B, C, T, wdtype, rs.dtype, out is not None)
        return o16

    @staticmethod
    def backward(ctx, g16):
        (mask,) = ctx.saved_tensors
        B, C, T, wdtype, dt, has_out = ctx.conf
        g16 = g16.to(dt).contiguous()
        dout = (torch.empty(B, C, T, device=mask.device, dtype=torch.float32)
                if has_out and ctx.needs_input_grad[0] else None)
        drs = torch.empty(B, C, T, device=mask.device, dtype=dt)
        check(_lib.load().vits_wn_final_backward(
            g16.data_ptr(), mask.data_ptr(), None if dout is None else dout.data_ptr(),
            drs.data_ptr(), B, C, T, wdtype, _stream_ptr(mask.device)), "vits_wn_final_backward")
        return dout, drs, None, None


def wn_final(out, rs: torch.Tensor, mask: torch.Tensor):
    """16-bit((out + rs) * mask) on the fused path (out fp32 or None), else
    None."""
    wdt = train_wdtype(rs)
    if not (_coupling_ok(wdt, rs) and _mask_ok(mask, rs.shape[0], rs.shape[2])):
        return None
    if out is not None:
        if out.dtype != torch.float32 or out.shape != rs.shape:
            return None
        out = out.contiguous()
    return WNFinal16.apply(out, rs, mask, wdt)


class Coupling16(torch.autograd.Function):
    """The mean-only coupling update (modules.py:352-360 with logs = 0):
    cat(x0, m + x1 * mask) forward, cat(x0, (x1 - m) * mask) reverse, m =
    p * mask for the 16-bit post-conv output p; optionally channel-flipped
    (the Flip that follows, models.py:219-235).  csrc/wnres.hip coupling."""

    @staticmethod
    def forward(ctx, x, p, mask, reverse: bool, flip: bool, wdtype: int):
        B, C2, T = x.shape
        half = C2 // 2
        x = x.contiguous()
        p = p.contiguous()
        out = torch.empty_like(x)
        check(_lib.load().vits_coupling_forward(
            x.data_ptr(), p.data_ptr(), mask.data_ptr(), out.data_ptr(), B, half, T, int(reverse),
            int(flip), wdtype, _stream_ptr(x.device)), "vits_coupling_forward")
        ctx.save_for_backward(mask)
        ctx.conf = (B, half, T, int(reverse), int(flip), wdtype, p.dtype)
        return out

    @staticmethod
    def backward(ctx, g):
        (mask,) = ctx.saved_tensors
        B, half, T, reverse, flip, wdtype, dt = ctx.conf
        g = g.float().contiguous()
        gx = torch.empty(B, 2 * half, T, device=g.device, dtype=torch.float32)
        gp = torch.empty(B, half, T, device=g.device, dtype=dt)
        check(_lib.load().vits_coupling_backward(
            g.data_ptr(), mask.data_ptr(), gx.data_ptr(), gp.data_ptr(), B, half, T, reverse, flip,
            wdtype, _stream_ptr(g.device)), "vits_coupling_backward")
        return gx, gp, None, None, None, None


def coupling_fused_ok(x: torch.Tensor, mask: torch.Tensor) -> bool:
    """Whether a coupling on x (fp32 [B, 2h, T]) takes the fused path."""
    wdt = train_wdtype(x)
    return (_coupling_ok(wdt) and x.dtype == torch.float32 and x.dim() == 3
            and _mask_ok(mask, x.shape[0], x.shape[2]))


def coupling_update(x: torch.Tensor, p: torch.Tensor, mask: torch.Tensor, reverse: bool,
                    flip: bool):
    """Coupling16 on the fused path (x fp32 [B, 2h, T], p 16-bit [B, h, T]),
    else None."""
    wdt = train_wdtype(x)
    if not (_coupling_ok(wdt, p) and x.dtype == torch.float32
            and _mask_ok(mask, x.shape[0], x.shape[2])
            and tuple(p.shape) == (x.shape[0], x.shape[1] // 2, x.shape[2])):
        return None
    return Coupling16.apply(x, p, mask, reverse, flip, wdt)


# 16-bit activations for the training convs / gates under fp16 autocast (the
# reference's autocast convs return fp16); False: the fp32-I/O kernels
TRAIN_IO16 = True


def _io16(wdt) -> bool:
    return TRAIN_IO16 and wdt == WDT_F16


def conv1d_hip(x: torch.Tensor, w: torch.Tensor, bias, dilation: int, padding: int,
               in_slope: float, wdt: int, residual: torch.Tensor | None = None,
               pre=None) -> torch.Tensor:
    """The HIP training conv of operand type ``wdt`` (+ ``residual``): 16-bit
    activations (Conv1dHip16; x cast to fp16 first, as autocast casts a
    conv's input; the residual added in the epilogue), fp32 training
    (WDT_F32: Conv1dHip32, fp32 arithmetic, the residual in the epilogue)
    or fp32 activations with 16-bit operands (Conv1dHip).  ``pre``: the
    weight's prepacked images (``prepacked``)."""
    if _io16(wdt):
        t16 = _TORCH_16[wdt]
        x16 = x if x.dtype == t16 else x.to(t16)
        if residual is not None and residual.dtype != t16:
            # an fp32 residual stream keeps the reference's fp32 add
            return Conv1dHip16.apply(x16, w, bias, dilation, padding, in_slope, wdt,
                                     None, pre) + residual
        return Conv1dHip16.apply(x16, w, bias, dilation, padding, in_slope, wdt, residual, pre)
    if wdt == WDT_F32:
        res = None if residual is None else residual.float()
        return Conv1dHip32.apply(x.float(), w, bias, dilation, padding, in_slope, res)
    y = Conv1dHip.apply(x, w, bias, dilation, padding, in_slope, wdt)
    return y if residual is None else y + residual


def gate(x: torch.Tensor, g) -> torch.Tensor:
    """The WN / ResBlock2 gate: the HIP op on a ROCm device (16-bit under
    fp16 autocast, fp32 in fp32 training; the convs around it are HIP too),
    torch on CPU / with HIP_TRAIN off."""
    wdt = train_wdtype(x)
    if wdt is not None and _io16(wdt) and x.dtype == _TORCH_16[wdt]:
        g16 = None if g is None else g.to(x.dtype)
        return GateHip16.apply(x, g16, wdt)
    if wdt is not None:
        return GateHip.apply(x, g)
    H = x.shape[1] // 2
    if g is not None:
        x = x + g.unsqueeze(-1)
    return torch.tanh(x[:, :H]) * torch.sigmoid(x[:, H:])


def supported(module: nn.Module) -> bool:
    return (isinstance(module, nn.Conv1d) and module.stride == (1,) and module.groups == 1
            and module.padding_mode == "zeros" and not isinstance(module.padding, str)
            and _lib_k_ok(module.kernel_size[0], module.dilation[0]))


def _lib_k_ok(k: int, dil: int) -> bool:
    return k in (1, 2, 3, 4, 5, 7, 9, 11) and 64 + (k - 1) * dil <= 128


def autocast_wdtype(device_type: str = "cuda"):
    """MFMA operand type of the enclosing autocast region (fp16 -> WDT_F16,
    bf16 -> WDT_BF16), or None when autocast is off."""
    if not torch.is_autocast_enabled(device_type):
        return None
    dt = torch.get_autocast_dtype(device_type)
    return {torch.float16: WDT_F16, torch.bfloat16: WDT_BF16}.get(dt)


# test switch: False runs every training conv / gate on torch (the
# reference's own arithmetic, MIOpen) on the same device
HIP_TRAIN = True


def train_wdtype(x: torch.Tensor):
    """Operand type of the HIP training kernels for an op on ``x``: the
    autocast dtype inside a 16-bit autocast region, WDT_F32 in fp32
    training (autocast off: the reference's fp16_run = false), None on CPU,
    under another autocast dtype, or with HIP_TRAIN off (torch path)."""
    if not HIP_TRAIN or x.device.type != "cuda":
        return None
    wdt = autocast_wdtype("cuda")
    if wdt is not None:
        return wdt
    return None if torch.is_autocast_enabled("cuda") else WDT_F32


def module_weight(module: nn.Module) -> torch.Tensor:
    """A layer's effective weight: the active weight-norm cache's, or the
    weight-norm / plain weight computed here."""
    w = cached_weight(module)
    return w if w is not None else weight_norm_effective(module)


def linear(module: nn.Module, x: torch.Tensor) -> torch.Tensor:
    """``module(x)`` for an nn.Linear / 1x1 nn.Conv1d (the conditioning
    layers, modules.py:76,120), with the weight of the active weight-norm
    cache (wnorm.WeightNormCache) when there is one; the module's own
    (hooked) forward otherwise."""
    w = cached_weight(module)
    if w is None:
        return module(x)
    if isinstance(module, nn.Conv1d):
        return F.conv1d(x, w, module.bias, module.stride, module.padding, module.dilation,
                        module.groups)
    return F.linear(x, w, module.bias)


def conv1d(module: nn.Module, x: torch.Tensor, in_slope: float = 1.0,
           residual: torch.Tensor | None = None) -> torch.Tensor:
    """``module(leaky_relu(x, in_slope)) (+ residual)`` for an nn.Conv1d
    (optionally legacy-weight-normed or spectral-normed).

    Inside a 16-bit autocast region on a ROCm device (the reference's
    ``fp16_run`` training, train_stft.py:165,216) this is the HIP training
    conv with operands of the autocast dtype.  Outside autocast the reference
    computes the conv in fp32, and so does this: the fp32 HIP training conv
    (Conv1dHip32).  On CPU it is the torch conv."""
    wdt = train_wdtype(x)
    if wdt is None or not supported(module):
        if in_slope != 1.0:
            x = F.leaky_relu(x, in_slope)
        return module(x) if residual is None else module(x) + residual
    w = weight_norm_effective(module)
    ent = _PREPACK.get(module)
    pre = ent[1] if (ent is not None and ent[0] is w and ent[2] == wdt and not ent[3]) else None
    return conv1d_hip(x, w, module.bias, module.dilation[0], module.padding[0], in_slope, wdt,
                      residual, pre)


def conv1d_cat(modules, x: torch.Tensor):
    """[m(x) for m in modules] for convs of one input and one geometry (the
    self-attention q / k / v projections, attentions.py:85-87) as ONE HIP
    conv over their concatenated weight rows: one forward, one input-
    gradient conv (the three gradients' sum comes out of a single K = 3C
    GEMM - no adds) and one weight gradient instead of three each.  Returns
    the outputs as channel slices of one [B, sum(C_out), T] tensor, or None
    where conv1d would not run the modules on the HIP kernels."""
    wdt = train_wdtype(x)
    m0 = modules[0]
    if (wdt is None or not (_io16(wdt) or wdt == WDT_F32) or not all(supported(m) for m in modules)
            or any(m.kernel_size != m0.kernel_size or m.dilation != m0.dilation
                   or m.padding != m0.padding or m.in_channels != m0.in_channels
                   or (m.bias is None) != (m0.bias is None) for m in modules)):
        return None
    w = torch.cat([weight_norm_effective(m) for m in modules], 0)
    b = None if m0.bias is None else torch.cat([m.bias for m in modules], 0)
    y = conv1d_hip(x, w, b, m0.dilation[0], m0.padding[0], 1.0, wdt)
    return y.split([m.out_channels for m in modules], 1)


# ---------------------------------------------------------------------------
# ConvTranspose1d (the Generator's upsamplers, models.py:306-310) in training
# ---------------------------------------------------------------------------

_POLY_INDEX = {}


def _poly_index(K: int, u: int, p: int, device):
    """Gather map of the polyphase lowering of ConvTranspose1d(K, stride u,
    padding p): output phase r of channel o is a stride-1 conv of x with
    P + 1 taps (P = ceil(K / u)), tap i reading x[q - (P - 1 - c0) + i]:
        W_poly[o*u + r][c][i] = W[c][o][u*m + r'],
        r' = (r + p) mod u, carry = (r + p) div u, c0 = p div u,
        m = P - 1 + carry - c0 - i,
    zero where u*m + r' is not a tap of W (the carries of the phases span
    c0 .. c0 + 1, hence one extra tap).  Returns (index [u, P+1] into K,
    valid mask [u, P+1])."""
    key = (K, u, p, str(device))
    if key not in _POLY_INDEX:
        P = (K + u - 1) // u
        idx = torch.zeros(u, P + 1, dtype=torch.long)
        ok = torch.zeros(u, P + 1, dtype=torch.bool)
        c0 = p // u
        for r in range(u):
            rp, carry = (r + p) % u, (r + p) // u
            for i in range(P + 1):
                m = P - 1 + carry - c0 - i
                j = u * m + rp
                if 0 <= m < P and 0 <= j < K:
                    idx[r, i], ok[r, i] = j, True
        _POLY_INDEX[key] = (idx.to(device), ok.to(device))
    return _POLY_INDEX[key]


_POLY_PERM = {}


def _poly_perm(C: int, O: int, K: int, u: int, p: int, device):
    """Flat gather maps of the polyphase weight: fwd[e] = the index into the
    [C, O, K] weight of element e of the [O*u, C, P+1] phase image (K*C*O
    of its entries; -1 for the structural zeros), and bwd = its inverse
    (every tap of W lands in exactly one phase slot, see _poly_index), so
    the weight gradient is a plain gather too - no index_put accumulation
    (torch's advanced-index backward: a sort + 0.44 ms for ups.0)."""
    key = (C, O, K, u, p, str(device))
    if key not in _POLY_PERM:
        idx, ok = _poly_index(K, u, p, "cpu")          # [u, P+1]
        P1 = idx.shape[1]
        o = torch.arange(O).view(O, 1, 1, 1)
        r = torch.arange(u).view(1, u, 1, 1)
        c = torch.arange(C).view(1, 1, C, 1)
        i = torch.arange(P1).view(1, 1, 1, P1)
        src = (c * O + o) * K + idx[r, i]              # [O, u, C, P+1]
        fwd = torch.where(ok[r, i], src, torch.full_like(src, -1)).reshape(-1)
        bwd = torch.empty(C * O * K, dtype=torch.long)
        valid = fwd >= 0
        bwd[fwd[valid]] = torch.nonzero(valid).squeeze(1)
        assert int(valid.sum()) == C * O * K  # a bijection onto the taps
        _POLY_PERM[key] = (fwd.clamp(min=0).to(device), valid.to(device), bwd.to(device), P1)
    return _POLY_PERM[key]


class PolyphaseWeight(torch.autograd.Function):
    """W [C, O, K] of ConvTranspose1d(K, stride u, padding p) -> the phase-
    stacked stride-1 weight [O*u, C, P+1] of conv_transpose1d's lowering;
    forward and backward are one gather each."""

    @staticmethod
    def forward(ctx, w, u: int, p: int):
        C, O, K = w.shape
        fwd, valid, bwd, P1 = _poly_perm(C, O, K, u, p, w.device)
        ctx.conf = (C, O, K, u, p)
        wp = w.reshape(-1).index_select(0, fwd) * valid.to(w.dtype)
        return wp.view(O * u, C, P1)

    @staticmethod
    def backward(ctx, g):
        C, O, K, u, p = ctx.conf
        _, _, bwd, _ = _poly_perm(C, O, K, u, p, g.device)
        return g.contiguous().view(-1).index_select(0, bwd).view(C, O, K), None, None


def conv_transpose1d(module: nn.Module, x: torch.Tensor, in_slope: float = 1.0) -> torch.Tensor:
    """``module(leaky_relu(x, in_slope))`` for an nn.ConvTranspose1d
    (optionally legacy-weight-normed, output_padding 0, groups 1, dilation 1).

    On a ROCm device (fp16 autocast or fp32 training): the polyphase lowering
    on the HIP training conv - one stride-1 Conv1dHip (forward, input and
    weight gradient on MFMA) over phase-stacked weight rows, the leaky-relu
    fused as its prologue, then one interleave of the phases into time.
    The weight gradient flows back through the (differentiable) gather that
    builds the phase weights.  Elsewhere: the torch module (MIOpen / CPU)."""
    wdt = train_wdtype(x)
    ok = (isinstance(module, nn.ConvTranspose1d) and module.groups == 1
          and module.dilation == (1,) and module.output_padding == (0,)
          and module.padding_mode == "zeros")
    if wdt is None or not ok:
        if in_slope != 1.0:
            x = F.leaky_relu(x, in_slope)
        return module(x)
    u, K, p = module.stride[0], module.kernel_size[0], module.padding[0]
    P = (K + u - 1) // u
    c0 = p // u
    # conv padding P - 1 - c0 must leave >= T outputs per phase
    if (P < 2 + 2 * c0 or not _lib_k_ok(P + 1, 1)
            or (x.shape[2] - 1) * u - 2 * p + K != x.shape[2] * u):
        if in_slope != 1.0:
            x = F.leaky_relu(x, in_slope)
        return module(x)
    w = weight_norm_effective(module)                  # [C, O, K]
    C, O = w.shape[0], w.shape[1]
    wp = PolyphaseWeight.apply(w, u, p)                # [O*u, C, P+1]
    bias = None if module.bias is None else module.bias.repeat_interleave(u)
    B, _, T = x.shape
    y = conv1d_hip(x, wp, bias, 1, P - 1 - c0, in_slope, wdt)  # [B, O*u, >= T]
    # phases -> time: y[b][o*u + r][q] -> out[b][o][q*u + r]  (T_out = T*u)
    return y[:, :, :T].reshape(B, O, u, T).permute(0, 1, 3, 2).reshape(B, O, T * u)


# ---------------------------------------------------------------------------
# conv -> gate as one launch (WN modules.py:136-146, ResBlock2 modules.py:252-255)
# ---------------------------------------------------------------------------
# in_layer / convs1 convs whose output only feeds the tanh * sigmoid gate run
# the GATE epilogue (gate-interleaved weight rows) and write the
# pre-activation for the gate's backward in the same launch; False (tests)
# keeps the separate conv + GateHip16 kernels
GATE_FUSED = True


def _pack16_pair_gate(w32, wdtype):
    """(gate-interleaved forward image, natural input-gradient image) of one
    weight: vits_conv1d_pack16_pairs with gate = 1."""
    cout, cin, k = w32.shape
    dt = _TORCH_16[wdtype]
    m_pad, cin_pad = (cout + 127) // 128 * 128, (cin + 15) // 16 * 16
    m_pad_t, cin_pad_t = (cin + 127) // 128 * 128, (cout + 15) // 16 * 16
    img = torch.empty(cin_pad // 16, k, 2, m_pad, 8, dtype=dt, device=w32.device)
    img_t = torch.empty(cin_pad_t // 16, k, 2, m_pad_t, 8, dtype=dt, device=w32.device)
    arr = (_lib.Pack16Layer * 1)()
    e = arr[0]
    e.w, e.cout, e.cin, e.k = w32.data_ptr(), cout, cin, k
    e.img, e.m_pad, e.cin_pad = img.data_ptr(), m_pad, cin_pad
    e.img_t, e.m_pad_t, e.cin_pad_t = img_t.data_ptr(), m_pad_t, cin_pad_t
    e.gate = 1
    check(_lib.load().vits_conv1d_pack16_pairs(arr, 1, wdtype, _stream_ptr(w32.device)),
          "vits_conv1d_pack16_pairs")
    return img, img_t


class ConvGateHip16(torch.autograd.Function):
    """acts = tanh(xin[:, :H] + g[:, :H]) * sigmoid(xin[:, H:] + g[:, H:]),
    xin = conv1d(leaky_relu(x, in_slope), W) + b, as ONE conv launch: the
    GATE epilogue on gate-interleaved weight rows (fp32 gate arithmetic on
    the fp32 accumulator) also writes xin (fp16) for the backward.  Backward:
    the gate backward kernel (dxin, the cond gradient summed over time)
    then the conv's input / weight gradients (Conv1dHip16's kernels).
    x, g, acts, xin fp16; W / b fp32 masters."""

    @staticmethod
    def forward(ctx, x, weight, bias, g, dilation: int, padding: int, in_slope: float,
                wdtype: int, pre=None, g16=None):
        """g: the cond (fp32 or 16-bit, [B, C2(, 1)], channel stride 1); g16
        (optional, not differentiated): the same values in the operand type
        for the backward's gate kernel - WN / ResBlock2 cast their whole
        cond tensor once instead of every layer's slice twice."""
        if x.stride(2) != 1:
            x = x.contiguous()
        B, _, T = x.shape
        w32 = weight.detach().float().contiguous()
        cout, cin, k = w32.shape
        H = cout // 2
        n_out = T + 2 * padding - (k - 1) * dilation
        b32 = None if bias is None else bias.detach().float().contiguous()
        img, img_t = pre if pre is not None else _pack16_pair_gate(w32, wdtype)
        layer, layer_t = _layers16((img, img_t), w32.shape, dilation, padding, wdtype, b32, n_out,
                                   T)
        layer.epi = EPI_GATE
        acts = torch.empty(B, H, n_out, device=x.device, dtype=x.dtype)
        xin = torch.empty(B, cout, n_out, device=x.device, dtype=x.dtype)
        cond = None
        if g is not None:
            cond = g.detach()
            if cond.dtype != torch.float32 or cond.stride(1) != 1:
                cond = cond.float().contiguous()
        d = make_desc(layer, x, make_out(acts), out1=make_out(xin), in_slope=in_slope, tin=T,
                      n_out=n_out, cond=cond, io16=True)
        conv1d_launch(d, B, x.device)
        ctx.layer_t = layer_t
        ctx.g_dtype = None if g is None else g.dtype
        ctx.g_shape = None if g is None else tuple(g.shape)
        ctx.save_for_backward(x, w32, xin, g16 if g16 is not None else g)
        ctx.conf = (dilation, padding, in_slope, wdtype, bias is not None)
        return acts

    @staticmethod
    def backward(ctx, dacts):
        x, w32, xin, g = ctx.saved_tensors
        dil, pad, slope, wdtype, has_bias = ctx.conf
        B, C2, T = xin.shape
        H = C2 // 2
        k = w32.shape[2]
        dacts = dacts.to(xin.dtype)
        if dacts.stride(2) != 1:
            dacts = dacts.contiguous()
        dxin = torch.empty(B, C2, T, device=xin.device, dtype=xin.dtype)
        want_dg = g is not None and ctx.needs_input_grad[3]
        dg = torch.empty(B, C2, device=xin.device, dtype=torch.float32) if want_dg else None
        g16 = None if g is None else g.to(xin.dtype)  # (a no-op when g16 was given)
        if g16 is not None and g16.stride(1) != 1:
            g16 = g16.contiguous()
        check(_lib.load().vits_gate_backward_io16(
            dacts.data_ptr(), dacts.stride(0), dacts.stride(1), xin.data_ptr(), xin.stride(0),
            xin.stride(1), None if g16 is None else g16.data_ptr(),
            0 if g16 is None else g16.stride(0), dxin.data_ptr(), dxin.stride(0), dxin.stride(1),
            None if dg is None else dg.data_ptr(), B, H, T, wdtype, _stream_ptr(xin.device)),
            "vits_gate_backward_io16")
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = _run(dxin, ctx.layer_t, x.shape[2], gmask=x if slope != 1.0 else None,
                      gmask_slope=slope, io16=True)
        ctx.layer_t = None
        if ctx.needs_input_grad[1] or (has_bias and ctx.needs_input_grad[2]):
            dw, db = wgrad(dxin, x, k, dil, pad, slope, with_bias=has_bias, wdtype=wdtype,
                           split=True)
        if dg is not None:
            dg = dg.to(ctx.g_dtype)
            if len(ctx.g_shape) == 3:
                dg = dg.unsqueeze(-1)
        return (dx, dw, db, dg, None, None, None, None, None, None)


COND_F32 = True


class _SplitCols(torch.autograd.Function):
    """x[:, i*w:(i+1)*w] for i < n as views; the backward concatenates the n
    column gradients in ONE launch (n slice backwards would each allocate a
    zero tensor of x's size, copy into it and add: 3n - 1 launches)."""

    @staticmethod
    def forward(ctx, x, n: int, w: int):
        ctx.shape, ctx.dtype = x.shape, x.dtype
        ctx.set_materialize_grads(False)
        return tuple(x[:, i * w:(i + 1) * w] for i in range(n))

    @staticmethod
    def backward(ctx, *gs):
        B = ctx.shape[0]
        w = ctx.shape[1] // len(gs)
        parts = [g if g is not None else
                 torch.zeros(B, w, device=next(t for t in gs if t is not None).device,
                             dtype=ctx.dtype) for g in gs]
        return torch.cat(parts, 1), None, None


def split_cols(x: torch.Tensor, n: int, w: int):
    """The n column blocks of width w of x [B, n * w] (the per-layer cond
    slices of modules.WN, modules.py:141-142), with a one-launch backward."""
    if not x.requires_grad or x.shape[1] != n * w:
        return [x[:, i * w:(i + 1) * w] for i in range(n)]
    return list(_SplitCols.apply(x, n, w))


def cond_f32(g: torch.Tensor | None):
    """fp32 copy of a 16-bit cond tensor (every layer's slice then feeds the
    fused gate's fp32 epilogue without a cast of its own), or None when the
    fused gate does not run (its callers keep the 16-bit slices)."""
    if (g is None or not GATE_FUSED or not COND_F32 or not g.is_cuda
            or g.dtype not in (torch.float16, torch.bfloat16)):
        return None
    return g.float()


def conv1d_gate(module: nn.Module, x: torch.Tensor, g, in_slope: float = 1.0, g16=None):
    """gate(module(leaky_relu(x, in_slope)), g) (WN / ResBlock2, the conv's
    output feeding only the gate) as one conv launch on a ROCm device
    (ConvGateHip16 under fp16 autocast, ConvGateHip32 in fp32 training);
    None when that does not apply (the caller runs conv1d + gate)."""
    wdt = train_wdtype(x)
    if (not GATE_FUSED or wdt is None or not (_io16(wdt) or wdt == WDT_F32)
            or not supported(module) or module.out_channels % 2):
        return None
    if wdt == WDT_F32:
        cond = None if g is None else g.float()
        return ConvGateHip32.apply(x.float(), weight_norm_effective(module), module.bias, cond,
                                   module.dilation[0], module.padding[0], in_slope)
    t16 = _TORCH_16[wdt]
    w = weight_norm_effective(module)
    ent = _PREPACK.get(module)
    pre = ent[1] if (ent is not None and ent[0] is w and ent[2] == wdt and ent[3]) else None
    if g is not None and g16 is None:
        g = g.to(t16)  # (the reference's cond is an autocast op's 16-bit output)
    if g16 is not None and g16.dtype != t16:
        g16 = None
    return ConvGateHip16.apply(x if x.dtype == t16 else x.to(t16), w, module.bias, g,
                               module.dilation[0], module.padding[0], in_slope, wdt, pre, g16)


# ---------------------------------------------------------------------------
# a Generator stage's three ResBlock2 branches as grouped launches
# (models.py:311-313, modules.py:250-260) under fp16 autocast
# ---------------------------------------------------------------------------
# The stage's branches (k = 3, 7, 11) read the same input and are independent
# until their mean, so pair p of every branch runs as ONE grouped launch
# (vits_conv1d_forward_groups, blockIdx.z = branch x utterance) each way:
# forward c1 + gate and c2 + residual, backward c2's input gradient, the
# three gate backwards (vits_gate_backward_io16_multi) and c1's input
# gradient with the leaky-relu derivative and the residual gradient in its
# epilogue.  Per stage 6 forward conv launches instead of 18 and 9 backward
# ones instead of 27, with three times the workgroups of one conv - the
# 48-frame decoder slices' 256-channel stage alone is 1.2 rounds of the chip.
# False: the per-branch ResBlock2.forward (Conv1dHip16 / ConvGateHip16).
STAGE_GROUPED = True
RB_SLOPE = 0.1  # modules.LRELU_SLOPE (modules.py:251)


def _stage_tile(m: int, T: int) -> int:
    """One tile for all three branches of a grouped launch (their own tile
    picks differ by k): 32-row layers 32x256, else 64x256 on time rows of
    whole 256-column tiles, 64x128 otherwise (the 384-frame stage)."""
    if m <= 32:
        return TILE_32x256
    return TILE_64x256 if T % 256 == 0 else TILE_64x128


def _img_layer(img, chans: int, rows: int, k: int, dil: int, pad_left: int, epi: int, T: int,
               wdtype: int, bias=None) -> PackedConv:
    tile = _stage_tile(rows, T)
    kc = _train_kc(img.shape[0] * 16, k, dil, tile, True)
    return PackedConv(img, bias, chans, rows, k, dil, pad_left, epi, tile, kc, out_channels=rows,
                      wdtype=wdtype)


def _gmask_desc(d, gm: torch.Tensor, slope: float):
    d.gmask, d.gmask_bstride, d.gmask_cstride = gm.data_ptr(), gm.stride(0), gm.stride(1)
    d.gmask_slope = slope
    return d


class ResblockStage16(torch.autograd.Function):
    """The three ResBlock2 branches of one Generator stage on fp16
    activations (x, the gated tensors, pre-activations, outputs and their
    gradients fp16; W / b fp32 masters, packed by ``prepacked``), returning
    the branch mean ((x0 + x1) + x2) / 3 as the reference's Generator sums
    them (models.py:311-313).

    forward(x, cond32, cond16, meta, *params): cond32 / cond16 are the
    stage's columns of the conditioning Linears' output (fp32 copy for the
    gate epilogue, 16-bit for the gate backward), meta[j][p] = (k, dil,
    pad1, pad2, column, (img1, img1_t), (img2, img2_t), wdtype), params =
    (w1, b1, w2, b2) per (branch j, pair p), branch-major."""

    @staticmethod
    def forward(ctx, x, cond32, cond16, meta, *params):
        B, C, T = x.shape
        H = C // 2
        dev = x.device
        wdt = meta[0][0][7]
        xs = [x, x, x]
        saved = []
        for p in range(3):
            acts = [torch.empty(B, H, T, device=dev, dtype=x.dtype) for _ in range(3)]
            xins = [torch.empty(B, C, T, device=dev, dtype=x.dtype) for _ in range(3)]
            ys = [torch.empty(B, C, T, device=dev, dtype=x.dtype) for _ in range(3)]
            g1, g2 = [], []
            for j in range(3):
                k, dil, pad1, pad2, col, im1, im2, _ = meta[j][p]
                w1, b1, w2, b2 = params[4 * (3 * j + p):4 * (3 * j + p) + 4]
                l1 = _img_layer(im1[0], C, C, k, dil, pad1, EPI_GATE, T, wdt,
                                b1.detach().float().contiguous())
                g1.append(make_desc(l1, xs[j], make_out(acts[j]), out1=make_out(xins[j]),
                                    in_slope=RB_SLOPE, tin=T, n_out=T, cond=cond32,
                                    cond_offset=col, io16=True))
                l2 = _img_layer(im2[0], H, C, k, 1, pad2, EPI_STORE, T, wdt,
                                b2.detach().float().contiguous())
                g2.append(make_desc(l2, acts[j], make_out(ys[j], res=xs[j]), tin=T, n_out=T,
                                    io16=True))
            conv1d_launch_seq([tuple(g1)], B, dev)
            conv1d_launch_seq([tuple(g2)], B, dev)
            saved.append((list(xs), acts, xins))
            xs = ys
        out = (xs[0] + xs[1] + xs[2]) / 3
        ctx.meta = meta
        ctx.stage = saved
        ctx.save_for_backward(cond16)
        ctx.nparams = len(params)
        return out

    @staticmethod
    def backward(ctx, g):
        (cond16,) = ctx.saved_tensors
        meta = ctx.meta
        x0 = ctx.stage[0][0][0]
        B, C, T = x0.shape
        H = C // 2
        dev = x0.device
        wdt = meta[0][0][7]
        lib = _lib.load()
        G = (g.to(x0.dtype) / 3).contiguous()  # DivBackward of the branch mean
        Gs = [G, G, G]
        dparams = [None] * ctx.nparams
        dcond = torch.empty(B, 9 * C, device=dev, dtype=torch.float32)
        for p in (2, 1, 0):
            xs, acts, xins = ctx.stage[p]
            dacts = [torch.empty(B, H, T, device=dev, dtype=x0.dtype) for _ in range(3)]
            dxins = [torch.empty(B, C, T, device=dev, dtype=x0.dtype) for _ in range(3)]
            dxs = [torch.empty(B, C, T, device=dev, dtype=x0.dtype) for _ in range(3)]
            g2, g1 = [], []
            jobs = (_lib.GateBwdJob * 3)()
            for j in range(3):
                k, dil, pad1, pad2, col, im1, im2, _ = meta[j][p]
                l2t = _img_layer(im2[1], C, H, k, 1, (k - 1) - pad2, EPI_STORE, T, wdt)
                g2.append(make_desc(l2t, Gs[j], make_out(dacts[j]), tin=T, n_out=T, io16=True))
                q = jobs[j]
                q.dy, q.dy_bstride, q.dy_cstride = dacts[j].data_ptr(), H * T, T
                q.x, q.x_bstride, q.x_cstride = xins[j].data_ptr(), C * T, T
                q.g = cond16.data_ptr() + cond16.element_size() * col
                q.g_bstride = cond16.stride(0)
                q.dx, q.dx_bstride, q.dx_cstride = dxins[j].data_ptr(), C * T, T
                q.dg, q.dg_bstride = dcond.data_ptr() + 4 * (3 * j + p) * C, 9 * C
                q.half_channels = H
                l1t = _img_layer(im1[1], C, C, k, dil, (k - 1) * dil - pad1, EPI_STORE, T, wdt)
                g1.append(_gmask_desc(
                    make_desc(l1t, dxins[j], make_out(dxs[j], res=Gs[j]), tin=T, n_out=T,
                              io16=True), xs[j], RB_SLOPE))
            conv1d_launch_seq([tuple(g2)], B, dev)
            check(lib.vits_gate_backward_io16_multi(jobs, 3, B, T, wdt, _stream_ptr(dev)),
                  "vits_gate_backward_io16_multi")
            conv1d_launch_seq([tuple(g1)], B, dev)
            for j in range(3):
                k, dil, pad1, pad2 = meta[j][p][:4]
                i0 = 4 * (3 * j + p)
                dparams[i0 + 2], dparams[i0 + 3] = wgrad(Gs[j], acts[j], k, 1, pad2, 1.0,
                                                         wdtype=wdt, split=True)
                dparams[i0], dparams[i0 + 1] = wgrad(dxins[j], xs[j], k, dil, pad1, RB_SLOPE,
                                                     wdtype=wdt, split=True)
            Gs = dxs
        dx = Gs[0] + Gs[1] + Gs[2]
        ctx.stage = None
        return (dx, dcond, None, None, *dparams)


def resblock_stage(x: torch.Tensor, resblocks, y16: torch.Tensor, y32: torch.Tensor, col0: int):
    """mean_j resblocks[j](x) for a Generator stage's three ResBlock2 (their
    conditioning Linears' outputs are the columns col0 .. of y16 / y32, the
    Generator's one conditioning GEMM) as ResblockStage16, or None when it
    does not apply (not the fp16 autocast training step, weights not
    prepacked, another topology): the caller runs the branches one by one."""
    wdt = train_wdtype(x)
    if (not STAGE_GROUPED or wdt is None or not _io16(wdt) or len(resblocks) != 3
            or x.dim() != 3 or y16 is None or y32 is None):
        return None
    t16 = _TORCH_16[wdt]
    C = x.shape[1]
    meta, params = [], []
    col = 0
    for rb in resblocks:
        if (len(rb.convs1) != 3 or rb.convs1[0].out_channels != C or rb.convs1[0].in_channels != C
                or C % 32):
            return None
        row = []
        for c1, c2 in zip(rb.convs1, rb.convs2):
            w1, w2 = weight_norm_effective(c1), weight_norm_effective(c2)
            e1, e2 = _PREPACK.get(c1), _PREPACK.get(c2)
            if (e1 is None or e2 is None or e1[0] is not w1 or e2[0] is not w2 or e1[2] != wdt
                    or e2[2] != wdt or not e1[3] or e2[3] or c1.bias is None or c2.bias is None
                    or c1.padding[0] * 2 != (c1.kernel_size[0] - 1) * c1.dilation[0]
                    or c2.padding[0] * 2 != c2.kernel_size[0] - 1 or c2.dilation[0] != 1):
                return None
            row.append((c1.kernel_size[0], c1.dilation[0], c1.padding[0], c2.padding[0], col,
                        e1[1], e2[1], wdt))
            params += [w1, c1.bias, w2, c2.bias]
            col += C
        meta.append(row)
    x16 = (x if x.dtype == t16 else x.to(t16)).contiguous()
    if x16.shape[2] % 4:
        return None
    cond32 = y32[:, col0:col0 + col]
    cond16 = y16[:, col0:col0 + col]
    if cond16.dtype != t16:
        return None
    return ResblockStage16.apply(x16, cond32, cond16, meta, *params)
