"""Training-conv parity (vits_amd/train_ops.py): forward, input gradient,
weight and bias gradient of the HIP path against torch autograd in fp32 on
the SAME fp16-rounded operands (x, W, dY rounded to fp16 as the reference's
autocast convs round them, train_stft.py:165).  With identical operands the
only difference is fp32 summation order, so the tolerance is 2e-4 of each
tensor's max magnitude (the bias-free check below uses the unrounded dY for
dbias, which the kernel sums in fp32 before rounding)."""
import math

import pytest
import torch
import torch.nn.functional as F
import torch.nn.functional as F_

from vits_amd import train_ops

pytestmark = pytest.mark.gpu

TOL = 2e-4
# outputs / input gradients of the 16-bit-activation path (Conv1dHip16,
# GateHip16: the reference's autocast convs return fp16) are rounded to fp16
# once more: 2^-11 of each element, within 1.5e-3 of the tensor's max
TOL16 = 1.5e-3
TOL_Y = TOL16 if train_ops.TRAIN_IO16 else TOL


def _close(a, b, what, tol=TOL):
    a = a.detach().float().cpu()
    b = b.detach().float().cpu()
    assert a.shape == b.shape, (what, a.shape, b.shape)
    scale = b.abs().max().item() + 1e-12
    err = (a - b).abs().max().item()
    assert err <= tol * scale, f"{what}: max err {err:.3e} vs scale {scale:.3e}"


def _r16(t):
    return t.half().float()


CASES = [
    # B, cin, cout, k, dil, pad, T, slope
    (2, 256, 512, 5, 1, 2, 500, 1.0),      # WN in_layer (enc_q / flows)
    (2, 256, 512, 1, 1, 0, 333, 1.0),      # WN res_skip
    (3, 96, 256, 1, 1, 0, 130, 1.0),       # coupling pre
    (2, 128, 128, 11, 5, 25, 768, 0.1),    # ResBlock2 c1 (leaky prologue, k11 d5)
    (2, 32, 32, 7, 3, 9, 1500, 0.1),       # ResBlock2 c1, 32-channel stage
    (2, 16, 32, 3, 1, 1, 1000, 1.0),       # ResBlock2 c2 (cin = C'/2)
    (2, 192, 512, 7, 1, 3, 48, 1.0),       # conv_pre on a 48-frame slice
    (2, 32, 1, 7, 1, 3, 9216, 0.01),       # conv_post
    (2, 64, 64, 5, 9, 0, 700, 0.2),        # WaveDiscriminator dilated valid conv
    (2, 1, 64, 1, 1, 0, 1000, 1.0),        # WaveDiscriminator input conv
    (1, 513, 256, 1, 1, 0, 77, 1.0),       # PosteriorEncoder pre (ragged T)
    (2, 160, 160, 5, 4, 0, 301, 0.2),      # MWD scale 3, odd length
]


@pytest.mark.parametrize("io16", [False, True])
@pytest.mark.parametrize("B,cin,cout,k,dil,pad,T,slope", CASES)
def test_conv1d_train_fwd_bwd(device, B, cin, cout, k, dil, pad, T, slope, io16):
    """fp32 activations (Conv1dHip) and fp16 activations (Conv1dHip16: x, y,
    dY, dX fp16, read / written by the kernels as such)."""
    g = torch.Generator().manual_seed(B * 7919 + cin * 31 + cout + k * 3 + dil)
    x = torch.randn(B, cin, T, generator=g)
    w = torch.randn(cout, cin, k, generator=g) / (cin * k) ** 0.5
    b = torch.randn(cout, generator=g) * 0.1
    T_out = T + 2 * pad - (k - 1) * dil
    dy = torch.randn(B, cout, T_out, generator=g)
    if io16:  # the fp16 tensors the autocast step hands over
        x, dy = _r16(x), _r16(dy)
    fn = train_ops.Conv1dHip16 if io16 else train_ops.Conv1dHip
    tol = TOL16 if io16 else TOL

    xd = (x.half() if io16 else x).to(device).requires_grad_(True)
    wd = w.to(device).requires_grad_(True)
    bd = b.to(device).requires_grad_(True)
    y = fn.apply(xd, wd, bd, dil, pad, slope, train_ops.TRAIN_WDTYPE)
    assert y.dtype == (torch.float16 if io16 else torch.float32)
    y.backward((dy.half() if io16 else dy).to(device))

    xr = _r16(x).requires_grad_(True)
    wr = _r16(w).requires_grad_(True)
    br = b.clone().requires_grad_(True)
    xa = F.leaky_relu(xr, slope) if slope != 1.0 else xr
    # the kernel rounds the ACTIVATED input: round after the prologue
    xa16 = xa + (_r16(xa.detach()) - xa.detach())
    yr = F.conv1d(xa16, wr, br, padding=pad, dilation=dil)
    yr.backward(_r16(dy))
    _close(y, yr, "y", tol=tol)
    _close(xd.grad, xr.grad, "dx", tol=tol)
    _close(wd.grad, wr.grad, "dw")
    # dbias: the kernel sums the dY it is given in fp32
    _close(bd.grad, dy.sum((0, 2)), "db")


def test_conv1d_train_module_helper_matches_torch_module(device):
    """train_ops.conv1d on a weight-normed module: same forward and the
    gradients reach weight_g / weight_v through torch._weight_norm."""
    torch.manual_seed(0)
    conv = torch.nn.utils.weight_norm(torch.nn.Conv1d(64, 128, 5, padding=4, dilation=2))
    ref = torch.nn.utils.weight_norm(torch.nn.Conv1d(64, 128, 5, padding=4, dilation=2))
    ref.load_state_dict(conv.state_dict())
    conv = conv.to(device)
    x = torch.randn(2, 64, 300)
    with torch.autocast("cuda", dtype=torch.float16):
        y = train_ops.conv1d(conv, x.to(device), in_slope=0.1)
    # fp16 like a torch autocast conv (the 16-bit-activation path), else fp32
    assert y.dtype == (torch.float16 if train_ops.TRAIN_IO16 else torch.float32)
    y.float().square().sum().backward()
    yr = ref(F.leaky_relu(x, 0.1))
    yr.square().sum().backward()
    _close(y, yr, "y", tol=3e-3)   # fp16 operands vs fp32 torch
    for name in ("weight_g", "weight_v", "bias"):
        _close(getattr(conv, name).grad, getattr(ref, name).grad, name, tol=5e-3)


def test_conv1d_train_autocast(device):
    """Under fp16 autocast the op takes fp16 inputs, returns fp32 and its
    gradients flow back to the fp16 producer."""
    conv = torch.nn.Conv1d(32, 32, 3, padding=1).to(device)
    x = torch.randn(2, 32, 100, device=device, requires_grad=True)
    with torch.autocast("cuda", dtype=torch.float16):
        h = x * 2.0
        h16 = h.half()
        y = train_ops.conv1d(conv, h16)
    assert y.dtype == (torch.float16 if train_ops.TRAIN_IO16 else torch.float32)
    y.float().sum().backward()
    assert x.grad is not None and torch.isfinite(x.grad).all()
    assert conv.weight.grad is not None and conv.bias.grad is not None


def _f64_conv_ref(x, w, b, dil, pad, slope, dy, res=None):
    """fp64 CPU autograd reference of y = conv1d(leaky_relu(x)) + b (+ res)."""
    xr = x.double().cpu().requires_grad_(True)
    wr = w.double().cpu().requires_grad_(True)
    br = b.double().cpu().requires_grad_(True)
    xa = F.leaky_relu(xr, slope) if slope != 1.0 else xr
    yr = F.conv1d(xa, wr, br, padding=pad, dilation=dil)
    if res is not None:
        yr = yr + res.double().cpu()
    yr.backward(dy.double().cpu())
    return yr, xr.grad, wr.grad, br.grad


# fp32 training convs (Conv1dHip32) vs fp64: fp32 operands and accumulation;
# the weight gradient sums B * T products per element, so its error grows
# like sqrt(B T) fp32 roundings - 2e-5 of the tensor's max covers T <= 9216
TOL32 = 2e-5


@pytest.mark.parametrize("B,cin,cout,k,dil,pad,T,slope", CASES)
def test_conv1d_train_fp32_fwd_bwd(device, B, cin, cout, k, dil, pad, T, slope):
    """fp32 training (autocast off, the reference's fp16_run: false): the
    fp32 HIP conv (split / exact fp32 MFMA forward and input gradient,
    exact-fp32 MFMA split-K weight gradient) against fp64 autograd."""
    g = torch.Generator().manual_seed(B * 7919 + cin * 31 + cout + k * 3 + dil + 1)
    x = torch.randn(B, cin, T, generator=g)
    w = torch.randn(cout, cin, k, generator=g) / (cin * k) ** 0.5
    b = torch.randn(cout, generator=g) * 0.1
    T_out = T + 2 * pad - (k - 1) * dil
    dy = torch.randn(B, cout, T_out, generator=g)
    xd, wd, bd = (t.to(device).requires_grad_(True) for t in (x, w, b))
    y = train_ops.Conv1dHip32.apply(xd, wd, bd, dil, pad, slope)
    assert y.dtype == torch.float32
    y.backward(dy.to(device))
    yr, dxr, dwr, dbr = _f64_conv_ref(x, w, b, dil, pad, slope, dy)
    _close(y, yr, "y", tol=TOL32)
    _close(xd.grad, dxr, "dx", tol=TOL32)
    _close(wd.grad, dwr, "dw", tol=TOL32)
    _close(bd.grad, dbr, "db", tol=TOL32)


def test_conv1d_train_fp32_residual_and_module_path(device):
    """train_ops.conv1d without autocast on the GPU is the fp32 HIP conv
    (the library's conv / wgrad counters move), with ResBlock2's residual in
    the epilogue; HIP_TRAIN = False gives torch's module bit for bit."""
    from vits_amd import _lib

    torch.manual_seed(0)
    conv = torch.nn.utils.weight_norm(torch.nn.Conv1d(64, 128, 5, padding=4, dilation=2)).to(device)
    x = torch.randn(2, 64, 300, device=device, requires_grad=True)
    res = torch.randn(2, 128, 300, device=device, requires_grad=True)
    _lib.dispatch_counts_reset()
    y = train_ops.conv1d(conv, x, in_slope=0.1, residual=res)
    dy = torch.randn_like(y)
    y.backward(dy)
    c = _lib.dispatch_counts()
    assert c["conv_split"] + c["conv_f32"] >= 2 and c["wgrad_f32"] >= 2, c
    w = torch._weight_norm(conv.weight_v, conv.weight_g, 0).detach()
    yr, dxr, dwr, dbr = _f64_conv_ref(x.detach(), w, conv.bias.detach(), 2, 4, 0.1, dy,
                                      res=res.detach())
    _close(y, yr, "y", tol=TOL32)
    _close(x.grad, dxr, "dx", tol=TOL32)
    _close(res.grad, dy, "dres", tol=0.0)
    orig = train_ops.HIP_TRAIN
    try:
        train_ops.HIP_TRAIN = False
        xt = x.detach()
        assert torch.equal(train_ops.conv1d(conv, xt, in_slope=0.2), conv(F.leaky_relu(xt, 0.2)))
    finally:
        train_ops.HIP_TRAIN = orig


@pytest.mark.parametrize("cin,H,k,dil,T,slope,with_g", [
    (192, 192, 5, 1, 333, 1.0, True),     # WN in_layer with cond (enc_q / flows)
    (128, 64, 7, 3, 700, 0.1, True),      # ResBlock2 c1 (leaky prologue)
    (32, 16, 11, 5, 1000, 0.1, False),    # 32-channel stage, exact-fp32 rows
])
def test_conv_gate_fp32_matches_fp64(device, cin, H, k, dil, T, slope, with_g):
    """ConvGateHip32 (conv + tanh * sigmoid gate in one launch, fp32) vs the
    fp64 conv-then-gate: acts and the gradients of x, W, b and the cond."""
    g_ = torch.Generator().manual_seed(cin + H + k)
    B = 2
    pad = (k - 1) * dil // 2
    x = torch.randn(B, cin, T, generator=g_)
    w = torch.randn(2 * H, cin, k, generator=g_) / (cin * k) ** 0.5
    b = torch.randn(2 * H, generator=g_) * 0.1
    cond = torch.randn(B, 2 * H, generator=g_) * 0.5 if with_g else None
    dy = torch.randn(B, H, T, generator=g_)
    xd, wd, bd = (t.to(device).requires_grad_(True) for t in (x, w, b))
    cd = None if cond is None else cond.to(device).requires_grad_(True)
    acts = train_ops.ConvGateHip32.apply(xd, wd, bd, cd, dil, pad, slope)
    acts.backward(dy.to(device))
    xr, wr, br = (t.double().requires_grad_(True) for t in (x, w, b))
    cr = None if cond is None else cond.double().requires_grad_(True)
    xa = F.leaky_relu(xr, slope) if slope != 1.0 else xr
    z = F.conv1d(xa, wr, br, padding=pad, dilation=dil)
    if cr is not None:
        z = z + cr[:, :, None]
    ar = torch.tanh(z[:, :H]) * torch.sigmoid(z[:, H:])
    ar.backward(dy.double())
    _close(acts, ar, "acts", tol=TOL32)
    _close(xd.grad, xr.grad, "dx", tol=TOL32)
    _close(wd.grad, wr.grad, "dw", tol=TOL32)
    _close(bd.grad, br.grad, "db", tol=TOL32)
    if cd is not None:
        _close(cd.grad, cr.grad, "dcond", tol=TOL32)


@pytest.mark.parametrize("B,C,T", [(1, 8, 5), (3, 96, 37), (2, 256, 64), (4, 64, 1001)])
@pytest.mark.parametrize("k,dil,pad,slope", [(1, 1, 0, 1.0), (3, 1, 1, 0.2), (5, 16, 0, 0.2),
                                             (11, 6, 30, 0.1)])
def test_wgrad_fp32_edges(device, B, C, T, k, dil, pad, slope):
    """The exact-fp32 weight-gradient kernel on ragged shapes: T shorter than
    one 32-step chunk, odd channel counts, the widest supported window
    ((k - 1) dil = 64), zero / valid / 'same' padding; vs fp64."""
    if T + 2 * pad - (k - 1) * dil <= 0:
        pytest.skip("no output")
    g = torch.Generator().manual_seed(B + C + T + k)
    x = torch.randn(B, C, T, generator=g)
    T_out = T + 2 * pad - (k - 1) * dil
    dy = torch.randn(B, C + 3, T_out, generator=g)
    dw, db = train_ops.wgrad(dy.to(device), x.to(device), k, dil, pad, slope, with_bias=True,
                             wdtype=train_ops.WDT_F32, split=True)
    xr = x.double().requires_grad_(True)
    wr = torch.zeros(C + 3, C, k, dtype=torch.float64, requires_grad=True)
    br = torch.zeros(C + 3, dtype=torch.float64, requires_grad=True)
    xa = F.leaky_relu(xr, slope) if slope != 1.0 else xr
    F.conv1d(xa, wr, br, padding=pad, dilation=dil).backward(dy.double())
    _close(dw, wr.grad, "dw", tol=TOL32)
    _close(db, br.grad, "db", tol=TOL32)


def test_training_forward_autocast_hip_convs(device):
    """Tiny-config training forward under fp16 autocast (HIP convs with fp16
    operands) against the same forward with torch autocast convs: the two
    round operands identically, so the waveform slices agree to ~1e-3."""
    from common import build_model, golden, tiny_cfg
    from vits_amd import train_ops as T

    c = tiny_cfg()
    m = build_model(c["model"], c["data"], device)
    gd = golden("tiny_forward.npz")
    t = {k: torch.from_numpy(v) for k, v in gd.items()}
    args = (t["x"].to(device), t["x_lengths"].to(device), t["spec"].to(device),
            t["y_lengths"].to(device), t["emo"].to(device), t["sid"].to(device))
    kw = dict(noise_q=t["noise_q"].to(device), noise_align=t["noise_align"].to(device),
              noise_flow=t["noise_flow"].to(device))
    outs = []
    for use_hip in (True, False):
        orig_rand, orig_hip = torch.rand, T.HIP_TRAIN
        torch.rand = lambda *a, **k: t["rand_slice"].clone()
        T.HIP_TRAIN = use_hip
        try:
            with torch.autocast("cuda", dtype=torch.float16):
                outs.append(m(*args, **kw))
        finally:
            torch.rand, T.HIP_TRAIN = orig_rand, orig_hip
    (o_h, _, attn_h, ids_h), (o_t, _, attn_t, ids_t) = outs[0][:4], outs[1][:4]
    assert torch.equal(ids_h, ids_t)
    _close(o_h, o_t, "o", tol=2e-2)
    _close(o_h, torch.from_numpy(gd["o"]), "o vs fp32 reference", tol=3e-2)


@pytest.mark.parametrize("B,H,T,with_g", [(2, 256, 500, True), (3, 16, 1537, True), (2, 64, 77, False)])
def test_gate_fwd_bwd(device, B, H, T, with_g):
    """Fused WN / ResBlock2 gate and its gradient (incl. the cond gradient
    summed over time) against torch autograd in fp32."""
    gen = torch.Generator().manual_seed(H + T)
    x = torch.randn(B, 2 * H, T, generator=gen)
    g = torch.randn(B, 3 * H, generator=gen) if with_g else None   # sliced below
    dy = torch.randn(B, H, T, generator=gen)
    xd = x.to(device).requires_grad_(True)
    gd = g.to(device).requires_grad_(True) if with_g else None
    y = train_ops.GateHip.apply(xd, gd[:, H:3 * H] if with_g else None)
    y.backward(dy.to(device))
    xr = x.clone().requires_grad_(True)
    gr = g.clone().requires_grad_(True) if with_g else None
    xx = xr + gr[:, H:3 * H].unsqueeze(-1) if with_g else xr
    yr = torch.tanh(xx[:, :H]) * torch.sigmoid(xx[:, H:])
    yr.backward(dy)
    _close(y, yr, "y", tol=1e-5)
    _close(xd.grad, xr.grad, "dx", tol=1e-5)
    if with_g:
        _close(gd.grad, gr.grad, "dg", tol=1e-5)


@pytest.mark.parametrize("B,H,T,with_g", [(2, 256, 500, True), (3, 16, 1537, True), (2, 64, 77, False)])
def test_gate_fwd_bwd_io16(device, B, H, T, with_g):
    """GateHip16 (x, g, y, dY, dX fp16; fp32 math, the cond gradient summed
    in fp32) against torch autograd in fp32 on the same fp16 inputs."""
    gen = torch.Generator().manual_seed(H + T + 1)
    x = _r16(torch.randn(B, 2 * H, T, generator=gen))
    g = _r16(torch.randn(B, 2 * H, generator=gen)) if with_g else None
    dy = _r16(torch.randn(B, H, T, generator=gen))
    xd = x.half().to(device).requires_grad_(True)
    gd = g.half().to(device).requires_grad_(True) if with_g else None
    y = train_ops.GateHip16.apply(xd, gd, train_ops.TRAIN_WDTYPE)
    assert y.dtype == torch.float16
    y.backward(dy.half().to(device))
    xr = x.clone().requires_grad_(True)
    gr = g.clone().requires_grad_(True) if with_g else None
    xx = xr + gr.unsqueeze(-1) if with_g else xr
    yr = torch.tanh(xx[:, :H]) * torch.sigmoid(xx[:, H:])
    yr.backward(dy)
    _close(y, yr, "y", tol=TOL16)
    _close(xd.grad, xr.grad, "dx", tol=TOL16)
    if with_g:
        _close(gd.grad, gr.grad, "dg", tol=2 * TOL16)


@pytest.mark.parametrize("split", [False, True])
@pytest.mark.parametrize("B,cin,cout,k,dil,pad,T,slope", [
    (2, 256, 512, 5, 1, 2, 500, 1.0),      # large weight (atomic by default)
    (3, 32, 32, 7, 3, 9, 1500, 0.1),       # small weight (split by default)
    (5, 1024, 1, 3, 1, 1, 11, 1.0),        # MPD conv_post: one output row, T < 64
    (4, 64, 64, 5, 9, 0, 4097, 0.2),       # many (b, t) chunks, odd length
])
@pytest.mark.parametrize("io16", [False, True])
def test_wgrad_atomic_and_split_modes(device, B, cin, cout, k, dil, pad, T, slope, split, io16):
    """Both weight-gradient modes (fp32 atomics into [k][cout][cin]; split-K
    partial tiles + reduce written in [cout][cin][k]) against torch fp32 on
    the same fp16-rounded operands; fp32 or fp16 (io16) dY / x tensors
    (aligned rows: 8-byte block loads; odd lengths: element loads)."""
    g = torch.Generator().manual_seed(cin * 17 + cout + k + T)
    x = torch.randn(B, cin, T, generator=g)
    T_out = T + 2 * pad - (k - 1) * dil
    dy = torch.randn(B, cout, T_out, generator=g)
    if io16:
        x, dy = _r16(x), _r16(dy)
    cast = (lambda t: t.half()) if io16 else (lambda t: t)
    dw, db = train_ops.wgrad(cast(dy).to(device), cast(x).to(device), k, dil, pad, slope,
                             split=split)
    xr = _r16(F.leaky_relu(x, slope) if slope != 1.0 else x)
    wr = torch.zeros(cout, cin, k, requires_grad=True)
    F.conv1d(xr, wr, None, padding=pad, dilation=dil).backward(_r16(dy))
    _close(dw, wr.grad, "dw")
    _close(db, dy.sum((0, 2)), "db")


@pytest.mark.parametrize("C,O,K,u,T", [(512, 256, 16, 8, 48), (256, 128, 12, 6, 384),
                                       (128, 64, 4, 2, 2304), (64, 32, 4, 2, 4608),
                                       (24, 8, 4, 2, 77), (16, 8, 8, 2, 50)])
def test_conv_transpose1d_train_polyphase(device, C, O, K, u, T):
    """Generator upsampler in training (train_ops.conv_transpose1d under fp16
    autocast: polyphase lowering on Conv1dHip, leaky-relu 0.1 prologue fused)
    against torch's conv_transpose1d in fp32 on the same fp16-rounded
    operands: output, input, weight and bias gradients."""
    from torch.nn.utils import weight_norm

    g = torch.Generator().manual_seed(C + O + K + T)
    m = weight_norm(torch.nn.ConvTranspose1d(C, O, K, u, padding=(K - u) // 2))
    with torch.no_grad():
        m.weight_v.copy_(torch.randn(m.weight_v.shape, generator=g))
        m.weight_g.copy_(torch.rand(m.weight_g.shape, generator=g) + 0.5)
        m.bias.copy_(torch.randn(O, generator=g) * 0.1)
    x = torch.randn(2, C, T, generator=g)
    dy = torch.randn(2, O, T * u, generator=g)
    md = m.to(device)
    xd = x.to(device).requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.float16):
        y = train_ops.conv_transpose1d(md, xd, in_slope=0.1)
    assert y.dtype == (torch.float16 if train_ops.TRAIN_IO16 else torch.float32)
    assert y.shape == (2, O, T * u)
    y.backward(dy.to(device).to(y.dtype))

    w = torch._weight_norm(m.weight_v.detach().cpu(), m.weight_g.detach().cpu(), 0)
    wr = _r16(w).requires_grad_(True)
    br = m.bias.detach().cpu().clone().requires_grad_(True)
    xr = x.clone().requires_grad_(True)
    xa = F.leaky_relu(xr, 0.1)
    xa16 = xa + (_r16(xa.detach()) - xa.detach())
    yr = F.conv_transpose1d(xa16, wr, br, stride=u, padding=(K - u) // 2)
    yr.backward(_r16(dy))
    _close(y, yr, "y", tol=TOL_Y)
    _close(xd.grad, xr.grad, "dx", tol=TOL_Y)
    # d weight_v / weight_g go through the weight-norm reparametrisation on
    # both sides; compare the effective-weight gradient via the module's
    w_grad = torch.autograd.grad(
        torch._weight_norm(md.weight_v, md.weight_g, 0), [md.weight_v, md.weight_g],
        grad_outputs=wr.grad.to(device), allow_unused=True)
    _close(md.weight_v.grad, w_grad[0], "dweight_v")
    _close(md.bias.grad, (_r16(dy) if train_ops.TRAIN_IO16 else dy).sum((0, 2)), "db")


@pytest.mark.parametrize("C,F,T,k0,s0,slope", [(1, 65, 289, 5, 2, 1.0), (1, 1025, 19, 5, 2, 1.0),
                                               (64, 31, 145, 5, 2, 1.0), (1, 257, 73, 7, 3, 1.0),
                                               (64, 61, 19, 5, 2, 0.2), (64, 13, 37, 5, 2, 0.2)])
def test_conv2d_freq_unfolded(device, C, F, T, k0, s0, slope):
    """STFT-discriminator Conv2d(C, 64, (k0, 5), stride (s0, 1), padding (0, 2))
    (after leaky_relu(slope)) as the unfolded, row-joined stride-1 Conv1d on
    the HIP training conv (discriminators.conv2d_freq): output, magnitude
    gradient, weight and bias gradients vs torch conv2d in fp32 on the same
    fp16-rounded operands."""
    import vits_amd.discriminators as D

    g = torch.Generator().manual_seed(C * 1000 + F + k0)
    layer = torch.nn.Conv2d(C, 64, (k0, 5), stride=(s0, 1), padding=(0, 2))
    with torch.no_grad():
        layer.weight.copy_(torch.randn(layer.weight.shape, generator=g) / (C * k0 * 5) ** 0.5)
        layer.bias.copy_(torch.randn(64, generator=g) * 0.1)
    x = torch.rand(2, C, F, T, generator=g)
    F_out = (F - k0) // s0 + 1
    dy = torch.randn(2, 64, F_out, T, generator=g)
    ld = layer.to(device)
    xd = x.to(device).requires_grad_(True)
    if slope != 1.0:
        x = x - 0.5  # (both signs through the leaky relu)
        xd = x.to(device).requires_grad_(True)
    y = D.conv2d_freq(ld, xd, train_ops.TRAIN_WDTYPE, in_slope=slope)
    y.backward(dy.to(device).to(y.dtype))
    wr = _r16(layer.weight.detach().cpu()).requires_grad_(True)
    br = layer.bias.detach().cpu().clone().requires_grad_(True)
    xr = _r16(x).requires_grad_(True)
    xa = F_.leaky_relu(xr, slope) if slope != 1.0 else xr
    yr = F_.conv2d(_r16(xa) if slope != 1.0 else xa, wr, br, stride=(s0, 1), padding=(0, 2))
    yr.backward(_r16(dy))
    _close(y, yr, "y", tol=TOL_Y)
    _close(xd.grad, xr.grad, "dx", tol=TOL_Y)
    _close(ld.weight.grad, wr.grad, "dw")
    _close(ld.bias.grad, (_r16(dy) if train_ops.TRAIN_IO16 else dy).sum((0, 2, 3)), "db")


def test_conv1d_train_io16_residual(device):
    """Conv1dHip16 with the residual in the epilogue (ResBlock2's
    ``x = c2(xt) + x``): y = res + conv, d res = dY, and the other gradients
    as without the residual."""
    g = torch.Generator().manual_seed(5)
    B, cin, cout, k, T = 2, 16, 32, 7, 600
    x = _r16(torch.randn(B, cin, T, generator=g))
    w = torch.randn(cout, cin, k, generator=g) / (cin * k) ** 0.5
    b = torch.randn(cout, generator=g) * 0.1
    r = _r16(torch.randn(B, cout, T, generator=g))
    dy = _r16(torch.randn(B, cout, T, generator=g))
    xd = x.half().to(device).requires_grad_(True)
    wd = w.to(device).requires_grad_(True)
    bd = b.to(device).requires_grad_(True)
    rd = r.half().to(device).requires_grad_(True)
    y = train_ops.Conv1dHip16.apply(xd, wd, bd, 1, 3, 1.0, train_ops.TRAIN_WDTYPE, rd)
    y.backward(dy.half().to(device))
    xr = x.clone().requires_grad_(True)
    wr = _r16(w).requires_grad_(True)
    br = b.clone().requires_grad_(True)
    rr = r.clone().requires_grad_(True)
    yr = F.conv1d(xr, wr, br, padding=3) + rr
    yr.backward(dy)
    _close(y, yr, "y", tol=TOL16)
    _close(rd.grad, rr.grad, "dres", tol=0)
    _close(xd.grad, xr.grad, "dx", tol=TOL16)
    _close(wd.grad, wr.grad, "dw")


@pytest.mark.parametrize("with_out", [True, False])
def test_wn_update_matches_torch(with_out):
    """WNUpdate16 (csrc/wnres.hip) vs the reference's torch ops of WN.forward
    (modules.py:93-182) under fp16 autocast: x' = (x + rs[:, :H]) * mask,
    out' = out + rs[:, H:], x16' = x'.half(); forward and every gradient
    bit-exact (same fp32 / fp16 roundings, element-wise)."""
    dev = torch.device("cuda:0")
    B, H, T = 3, 192, 157
    gen = torch.Generator(device=dev).manual_seed(4)
    x = torch.randn(B, H, T, device=dev, generator=gen)
    rs = torch.randn(B, 2 * H, T, device=dev, generator=gen).half()
    mask = torch.ones(B, 1, T, device=dev)
    mask[1, :, 100:] = 0
    out = torch.randn(B, H, T, device=dev, generator=gen) if with_out else None
    a = torch.randn(B, H, T, device=dev, generator=gen)
    b16 = torch.randn(B, H, T, device=dev, generator=gen).half()
    c = torch.randn(B, H, T, device=dev, generator=gen)

    def run(fused):
        xs = x.clone().requires_grad_()
        rss = rs.clone().requires_grad_()
        outs = None if out is None else out.clone().requires_grad_()
        with torch.autocast("cuda", dtype=torch.float16):
            if fused:
                xn, x16, on = train_ops.wn_update(xs, rss, mask, outs)
            else:
                xn = (xs + rss[:, :H]) * mask
                on = (torch.zeros_like(xs) if outs is None else outs) + rss[:, H:]
                x16 = xn.half()
        loss = (xn * a).sum() + (x16 * b16).float().sum() + (on * c).sum()
        leaves = [xs, rss] + ([] if outs is None else [outs])
        grads = torch.autograd.grad(loss, leaves)
        return [xn, x16, on] + list(grads)

    assert train_ops.TRAIN_IO16
    got, want = run(True), run(False)
    for i, (g, w) in enumerate(zip(got, want)):
        assert g.dtype == w.dtype and g.shape == w.shape, i
        assert torch.equal(g, w), (i, (g.float() - w.float()).abs().max().item())


def test_prepacked_network_bitwise_equals_per_call_pack(device):
    """train_ops.prepacked: the 16-bit images of every HIP conv of a network
    packed in one vits_conv1d_pack16_pairs launch (48 layers per launch) give
    bit-identical outputs and gradients to the per-call
    vits_conv1d_pack16_pair path, for a mix of shapes (k 1..11, dilations,
    ragged channel counts, more layers than one launch holds)."""
    torch.manual_seed(3)
    specs = [(20, 36, 5, 1), (36, 64, 3, 3), (64, 17, 11, 1), (17, 40, 1, 1), (40, 40, 7, 2)]
    layers = torch.nn.ModuleList()
    for i in range(60):  # > 48: two launches
        cin, cout, k, dil = specs[i % len(specs)]
        if i > 0:
            cin = layers[-1].out_channels
        layers.append(torch.nn.Conv1d(cin, cout, k, dilation=dil, padding=dil * (k - 1) // 2))
    net = layers.to(device)
    x = torch.randn(2, 20, 136, device=device)

    def run(pre):
        for p in net.parameters():
            p.grad = None
        xi = x.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.float16):
            ctx = train_ops.prepacked(net) if pre else torch.autocast("cuda", enabled=True,
                                                                      dtype=torch.float16)
            with ctx:
                h = xi
                for i, m in enumerate(net):
                    h = train_ops.conv1d(m, h, in_slope=0.1 if i % 2 else 1.0)
        h.float().square().mean().backward()
        return h.detach().clone(), xi.grad.clone(), [p.grad.clone() for p in net.parameters()]

    a = run(False)
    orig = train_ops._pack16_pair

    def no_pack(*args, **kw):
        raise AssertionError("per-call pack inside a prepacked scope")

    train_ops._pack16_pair = no_pack
    try:
        b = run(True)
    finally:
        train_ops._pack16_pair = orig
    assert not train_ops._PREPACK  # scope cleared
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    for ga, gb in zip(a[2], b[2]):
        assert torch.equal(ga, gb)


@pytest.mark.parametrize("cin,H,k,dil,T,slope,with_g", [(64, 64, 5, 1, 500, 1.0, True),
                                                        (64, 32, 7, 3, 384, 0.1, True),
                                                        (48, 40, 3, 1, 130, 1.0, False)])
def test_conv_gate_fused_matches_conv_then_gate(device, cin, H, k, dil, T, slope, with_g):
    """train_ops.conv1d_gate (one conv launch: GATE epilogue on gate-
    interleaved weight rows + the pre-activation output for the backward)
    against the unfused conv1d -> GateHip16 path on the same inputs under
    fp16 autocast: acts and the gradients of x, W, b, g agree to 2e-3 of each
    tensor's max (the fused gate reads the fp32 accumulator instead of the
    fp16-rounded conv output), and the pre-activation it saves equals the
    unfused conv output to fp16 rounding."""
    torch.manual_seed(4)
    B = 2
    conv = torch.nn.Conv1d(cin, 2 * H, k, dilation=dil, padding=dil * (k - 1) // 2).to(device)
    conv._vits_gate = True
    x = torch.randn(B, cin, T, device=device)
    g = torch.randn(B, 2 * H, device=device) if with_g else None
    gy = torch.randn(B, H, T, device=device)

    def run(fused):
        for p in conv.parameters():
            p.grad = None
        xi = x.clone().requires_grad_(True)
        gi = None if g is None else g.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.float16):
            if fused:
                y = train_ops.conv1d_gate(conv, xi, gi, in_slope=slope)
                assert y is not None
            else:
                y = train_ops.gate(train_ops.conv1d(conv, xi, in_slope=slope), gi)
        y.float().backward(gy)
        return [y.float(), xi.grad, conv.weight.grad, conv.bias.grad] + (
            [gi.grad.float()] if gi is not None else [])

    a, b = run(False), run(True)
    for i, (u, v) in enumerate(zip(a, b)):
        err = (u.float() - v.float()).abs().max().item() / u.float().abs().max().item()
        assert err <= 2e-3, (i, err)


def test_qkv_cat_matches_three_convs(device, monkeypatch):
    """Self-attention's q / k / v projections as one HIP conv over the
    concatenated weight rows (train_ops.conv1d_cat) against three conv1d
    calls under fp16 autocast: outputs and the gradients of x and of every
    projection weight / bias agree to 2e-3 of each tensor's max (the input
    gradient is one K = 3C GEMM instead of three GEMMs and two fp16 adds)."""
    from vits_amd import attentions

    torch.manual_seed(7)
    mha = attentions.MultiHeadAttention(192, 192, 2, p_dropout=0.0).to(device)
    x = torch.randn(4, 192, 100, device=device)
    gy = torch.randn(4, 192, 100, device=device)
    mask = torch.ones(4, 1, 100, 100, device=device)

    def run(cat):
        monkeypatch.setattr(attentions, "QKV_CAT", cat)
        for p in mha.parameters():
            p.grad = None
        xi = x.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.float16):
            y = mha(xi, xi, mask)
        y.float().backward(gy)
        return [y.float(), xi.grad] + [p.grad for p in mha.parameters()]

    a, b = run(False), run(True)
    for i, (u, v) in enumerate(zip(a, b)):
        err = (u.float() - v.float()).abs().max().item() / u.float().abs().max().item()
        assert err <= 2e-3, (i, err)


def test_resblock_stage_grouped_matches_per_branch(device, monkeypatch):
    """train_ops.ResblockStage16 (a Generator stage's three ResBlock2 branches
    as grouped launches, their gate backwards as one multi-job launch) against
    the per-branch ResBlock2 path on the base config's decoder under fp16
    autocast with the prepacked images, 8 frames x 2 utterances (every stage:
    256 / 128 / 64 / 32 channels; T = 64 .. 1536).  Forward: bit-identical
    (same kernels and k-order, only the launch grouping differs), with 6
    forward conv launches per stage instead of 18.  Gradients: the grouped
    input gradient rounds `residual + conv` to fp16 once where autograd rounds
    the conv and then the add, so both are measured against the same step in
    fp32 (autocast off: the fp32 HIP training kernels) and the grouped path
    must be as close to it as the per-branch path (relative L2 within 1.25x
    + 1e-4 per tensor) and within 1e-2 relative L2 of the per-branch path."""
    from common import base_model
    from vits_amd import _lib
    from vits_amd.wnorm import WeightNormCache

    torch.manual_seed(11)
    m = base_model(device)
    dec = m.dec.train()
    z = torch.randn(2, 192, 8, device=device)
    g = torch.randn(2, 1024, device=device) * 0.5
    cache = WeightNormCache(dec)

    def run(grouped, fp16=True):
        monkeypatch.setattr(train_ops, "STAGE_GROUPED", grouped)
        for p in dec.parameters():
            p.grad = None
        zi = z.clone().requires_grad_(True)
        gi = g.clone().requires_grad_(True)
        _lib.dispatch_counts_reset()
        with torch.autocast("cuda", dtype=torch.float16, enabled=fp16), cache.active(), \
                train_ops.prepacked(dec):
            y = dec(zi, gi)
        torch.cuda.synchronize()
        nconv = _lib.dispatch_counts()["conv_16"]
        (y.float() * torch.linspace(-1, 1, y.shape[-1], device=device)).sum().backward()
        grads = {n: p.grad.detach().double().clone() for n, p in dec.named_parameters()
                 if p.grad is not None}
        grads["dz"], grads["dg"] = zi.grad.double(), gi.grad.double()
        return y.detach().clone(), grads, nconv

    ya, ga, na = run(False)
    yb, gb, nb = run(True)
    _, gr, _ = run(False, fp16=False)
    assert torch.equal(ya, yb), (ya.float() - yb.float()).abs().max().item()
    assert nb == na - 4 * 12, (na, nb)  # 4 stages: 6 grouped launches instead of 18
    assert set(ga) == set(gb) == set(gr)

    def rl2(a, b):
        return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()

    worst = []
    for n in ga:
        if gr[n].norm() == 0:
            continue
        ea, eb = rl2(ga[n], gr[n]), rl2(gb[n], gr[n])
        worst.append((eb - ea, n, ea, eb))
        assert eb <= 1.25 * ea + 1e-4 and rl2(gb[n], ga[n]) < 1e-2, (n, ea, eb)
    print("largest grouped-minus-per-branch error vs fp32:", sorted(worst)[-3:])


@pytest.mark.parametrize("B,C,F_out,T,p1", [(2, 64, 61, 19, 2), (3, 64, 7, 289, 2),
                                           (1, 8, 5, 3, 0), (2, 128, 33, 37, 1)])
def test_stftd_join_to_cl(device, B, C, F_out, T, p1):
    """discriminators._JoinToCL (stftd.hip join_to_cl) against torch's slice
    of the joined rows + channels-last copy + leaky_relu on the same fp16
    tensor: the output and the joined-row data gradient (zeros at the pad
    columns) bit-equal to torch autograd's."""
    import vits_amd.discriminators as D

    g = torch.Generator().manual_seed(B * 100 + C + F_out)
    L = (T + 2 * p1 + 3) // 4 * 4
    y = torch.randn(B, C, F_out * L, generator=g).half().to(device)
    y[:, :, :5] = 0  # (zeros through the activation)
    yd = y.clone().requires_grad_(True)
    out = D._JoinToCL.apply(yd, F_out, L, p1, T, 0.2)
    yr = y.clone().requires_grad_(True)
    ref = F.leaky_relu(yr.view(B, C, F_out, L)[..., p1:p1 + T], 0.2).contiguous(
        memory_format=torch.channels_last)
    assert out.shape == ref.shape and out.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(out, ref)
    dy = torch.randn(B, C, F_out, T, generator=g).half().to(device)
    out.backward(dy)
    ref.backward(dy)
    assert torch.equal(yd.grad, yr.grad)


@pytest.mark.parametrize("B,C,H,W", [(2, 64, 29, 37), (3, 64, 1, 19), (1, 32, 3, 5),
                                     (4, 128, 13, 73)])
def test_bias_lrelu_cl(device, B, C, H, W):
    """discriminators.bias_lrelu_cl (stftd.hip bias_lrelu) against torch's
    conv-bias add + leaky_relu on a channels-last fp16 tensor: output and
    data gradient bit-equal; the bias gradient (fp32 sum, rounded through
    fp16 as the reference's fp16 bias gradient) within one fp16 ulp of the
    fp64 sum, and identical run to run (ordered partials)."""
    import vits_amd.discriminators as D

    g = torch.Generator().manual_seed(B * 10 + C + H)
    y = torch.randn(B, C, H, W, generator=g).half().to(device).contiguous(
        memory_format=torch.channels_last)
    bias = (torch.randn(C, generator=g) * 0.3).to(device).requires_grad_(True)
    yd = y.clone().requires_grad_(True)
    out = D.bias_lrelu_cl(yd, bias, 0.2)
    yr = y.clone().requires_grad_(True)
    br = bias.detach().clone().requires_grad_(True)
    ref = F.leaky_relu(yr + br.half().view(1, C, 1, 1), 0.2)
    assert torch.equal(out, ref)
    dy = torch.randn(B, C, H, W, generator=g).half().to(device).contiguous(
        memory_format=torch.channels_last)
    out.backward(dy)
    ref.backward(dy)
    assert torch.equal(yd.grad, yr.grad)
    d16 = yr.grad.double().sum((0, 2, 3))
    ulp = d16.abs().half().float().double() * 2.0 ** -10 + 1e-6
    assert ((bias.grad.double() - d16).abs() <= ulp.to(device)).all()
    g1 = bias.grad.clone()
    bias.grad = None
    D.bias_lrelu_cl(y.clone().requires_grad_(True), bias, 0.2).backward(dy)
    assert torch.equal(bias.grad, g1)
    # the bias not requiring a gradient: the data gradient alone, unchanged
    yd2 = y.clone().requires_grad_(True)
    D.bias_lrelu_cl(yd2, bias.detach(), 0.2).backward(dy)
    assert torch.equal(yd2.grad, yr.grad)


@pytest.mark.parametrize("reverse", [False, True])
def test_coupling_block_fused_matches_reference_ops(reverse):
    """ResidualCouplingBlock under fp16 autocast with the coupling glue on
    wnres.hip (mask_cast, wn_final, the coupling update with the Flip folded
    in) vs the reference's op sequence (models.py:219-235, modules.py:314-360:
    pre * mask, WN output * mask, exp(logs = 0), cat, Flip) on the same HIP
    convs: the output, the input gradient and every parameter gradient
    bit-equal (the fused kernels round where autocast does; x1 * exp(0) is
    x1 exactly)."""
    from vits_amd import models

    dev = torch.device("cuda:0")
    torch.manual_seed(11)
    B, C, H, T, gin = 2, 16, 32, 157, 24
    blk = models.ResidualCouplingBlock(C, H, 5, [1, 1, 1, 1], 4, n_flows=4,
                                       gin_channels=gin).to(dev)
    with torch.no_grad():
        for f in blk.flows:
            if hasattr(f, "post"):  # (zero-initialised in the reference)
                f.post.weight.normal_(0, 0.05)
                f.post.bias.normal_(0, 0.05)
    x = torch.randn(B, C, T, device=dev)
    g = torch.randn(B, gin, device=dev)
    mask = torch.ones(B, 1, T, device=dev)
    mask[1, :, 120:] = 0
    w = torch.randn(B, C, T, device=dev)

    def run(fused):
        old = train_ops.COUPLING_FUSED
        train_ops.COUPLING_FUSED = fused
        try:
            blk.zero_grad(set_to_none=True)
            xs = x.clone().requires_grad_()
            with torch.autocast("cuda", dtype=torch.float16):
                if fused:
                    y = blk(xs, mask, g=g, reverse=reverse)
                else:  # the reference's loop: coupling, then the Flip module
                    y = xs
                    for f in (blk.flows if not reverse else list(blk.flows)[::-1]):
                        if reverse:
                            y = f(y, mask, g=g, reverse=True)
                        else:
                            y, _ = f(y, mask, g=g)
            (y * w).sum().backward()
            return [y.detach(), xs.grad] + [p.grad.clone() for p in blk.parameters()
                                            if p.grad is not None]
        finally:
            train_ops.COUPLING_FUSED = old

    got, want = run(True), run(False)
    assert len(got) == len(want)
    for i, (a, b) in enumerate(zip(got, want)):
        assert a.dtype == b.dtype and a.shape == b.shape, i
        assert torch.equal(a, b), (i, (a.float() - b.float()).abs().max().item())
