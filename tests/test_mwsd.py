"""MultiWaveSTFTDiscriminator (train_stft.py's D, reference mrd.py:200-236)
against golden vectors recorded from the reference itself
(tests/golden/make_golden.py::make_mwsd): same keys and shapes, the ten
scores of one training-mode forward (one spectral-norm power iteration per
layer), the u vectors / v checksums after it, d(generator_loss)/d(input)
for the waveform and the five magnitude maps, and every parameter gradient.

CPU: fp32 torch convs + GroupedSpectralNorm (batched power iteration).
GPU fp32: torch convs, spectral norm as the one-launch HIP
``spectral_norm_all`` (wnorm.hip).
GPU fp16 autocast (the training configuration, fp16_run=true): the wave
discriminators' convs on the HIP training conv (Conv1dHip16), the STFT
discriminators' first layer unfolded onto it, the rest MIOpen.  Operands
round to fp16 as the reference's autocast convs do, so the tolerances are
measured against the reference's own fp16 arithmetic (the same forward /
backward with torch's autocast convs on the same GPU, vs the same fp32
golden); the fp32 paths are held to 1e-4 / 2e-4.
"""
import json
import os

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


def _load():
    return dict(np.load(os.path.join(GOLD, "mwsd.npz"), allow_pickle=False))


def _build(device):
    from vits_amd.discriminators import MultiWaveSTFTDiscriminator
    from vits_amd.utils import deterministic_fill_, deterministic_fill_sn_

    d = MultiWaveSTFTDiscriminator()
    deterministic_fill_(d)
    deterministic_fill_sn_(d)
    return d.to(device).train()


def _run(d, G, device, autocast=False, loss_scale=1.0):
    """One training-mode forward + backward of generator_loss; under
    autocast the loss is scaled before the fp16 backward and the gradients
    unscaled after it (GradScaler's contract, train_stft.py:232)."""
    from vits_amd.losses import generator_loss

    y = torch.from_numpy(G["y"]).to(device).requires_grad_(True)
    mags = [torch.from_numpy(G[f"mag{i}"]).to(device).requires_grad_(True) for i in range(5)]
    with torch.autocast(device.type, dtype=torch.float16, enabled=autocast):
        outs = d(y, mags)
        with torch.autocast(device.type, enabled=False):
            lg, _ = generator_loss(outs)
    (lg * loss_scale).backward()
    return outs, lg, y.grad / loss_scale, [m.grad / loss_scale for m in mags]


def _nerr(got, ref):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    return float(np.abs(got - ref).max() / max(np.abs(ref).max(), 1e-30))


def _check(G, d, res, tol_out, tol_grad, tol_pgrad, tol_u):
    outs, lg, gy, gmags = res
    assert len(outs) == 10
    for i, o in enumerate(outs):
        ref = G[f"out{i}"]
        got = o.detach().float().cpu().numpy()
        assert got.shape == ref.shape, (i, got.shape, ref.shape)
        assert _nerr(got, ref) <= tol_out, (i, _nerr(got, ref))
    assert abs(float(lg.detach()) - float(G["loss_gen"])) <= tol_out * abs(float(G["loss_gen"]))
    assert _nerr(gy.cpu(), G["grad_y"]) <= tol_grad, _nerr(gy.cpu(), G["grad_y"])
    for i, gm in enumerate(gmags):
        head = gm[:, :, :4].float().cpu().numpy()
        assert _nerr(head, G[f"grad_mag{i}_head"]) <= tol_grad, (i, _nerr(head, G[f"grad_mag{i}_head"]))
        nrm = gm.double().norm().item()
        ref_nrm = float(G[f"grad_mag{i}_stats"][0])
        assert abs(nrm - ref_nrm) <= tol_grad * ref_nrm, (i, nrm, ref_nrm)
    # every parameter gradient: norm within tol, full tensors of the small ones
    params = dict(d.named_parameters())
    for k, (gn, gs, _, _) in zip(G["keys"], G["stats"]):
        g = params[str(k)].grad.double().cpu()
        assert abs(g.norm().item() - gn) <= tol_pgrad * gn, (str(k), g.norm().item(), gn)
    off = 0
    total = dict(d.named_parameters())
    for k in G["small_keys"]:
        g = total[str(k)].grad.float().cpu().numpy().ravel()
        ref = G["small_grad"][off:off + g.size]
        off += g.size
        assert _nerr(g, ref) <= tol_pgrad, (str(k), _nerr(g, ref))
    # spectral-norm state after the one power iteration of this forward
    sd = d.state_dict()
    off = 0
    for k, vsum in zip(G["sn_keys"], G["sn_vsum"]):
        u = sd[str(k) + "_u"].float().cpu().numpy()
        ref = G["sn_u"][off:off + u.size]
        off += u.size
        assert _nerr(u, ref) <= tol_u, (str(k), _nerr(u, ref))
        v = sd[str(k) + "_v"].double().sum().item()
        assert abs(v - vsum) <= tol_u * max(1.0, abs(vsum)), (str(k), v, vsum)


def test_mwsd_state_dict_keys_match_reference():
    with open(os.path.join(GOLD, "mwsd_state_dict_shapes.json")) as f:
        ref = json.load(f)
    got = {k: list(v.shape) for k, v in _build(torch.device("cpu")).state_dict().items()}
    assert got == ref


def test_mwsd_cpu_fp32_vs_reference():
    torch.set_num_threads(8)
    G = _load()
    d = _build(torch.device("cpu"))
    _check(G, d, _run(d, G, torch.device("cpu")), tol_out=1e-4, tol_grad=2e-4, tol_pgrad=2e-4,
           tol_u=1e-5)


@pytest.mark.gpu
def test_mwsd_gpu_fp32_vs_reference(device):
    G = _load()
    d = _build(device)
    _check(G, d, _run(d, G, device), tol_out=1e-4, tol_grad=2e-4, tol_pgrad=2e-4, tol_u=1e-5)


def _errors(G, d, res):
    """{metric: max error} of one forward/backward vs the golden."""
    outs, lg, gy, gmags = res
    e = {"out": max(_nerr(o.detach().float().cpu().numpy(), G[f"out{i}"])
                    for i, o in enumerate(outs)),
         "grad_y": _nerr(gy.cpu(), G["grad_y"]),
         "grad_mag": max(_nerr(g[:, :, :4].float().cpu().numpy(), G[f"grad_mag{i}_head"])
                         for i, g in enumerate(gmags))}
    params = dict(d.named_parameters())
    e["param_gnorm"] = max(abs(params[str(k)].grad.double().norm().item() / 1024.0 - gn) / gn
                           for k, (gn, _, _, _) in zip(G["keys"], G["stats"]))
    return e


@pytest.mark.gpu
@pytest.mark.parametrize("rows", [False, True])
def test_mwsd_gpu_fp16_autocast_vs_reference(device, monkeypatch, rows):
    """fp16 autocast (loss scaled by 1024 before the fp16 backward, as
    GradScaler does) vs the fp32 golden; the bar is the reference's own fp16
    arithmetic on this GPU (torch's autocast convs for every layer), within
    2x (+1e-3).  Measured on MI355X: scores 7e-3 (HIP) vs 1.2e-2 (torch),
    d/dy 6.2e-2 vs 1.0e-1, d/dmag 8.0e-2 vs 6.4e-2, worst parameter
    gradient norm 1.2e-2 vs 7.0e-3.  rows: the STFT discriminators' layers
    2+ as row-joined HIP convs (discriminators.STFT_D_ROWS, off by default)."""
    from vits_amd import discriminators, train_ops

    G = _load()
    monkeypatch.setattr(discriminators, "STFT_D_ROWS", rows)
    d = _build(device)
    hip = _errors(G, d, _run(d, G, device, autocast=True, loss_scale=1024.0))
    with monkeypatch.context() as mp:
        mp.setattr(train_ops, "autocast_wdtype", lambda *a, **k: None)
        mp.setattr(discriminators, "STFT_D_HIP", False)
        d2 = _build(device)
        ref16 = _errors(G, d2, _run(d2, G, device, autocast=True, loss_scale=1024.0))
    print("HIP fp16 :", hip)
    print("torch f16:", ref16)
    for k in hip:
        assert hip[k] <= 2.0 * ref16[k] + 1e-3, (k, hip[k], ref16[k])


@pytest.mark.parametrize("C,F,T,k0,s0,slope", [(1, 65, 19, 5, 2, 1.0), (64, 61, 37, 5, 2, 0.2),
                                               (64, 7, 23, 7, 1, 0.2), (3, 30, 9, 3, 3, 0.2)])
def test_conv2d_freq_joined_rows_layout_cpu(monkeypatch, C, F, T, k0, s0, slope):
    """The STFT-discriminator lowering (discriminators.conv2d_freq: frequency
    windows unfolded into channels, the F_out rows joined along time with
    their own zero padding) restated on the CPU: the HIP training conv is
    swapped for torch conv1d (with the leaky-relu prologue), so this checks
    only the unfold / join / slice index math against torch conv2d, fp64."""
    import torch.nn.functional as F_

    import vits_amd.discriminators as D

    def conv1d_hip(x, w, bias, dilation, padding, in_slope, wdt, residual=None):
        xa = F_.leaky_relu(x, in_slope) if in_slope != 1.0 else x
        return F_.conv1d(xa, w.to(x.dtype), None if bias is None else bias.to(x.dtype),
                         padding=padding, dilation=dilation)

    monkeypatch.setattr(D.train_ops, "conv1d_hip", conv1d_hip)
    g = torch.Generator().manual_seed(C + F + T)
    layer = torch.nn.Conv2d(C, 16, (k0, 5), stride=(s0, 1), padding=(0, 2)).double()
    x = torch.randn(2, C, F, T, generator=g, dtype=torch.float64, requires_grad=True)
    y = D.conv2d_freq(layer, x, None, in_slope=slope)
    xa = F_.leaky_relu(x, slope) if slope != 1.0 else x
    ref = F_.conv2d(xa, layer.weight, layer.bias, stride=(s0, 1), padding=(0, 2))
    assert y.shape == ref.shape
    assert torch.allclose(y, ref, atol=1e-12, rtol=1e-12)
    dy = torch.randn(ref.shape, generator=g, dtype=torch.float64)
    gx, gw = torch.autograd.grad(y, (x, layer.weight), dy)
    rx, rw = torch.autograd.grad(ref, (x, layer.weight), dy)
    assert torch.allclose(gx, rx, atol=1e-12) and torch.allclose(gw, rw, atol=1e-10)


class _EmuLib:
    """Restatement of the conv / wgrad kernels' addressing (vits_conv1d_desc
    x_rowlen / x_cgroup / y_rowlen, vits_conv1d_wgrad_desc) over CPU tensors,
    to check the row-joined STFT-discriminator descriptors on the CPU:
    pointers are resolved against the registered tensors, elements are read
    with the same per-column / per-chunk offset formulas as conv1d_impl.h and
    conv1d_train.hip (float64, no 16-bit rounding)."""

    def __init__(self):
        self.tensors = []
        self.weights = {}

    def reg(self, *ts):
        self.tensors += [t for t in ts if t is not None]

    def _find(self, ptr):
        for t in self.tensors:
            base = t.data_ptr()
            if base <= ptr < base + t.numel() * t.element_size():
                return t.view(-1), (ptr - base) // t.element_size()
        raise AssertionError("pointer of no registered tensor")

    @staticmethod
    def _xcol(t, rowlen, rowmul):
        if rowlen > 0:
            f = t // rowlen
            return f * rowmul + (t - f * rowlen)
        return t

    @staticmethod
    def _vbase(v, cstride, cgroup, gstride):
        if cgroup > 0:
            i = v // cgroup
            return (v - i * cgroup) * cstride + i * gstride
        return v * cstride

    def conv(self, d, B):
        xf, xo = self._find(d.x)
        w = self.weights[d.w]                      # [m][cin][k] fp64, taps in kernel order
        yf, yo = self._find(d.out0.y)
        n = torch.arange(d.n_out)
        for b in range(B):
            acc = torch.zeros(d.m, d.n_out, dtype=torch.float64)
            for v in range(d.cin):
                vb = xo + b * d.x_bstride + self._vbase(v, d.x_cstride, d.x_cgroup, d.x_gstride)
                for j in range(d.k):
                    col = n - d.pad_left + j * d.dil
                    ok = (col >= 0) & (col < d.tin)
                    idx = vb + self._xcol(col.clamp(min=0), d.x_rowlen, d.x_rowmul)
                    xv = torch.where(ok, xf[idx.clamp(0, xf.numel() - 1)].double(),
                                     torch.zeros((), dtype=torch.float64))
                    if d.in_slope != 1.0:
                        xv = torch.where(xv < 0, xv * d.in_slope, xv)
                    acc += w[:, v, j, None] * xv[None]
            if d.bias:
                bf, bo = self._find(d.bias)
                acc += bf[bo:bo + d.m].double()[:, None]
            ncol = self._xcol(n, d.y_rowlen, d.y_rowmul)
            if d.y_rowlen > 0:
                tl = n % d.y_rowlen
                rm = (tl < d.y_rowpad) | (tl >= d.y_rowpad + d.y_rowvalid)
            else:
                rm = torch.zeros_like(n, dtype=torch.bool)
            if d.gmask:
                gf, go = self._find(d.gmask)
                for m in range(d.m):
                    gv = gf[go + b * d.gmask_bstride + m * d.gmask_cstride + ncol].double()
                    acc[m] = torch.where(gv > 0, acc[m], acc[m] * d.gmask_slope)
            acc[:, rm] = 0
            for m in range(d.m):
                yf[yo + b * d.out0.y_bstride + m * d.out0.y_cstride + ncol] = acc[m].to(yf.dtype)

    def vits_conv1d_wgrad_workspace(self, wd, B):
        return 1

    def vits_conv1d_wgrad_split(self, wd, B, ws, nws, stream):
        dyf, dyo = self._find(wd.dy)
        xf, xo = self._find(wd.x)
        dwf, dwo = self._find(wd.dw_t)
        n = torch.arange(wd.n_out)
        dw = torch.zeros(wd.cout, wd.cin, wd.k, dtype=torch.float64)
        db = torch.zeros(wd.cout, dtype=torch.float64)
        for b in range(B):
            dy = torch.stack([dyf[dyo + b * wd.dy_bstride + o * wd.dy_cstride + n].double()
                              for o in range(wd.cout)])
            db += dy.sum(1)
            for v in range(wd.cin):
                vb = xo + b * wd.x_bstride + self._vbase(v, wd.x_cstride, wd.x_cgroup, wd.x_gstride)
                for j in range(wd.k):
                    col = n - wd.pad_left + j * wd.dil
                    ok = (col >= 0) & (col < wd.tin)
                    idx = vb + self._xcol(col.clamp(min=0), wd.x_rowlen, wd.x_rowmul)
                    xv = torch.where(ok, xf[idx.clamp(0, xf.numel() - 1)].double(),
                                     torch.zeros((), dtype=torch.float64))
                    if wd.in_slope != 1.0:
                        xv = torch.where(xv < 0, xv * wd.in_slope, xv)
                    dw[:, v, j] += dy @ xv
        dwf[dwo:dwo + dw.numel()] = dw.reshape(-1).to(dwf.dtype)
        if wd.dbias:
            bf, bo = self._find(wd.dbias)
            bf[bo:bo + wd.cout] = db.to(bf.dtype)
        return 0


@pytest.mark.parametrize("C,O,k0,s0,k1,F,T,slope", [(8, 6, 5, 2, 5, 17, 7, 0.2),
                                                    (8, 8, 5, 2, 3, 12, 5, 1.0),
                                                    (8, 1, 1, 1, 1, 1, 6, 0.2)])
def test_conv2d_rows_descriptors_cpu(monkeypatch, C, O, k0, s0, k1, F, T, slope):
    """train_ops.Conv2dRowsHip16's descriptors (row-padded layout, virtual
    channels, phase input-gradient convs, row-joined wgrad) run through a
    CPU restatement of the kernels' addressing (_EmuLib) reproduce torch
    conv2d's output and gradients in fp64 - the index math, on the CPU."""
    from vits_amd import train_ops

    emu = _EmuLib()
    R, p1, lp = train_ops.ROW_PAD, k1 // 2, 2

    def pack(w3, transpose, wdtype):
        w = w3.double()
        if transpose:  # rows = cin, channels = cout, taps reversed
            w = w.permute(1, 0, 2).flip(2)
        key = len(emu.weights) + 1
        emu.weights[key] = w.contiguous()

        class Img:
            shape = (1, 1, 1, 128, 8)

            def data_ptr(self):
                return key
        return Img()

    monkeypatch.setattr(train_ops, "_pack16_img", pack)
    monkeypatch.setattr(train_ops, "conv1d_launch", lambda d, B, dev: emu.conv(d, B))
    monkeypatch.setattr(train_ops, "_train_kc", lambda *a, **k: 16 if C % 16 == 0 else C)
    monkeypatch.setattr(train_ops._lib, "load", lambda: emu)
    monkeypatch.setattr(train_ops, "check", lambda rc, what: None)
    monkeypatch.setattr(train_ops, "_stream_ptr", lambda dev: 0)
    torch.manual_seed(2)
    B = 2
    L = train_ops.rows_len(T, lp)
    # fp32 tensors (the op's .float() views then alias them: registrable);
    # the restated kernel accumulates in fp64
    x = torch.randn(B, C, F, T)
    w = torch.randn(O, C, k0, k1)
    bias = torch.randn(O)
    xp = torch.nn.functional.pad(x, (lp, L - T - lp, R, R)).requires_grad_(True)
    wa, ba = w.clone().requires_grad_(True), bias.clone().requires_grad_(True)
    F_out = (F - k0) // s0 + 1
    orig_zeros = torch.zeros

    def zeros(*a, **k):  # register every buffer the op allocates
        t = orig_zeros(*a, **k)
        emu.reg(t)
        return t

    orig_empty = torch.empty

    def empty(*a, **k):
        t = orig_empty(*a, **k)
        emu.reg(t)
        return t

    monkeypatch.setattr(torch, "zeros", zeros)
    monkeypatch.setattr(torch, "zeros_like", lambda t, **k: zeros(t.shape, dtype=t.dtype))
    monkeypatch.setattr(torch, "empty", empty)
    emu.reg(xp, wa, ba)
    y = train_ops.Conv2dRowsHip16.apply(xp, wa, ba, s0, p1, lp, T, slope, train_ops.WDT_F16)
    gy = torch.randn(B, O, F_out, T)
    gyp = torch.nn.functional.pad(gy, (lp, L - T - lp, R, R))
    emu.reg(gyp)
    y.backward(gyp)
    monkeypatch.undo()
    xr = x.clone().requires_grad_(True)
    wr, br = w.clone().requires_grad_(True), bias.clone().requires_grad_(True)
    yr = torch.nn.functional.conv2d(torch.nn.functional.leaky_relu(xr, slope), wr, br,
                                    stride=(s0, 1), padding=(0, p1))
    yr.backward(gy)
    tol = dict(rtol=1e-4, atol=1e-4)
    assert torch.allclose(y[:, :, R:R + F_out, lp:lp + T], yr, **tol)
    assert y.abs().sum().item() == pytest.approx(yr.abs().sum().item(), rel=1e-5)  # pads 0
    assert torch.allclose(xp.grad[:, :, R:R + F, lp:lp + T], xr.grad, **tol)
    assert xp.grad.abs().sum().item() == pytest.approx(xr.grad.abs().sum().item(), rel=1e-5)
    assert torch.allclose(wa.grad, wr.grad, **tol)
    assert torch.allclose(ba.grad, br.grad, **tol)
