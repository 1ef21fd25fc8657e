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
def test_mwsd_gpu_fp16_autocast_vs_reference(device, monkeypatch):
    """fp16 autocast (loss scaled by 1024 before the fp16 backward, as
    GradScaler does) vs the fp32 golden; the bar is the reference's own fp16
    arithmetic on this GPU (torch's autocast convs for every layer), within
    2x (+1e-3).  Measured on MI355X: scores 7e-3 (HIP) vs 1.2e-2 (torch),
    d/dy 6.2e-2 vs 1.0e-1, d/dmag 8.0e-2 vs 6.4e-2, worst parameter
    gradient norm 1.2e-2 vs 7.0e-3."""
    from vits_amd import discriminators, train_ops

    G = _load()
    d = _build(device)
    hip = _errors(G, d, _run(d, G, device, autocast=True, loss_scale=1024.0))
    with monkeypatch.context() as mp:
        mp.setattr(train_ops, "HIP_TRAIN", False)
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
