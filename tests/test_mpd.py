"""MultiPeriodDiscriminator (train.py's D, reference models.py:321-408)
against the golden vectors recorded from the reference itself
(tests/golden/make_golden.py::make_mpd): scores, feature-map sums, the three
GAN losses and d(loss_gen + loss_fm)/dy_hat.

CPU: fp32, the torch conv path (the period branch in its 1-D column layout).
GPU: fp32 (torch convs) and fp16 autocast (the stride-1 1024-channel layers
and conv_post on the HIP training conv, the rest MIOpen) — autocast rounds
operands to fp16 as the reference's autocast does, so its tolerance is the
fp16 one (1e-2 relative on losses, 3e-2 on the gradient's norm-relative
error); fp32 paths are held to 2e-5 / 1e-4.
"""
import json
import os

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


def _load():
    return dict(np.load(os.path.join(GOLD, "mpd.npz")))


def _build(device):
    from vits_amd.models import MultiPeriodDiscriminator
    from vits_amd.utils import deterministic_fill_

    d = MultiPeriodDiscriminator(False)
    deterministic_fill_(d)
    return d.to(device)


def _run(d, G, device, autocast=False):
    from vits_amd.losses import discriminator_loss, feature_loss, generator_loss

    y = torch.from_numpy(G["y"]).to(device)
    y_hat = torch.from_numpy(G["y_hat"]).to(device).requires_grad_(True)
    with torch.autocast(device.type, dtype=torch.float16, enabled=autocast):
        y_d_rs, y_d_gs, fmap_rs, fmap_gs = d(y, y_hat)
        with torch.autocast(device.type, enabled=False):
            loss_disc, _, _ = discriminator_loss(y_d_rs, [t.detach() for t in y_d_gs])
            loss_fm = feature_loss(fmap_rs, fmap_gs)
            loss_gen, _ = generator_loss(y_d_gs)
    (loss_gen + loss_fm).backward()
    return y_d_rs, y_d_gs, fmap_rs, fmap_gs, loss_disc, loss_fm, loss_gen, y_hat.grad


def _check(G, out, tol_loss, tol_grad, tol_score, tol_fmap):
    y_d_rs, y_d_gs, fmap_rs, fmap_gs, loss_disc, loss_fm, loss_gen, grad = out
    for name, got in (("loss_disc", loss_disc), ("loss_fm", loss_fm), ("loss_gen", loss_gen)):
        ref = float(G[name])
        assert abs(float(got) - ref) <= tol_loss * abs(ref), (name, float(got), ref)
    for i in range(len(y_d_rs)):
        for key, t in ((f"r{i}", y_d_rs[i]), (f"g{i}", y_d_gs[i])):
            ref = G[key]
            got = t.detach().float().cpu().numpy()
            assert got.shape == ref.shape, (key, got.shape, ref.shape)
            err = np.abs(got - ref).max() / max(np.abs(ref).max(), 1e-6)
            assert err <= tol_score, (key, err)
        for j, (a, b) in enumerate(zip(fmap_rs[i], fmap_gs[i])):
            assert list(a.shape) == list(G[f"fr{i}_{j}_shape"]), (i, j, a.shape)
            ab = float(a.detach().double().abs().sum())
            ref_abs = float(G[f"fr{i}_{j}_abs"])
            assert abs(ab - ref_abs) <= tol_fmap * ref_abs, (i, j, ab, ref_abs)
            for key, t in ((f"fr{i}_{j}_sum", a), (f"fg{i}_{j}_sum", b)):
                s = float(t.detach().double().sum())
                assert abs(s - float(G[key])) <= tol_fmap * ref_abs, (key, s, float(G[key]))
    ref = G["grad_y_hat"]
    got = grad.detach().float().cpu().numpy()
    err = np.abs(got - ref).max() / np.abs(ref).max()
    assert err <= tol_grad, err


def test_mpd_state_dict_keys_match_reference():
    with open(os.path.join(GOLD, "mpd_state_dict_shapes.json")) as f:
        ref = json.load(f)
    got = {k: list(v.shape) for k, v in _build(torch.device("cpu")).state_dict().items()}
    assert got == ref


def test_mpd_cpu_fp32_vs_reference():
    G = _load()
    out = _run(_build(torch.device("cpu")), G, torch.device("cpu"))
    _check(G, out, tol_loss=2e-5, tol_grad=1e-4, tol_score=1e-4, tol_fmap=1e-5)


def test_mpd_reexported_from_models():
    import vits_amd.discriminators as D
    import vits_amd.models as M

    assert M.MultiPeriodDiscriminator is D.MultiPeriodDiscriminator


@pytest.mark.gpu
def test_mpd_gpu_fp32_vs_reference(device):
    G = _load()
    out = _run(_build(device), G, device)
    _check(G, out, tol_loss=2e-5, tol_grad=1e-4, tol_score=1e-4, tol_fmap=1e-5)


@pytest.mark.gpu
def test_mpd_gpu_fp16_autocast_vs_reference(device):
    G = _load()
    out = _run(_build(device), G, device, autocast=True)
    _check(G, out, tol_loss=1e-2, tol_grad=3e-2, tol_score=3e-2, tol_fmap=1e-2)
