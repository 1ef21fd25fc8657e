"""FusedRAdam (vits_amd/optim.py, csrc/optim.hip) against a restatement of
the reference's radam.py (radam.py:35-99: the D optimizer of
train_stft.py:97) in the reference's arithmetic (fp32 tensors, Python-double
scalars), including the warm-up branch (N_sma < 5 for the first steps) and
GradScaler's skip rule (found_inf) without a host sync.  Tolerance: 1e-6 of
the parameter magnitude (a few fp32 ulps after 8 steps; only the FMA
contraction of the kernel differs)."""
import math

import pytest
import torch

from vits_amd.optim import FusedRAdam

pytestmark = pytest.mark.gpu


def radam_ref(params, grads_seq, lr=1e-4, b1=0.9, b2=0.999, eps=1e-8, wd=0.0):
    ps = [p.float().clone() for p in params]
    m = [torch.zeros_like(p) for p in ps]
    v = [torch.zeros_like(p) for p in ps]
    for t, grads in enumerate(grads_seq, 1):
        b2t = b2 ** t
        nmax = 2 / (1 - b2) - 1
        n = nmax - 2 * t * b2t / (1 - b2t)
        if n >= 5:
            step = math.sqrt((1 - b2t) * (n - 4) / (nmax - 4) * (n - 2) / n * nmax / (nmax - 2)) / (1 - b1 ** t)
        else:
            step = 1.0 / (1 - b1 ** t)
        for i, g in enumerate(grads):
            g = g.float()
            v[i].mul_(b2).addcmul_(g, g, value=1 - b2)
            m[i].mul_(b1).add_(g, alpha=1 - b1)
            if wd:
                ps[i].add_(ps[i], alpha=-wd * lr)
            if n >= 5:
                ps[i].addcdiv_(m[i], v[i].sqrt().add_(eps), value=-step * lr)
            else:
                ps[i].add_(m[i], alpha=-step * lr)
    return ps


def test_fused_radam_matches_radam_py(device):
    gen = torch.Generator().manual_seed(0)
    shapes = [(64, 1, 1), (1, 64, 5), (160, 160, 5), (7,), (513,)] + [(3, 3)] * 120  # > 96 tensors
    params = [torch.randn(*s, generator=gen) for s in shapes]
    grads_seq = [[torch.randn(*s, generator=gen) * 0.1 for s in shapes] for _ in range(8)]
    pd = [p.to(device).requires_grad_(True) for p in params]
    opt = FusedRAdam(pd, 1e-4, weight_decay=0.01)
    for grads in grads_seq:
        for p, g in zip(pd, grads):
            p.grad = g.to(device)
        opt.step()
    ref = radam_ref(params, grads_seq, wd=0.01)
    for p, r, p0 in zip(pd, ref, params):
        assert not torch.equal(r, p0)
        err = (p.detach().cpu() - r).abs().max().item()
        assert err <= 1e-6 * r.abs().max().item(), err
    assert float(opt.state[pd[0]]["step"]) == 8.0


def test_fused_radam_gradscaler_skip(device):
    """found_inf set by the scaler -> no parameter, moment or step change;
    the scaler drives the optimizer through _step_supports_amp_scaling
    (no .item() on found_inf)."""
    w = torch.randn(32, 16, device=device, requires_grad=True)
    opt = FusedRAdam([w], 1e-3)
    scaler = torch.amp.GradScaler("cuda", init_scale=4.0)
    scaler.scale(w.sum() * 2).backward()
    scaler.unscale_(opt)
    scaler.step(opt)
    scaler.update()
    w1 = w.detach().clone()
    m1 = opt.state[w]["exp_avg"].clone()
    assert float(opt.state[w]["step"]) == 1.0
    opt.zero_grad()
    scaler.scale(w.sum()).backward()
    w.grad.fill_(float("inf"))
    scaler.step(opt)   # stage READY: the scaler unscales and passes found_inf
    scaler.update()
    torch.cuda.synchronize()
    assert torch.equal(w.detach(), w1) and torch.equal(opt.state[w]["exp_avg"], m1)
    assert float(opt.state[w]["step"]) == 1.0
    assert scaler.get_scale() < 4.0
