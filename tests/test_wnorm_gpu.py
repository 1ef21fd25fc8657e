"""One-launch weight / spectral normalisation (vits_amd/wnorm.py,
csrc/wnorm.hip) against torch's own hooks - the reference's
torch.nn.utils.weight_norm (modules.py:58-109, models.py:233) and
torch.nn.utils.spectral_norm (mrd.py) - on the same parameters.

Tolerances: weight norm is fp32 on both sides (summation order only): 2e-6
of each tensor's max for weights, 1e-5 for gradients.  Spectral norm in
fp32: 1e-5.  Inside fp16 autocast the reference's mv rounds its operands
and result to fp16 and so does the kernel; the BLAS and the kernel sum in
different orders, so a result can land one fp16 ulp apart: 2e-3."""
import copy

import pytest
import torch
from torch import nn

from vits_amd import ops, wnorm
from vits_amd.discriminators import GroupedSpectralNorm

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _close(a, b, tol, what):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    assert a.shape == b.shape, (what, a.shape, b.shape)
    scale = b.abs().max().item() + 1e-30
    err = (a - b).abs().max().item()
    assert err <= tol * scale, f"{what}: max err {err:.3e} vs scale {scale:.3e}"


def _wn_layers(n_extra=0):
    torch.manual_seed(0)
    mods = [
        nn.utils.weight_norm(nn.Conv1d(192, 384, 5, padding=2)),        # WN in_layer
        nn.utils.weight_norm(nn.Conv1d(192, 384, 1)),                   # res_skip
        nn.utils.weight_norm(nn.ConvTranspose1d(512, 256, 16, 8, 4)),   # upsampler (dim 0 = in)
        nn.utils.weight_norm(nn.Linear(256, 768)),                      # conditioning Linear
        nn.utils.weight_norm(nn.Conv1d(32, 16, 11, padding=5)),         # small ResBlock2 conv
    ]
    for i in range(n_extra):  # > VITS_WNORM_MAX layers: several launches
        mods.append(nn.utils.weight_norm(nn.Conv1d(8 + i % 5, 4 + i % 7, 3)))
    root = nn.ModuleList(mods).to(DEV)
    with torch.no_grad():  # g away from ||v|| so the reparametrisation matters
        for m in root:
            m.weight_g.mul_(torch.rand_like(m.weight_g) + 0.5)
    return root


@pytest.mark.parametrize("n_extra", [0, 70])
def test_weight_norm_forward_backward_matches_torch(n_extra):
    root = _wn_layers(n_extra)
    cache = wnorm.WeightNormCache(root)
    assert len(cache.mods) == len(root)
    ws = cache.weights()
    refs = [torch._weight_norm(m.weight_v, m.weight_g, 0) for m in root]
    for m, ref in zip(root, refs):
        _close(ws[m], ref, 2e-6, "w")
    # backward: one loss over all weights
    gen = torch.Generator(device=DEV).manual_seed(1)
    cot = [torch.randn(r.shape, device=DEV, generator=gen) for r in refs]
    params = [p for m in root for p in (m.weight_g, m.weight_v)]
    got = torch.autograd.grad(sum((ws[m] * c).sum() for m, c in zip(root, cot)), params)
    want = torch.autograd.grad(sum((r * c).sum() for r, c in zip(refs, cot)), params)
    for i, (a, b) in enumerate(zip(got, want)):
        _close(a, b, 1e-5, f"grad {i}")


def test_weight_norm_cache_serves_layers():
    root = _wn_layers()
    cache = wnorm.WeightNormCache(root)
    with cache.active():
        w_conv = ops.weight_norm_effective(root[0])
        assert ops.cached_weight(root[0]) is w_conv
    assert ops.cached_weight(root[0]) is None
    _close(w_conv, torch._weight_norm(root[0].weight_v, root[0].weight_g, 0), 2e-6, "cached")


def _sn_stack():
    torch.manual_seed(2)
    mods = nn.ModuleList([
        nn.utils.spectral_norm(nn.Conv1d(64, 64, 5, padding=2)),        # wave discriminator
        nn.utils.spectral_norm(nn.Conv2d(64, 64, (5, 3), padding=(2, 1))),  # STFT discriminator
        nn.utils.spectral_norm(nn.Conv2d(1, 64, (7, 5))),
        nn.utils.spectral_norm(nn.Conv1d(64, 1, 3, padding=1)),
        nn.utils.spectral_norm(nn.Conv1d(64, 64, 5, padding=2)),
    ]).to(DEV)
    return mods


def _run_sn(mods, sn, fused, training, autocast):
    """W_sn of every layer (sn = GroupedSpectralNorm(mods), which takes over
    the modules' hooks), then grads of weight_orig for a fixed cotangent."""
    wnorm_flag = wnorm.FUSED_NORMS
    wnorm.FUSED_NORMS = fused
    try:
        with torch.autocast("cuda", dtype=torch.float16, enabled=autocast):
            sn.apply(training)
        if fused:
            assert sn._fused_ok()
    finally:
        wnorm.FUSED_NORMS = wnorm_flag
    ws = [m.weight for m in mods]
    gen = torch.Generator(device=DEV).manual_seed(3)
    cot = [torch.randn(w.shape, device=DEV, generator=gen) for w in ws]
    origs = [m.weight_orig for m in mods]
    grads = torch.autograd.grad(sum((w.float() * c).sum() for w, c in zip(ws, cot)), origs)
    return ws, grads, [m.weight_u.clone() for m in mods], [m.weight_v.clone() for m in mods]


@pytest.mark.parametrize("autocast", [False, True])
@pytest.mark.parametrize("training", [True, False])
def test_spectral_norm_matches_torch_hooks(training, autocast):
    """Fused one-launch path vs the batched torch path (which equals torch's
    per-layer hooks, tests/test_train.py) from identical u / v buffers; two
    consecutive forwards (u / v updated in place by the first)."""
    base = _sn_stack()
    a, b = copy.deepcopy(base), copy.deepcopy(base)
    sa, sb = GroupedSpectralNorm(a), GroupedSpectralNorm(b)
    tol = 2e-3 if autocast else 1e-5
    for it in range(2):
        wa, ga, ua, va = _run_sn(a, sa, True, training, autocast)
        wb, gb, ub, vb = _run_sn(b, sb, False, training, autocast)
        for i in range(len(base)):
            _close(wa[i], wb[i], tol, f"it{it} W_sn {i}")
            _close(ga[i], gb[i], tol, f"it{it} dW {i}")
            _close(ua[i], ub[i], tol, f"it{it} u {i}")
            _close(va[i], vb[i], tol, f"it{it} v {i}")


def test_spectral_norm_matches_per_layer_torch_hook():
    """fp32, training: the fused path against torch's own per-layer hook."""
    base = _sn_stack()
    a, ref = copy.deepcopy(base), copy.deepcopy(base)
    wa, ga, ua, va = _run_sn(a, GroupedSpectralNorm(a), True, True, False)
    ref.train()
    for m in ref:
        m(torch.zeros(1, m.in_channels, *([8] * (m.weight.dim() - 2)), device=DEV))
    origs = [m.weight_orig for m in ref]
    gen = torch.Generator(device=DEV).manual_seed(3)
    cot = [torch.randn(m.weight.shape, device=DEV, generator=gen) for m in ref]
    gr = torch.autograd.grad(sum((m.weight * c).sum() for m, c in zip(ref, cot)), origs)
    for i, m in enumerate(ref):
        _close(wa[i], m.weight, 1e-5, f"W_sn {i}")
        _close(ua[i], m.weight_u, 1e-5, f"u {i}")
        _close(va[i], m.weight_v, 1e-5, f"v {i}")
        _close(ga[i], gr[i], 1e-5, f"dW {i}")


def _rel_l2(a, b):
    a, b = a.detach().double(), b.detach().double()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def _within_noise(ga, gb, gns, mult=3.0):
    """Every parameter gradient of the fused path (ga) within mult x the hook
    path's own noise envelope (the worst of its perturbed runs gns, each a
    1-ulp weight perturbation) of the hook path (gb), plus 1e-3.  weight_g
    (<dW_row, v_row> / ||v_row||, which cancels over the row: condition ~
    sqrt(fan-in)) is held apart from the other parameters, each against its
    own group's envelope; several perturbation draws (not one) set the
    envelope, so a single noisy draw does not decide the bar."""
    def worst(pairs, want_g):
        return max(_rel_l2(a, b) for (n, a), (_, b) in pairs if n.endswith("weight_g") == want_g)

    for want_g in (False, True):
        fused = worst(zip(ga, gb), want_g)
        floor = max(worst(zip(gn, gb), want_g) for gn in gns)
        assert fused <= mult * floor + 1e-3, (want_g, fused, floor)


def test_train_step_fused_spectral_norm_matches_torch_hooks():
    """One train_stft step (tiny config, fp16 autocast) with the one-launch
    spectral norm vs torch's hooks from identical models, batch and RNG
    state (the generator side identical, so y_hat is bit-equal): the same
    losses (1e-3), u / v buffers (2e-3), and gradients of every G and D
    parameter as close as the hook path is to itself when the D weights are
    perturbed by one fp32 ulp (W / sigma agrees to fp32 rounding; an element
    that rounds to the other fp16 neighbour in an autocast conv moves the
    fp16 gradients, measured here as the noise floor over three perturbation
    draws; fused within 3x, weight_g included)."""
    from test_train import _batch, _make, tiny_hps

    hps = tiny_hps()
    batch = [t.to(DEV) for t in _batch(hps, 4, seed=0)]
    res = []
    flags = wnorm.FUSED_NORMS, wnorm.FUSED_WN
    old_det = torch.backends.cudnn.deterministic
    try:
        wnorm.FUSED_WN = False
        # MIOpen's deterministic solvers: its default find makes the STFT
        # discriminators' Conv2d layers differ from run to run
        torch.backends.cudnn.deterministic = True
        for fused, perturb in ((True, 0), (False, 0), (False, 11), (False, 12), (False, 13)):
            wnorm.FUSED_NORMS = fused
            st = _make(hps, DEV, seed=0)
            if perturb:
                gen = torch.Generator(device=DEV).manual_seed(perturb)
                with torch.no_grad():
                    for n, p in st.net_d.named_parameters():
                        if n.endswith("weight_orig"):
                            p.mul_(1 + 2.0 ** -23 * torch.randn(p.shape, device=DEV,
                                                                generator=gen))
            st.scaler = torch.amp.GradScaler("cuda", init_scale=64.0)
            torch.manual_seed(5)
            out = st.step(batch)
            torch.cuda.synchronize()
            grads = [(f"{tag}.{n}", p.grad.detach().clone())
                     for tag, net in (("G", st.net_g), ("D", st.net_d))
                     for n, p in net.named_parameters() if p.grad is not None]
            res.append((out, grads, [b.detach().clone() for b in st.net_d.buffers()]))
    finally:
        wnorm.FUSED_NORMS, wnorm.FUSED_WN = flags
        torch.backends.cudnn.deterministic = old_det
    (oa, ga, ba), (ob, gb, bb) = res[:2]
    for k in ("loss_disc", "loss_gen_all", "loss_stft"):
        _close(oa[k], ob[k], 1e-3, k)
    assert all(len(r[1]) == len(ga) for r in res) and len(ga) > 100
    _within_noise(ga, gb, [r[1] for r in res[2:]])
    for i, (a, b) in enumerate(zip(ba, bb)):
        _close(a, b, 2e-3, f"D buffer {i}")


def test_generator_fused_weight_norm_matches_torch_hooks():
    """The generator forward of the train step (fp16 autocast) with every
    weight-normed layer's weight from the one-launch kernel vs torch's hooks
    (same model, inputs and RNG): y_hat within 2e-3 of its magnitude, and
    the parameter gradients for a fixed cotangent on y_hat as close as the
    hook path is to itself under a 1-ulp perturbation of the weights.

    Weights that differ in the last fp32 bit (summation order of ||v||)
    round to the other fp16 neighbour in some autocast convs, and the fp16
    gate / conv chain carries that through; the noise floor is measured here
    by running the hook path with weight_g scaled by (1 + 2^-23 r), r ~ N(0,1),
    three draws, and the fused path must stay within 3x of the worst.  (The train_stft losses
    are not a usable probe: the MR-STFT log-magnitude term's gradient is
    discontinuous in y_hat.)"""
    from test_train import _batch, _make, tiny_hps

    hps = tiny_hps()
    x, x_len, spec, spec_len, _, _, emo, spk = [t.to(DEV) for t in _batch(hps, 4, seed=0)]
    st = _make(hps, DEV, seed=0)
    gs = [p for n, p in st.net_g.named_parameters() if n.endswith("weight_g")]
    g0 = [p.detach().clone() for p in gs]
    res = []
    flag = wnorm.FUSED_WN
    try:
        for fused, perturb in ((True, 0), (False, 0), (False, 11), (False, 12), (False, 13)):
            wnorm.FUSED_WN = fused
            with torch.no_grad():
                gen = torch.Generator(device=DEV).manual_seed(perturb or 11)
                for p, p0 in zip(gs, g0):
                    p.copy_(p0 * (1 + 2.0 ** -23 * torch.randn(p.shape, device=DEV,
                                                                generator=gen))
                            if perturb else p0)
            st.net_g.zero_grad(set_to_none=True)
            torch.manual_seed(5)
            with st.autocast(), st._g_weights():
                y_hat = st.net_g(x, x_len, spec, spec_len, emo, spk)[0]
            cot = torch.randn(y_hat.shape, device=DEV,
                              generator=torch.Generator(device=DEV).manual_seed(7))
            (y_hat.float() * cot).sum().backward()
            torch.cuda.synchronize()
            res.append((y_hat.detach().float(), [(n, p.grad.detach().clone())
                                                 for n, p in st.net_g.named_parameters()
                                                 if p.grad is not None]))
    finally:
        wnorm.FUSED_WN = flag
        with torch.no_grad():
            for p, p0 in zip(gs, g0):
                p.copy_(p0)
    (ya, ga), (yb, gb) = res[:2]
    _close(ya, yb, 2e-3, "y_hat")
    assert all(len(r[1]) == len(ga) for r in res) and len(ga) > 50
    _within_noise(ga, gb, [r[1] for r in res[2:]])


def test_generator_fused_weight_norm_fp32_step():
    """The same comparison in fp32 training (autocast off: every generator
    conv on the fp32 HIP training kernels): no fp16 rounding to amplify, so
    fused and hook paths must agree to fp32 summation order - y_hat to 1e-5
    of its magnitude, every gradient (weight_g included) to 1e-3 relative."""
    from test_train import _batch, _make, tiny_hps

    hps = tiny_hps()
    x, x_len, spec, spec_len, _, _, emo, spk = [t.to(DEV) for t in _batch(hps, 4, seed=0)]
    st = _make(hps, DEV, seed=0)
    res = []
    flag = wnorm.FUSED_WN
    try:
        for fused in (True, False):
            wnorm.FUSED_WN = fused
            st.net_g.zero_grad(set_to_none=True)
            torch.manual_seed(5)
            with st._g_weights():
                y_hat = st.net_g(x, x_len, spec, spec_len, emo, spk)[0]
            cot = torch.randn(y_hat.shape, device=DEV,
                              generator=torch.Generator(device=DEV).manual_seed(7))
            (y_hat * cot).sum().backward()
            torch.cuda.synchronize()
            res.append((y_hat.detach(), [(n, p.grad.detach().clone())
                                         for n, p in st.net_g.named_parameters()
                                         if p.grad is not None]))
    finally:
        wnorm.FUSED_WN = flag
    (ya, ga), (yb, gb) = res
    _close(ya, yb, 1e-5, "y_hat")
    worst = max(((_rel_l2(a, b), n) for (n, a), (_, b) in zip(ga, gb)))
    assert worst[0] <= 1e-3, worst
