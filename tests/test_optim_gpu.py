"""FusedRAdam (vits_amd/optim.py, csrc/optim.hip) against a restatement of
the reference's radam.py (radam.py:35-99: the D optimizer of
train_stft.py:97) in the reference's arithmetic (fp32 tensors, Python-double
scalars), including the warm-up branch (N_sma < 5 for the first steps) and
GradScaler's skip rule (found_inf) without a host sync.  Tolerance: 1e-6 of
the parameter magnitude (a few fp32 ulps after 8 steps; only the FMA
contraction of the kernel differs)."""
import pytest
import torch

from common import radam_ref
from vits_amd.optim import FusedRAdam

pytestmark = pytest.mark.gpu


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


def _shapes():
    return [(64, 1, 1), (1, 64, 5), (40, 40, 5), (7,), (3, 3)]


def _seq(shapes, n, seed):
    gen = torch.Generator().manual_seed(seed)
    params = [torch.randn(*s, generator=gen) for s in shapes]
    grads = [[torch.randn(*s, generator=gen) * 0.1 for s in shapes] for _ in range(n)]
    return params, grads


def test_fused_radam_resume_continues_step(device, tmp_path):
    """save -> load -> step continues at t+1 (the device step
    counter was not restored, so a resumed D re-ran RAdam's warm-up): a
    3 + 3 step run through torch.save / load_state_dict is bit-identical
    to 6 uninterrupted steps, and both match radam.py."""
    shapes = _shapes()
    params, grads = _seq(shapes, 6, 1)
    pa = [p.to(device).requires_grad_(True) for p in params]
    oa = FusedRAdam(pa, 1e-4, weight_decay=0.01)
    for gs in grads:
        for p, g in zip(pa, gs):
            p.grad = g.to(device)
        oa.step()
    pb = [p.to(device).requires_grad_(True) for p in params]
    ob = FusedRAdam(pb, 1e-4, weight_decay=0.01)
    for gs in grads[:3]:
        for p, g in zip(pb, gs):
            p.grad = g.to(device)
        ob.step()
    torch.save({"optimizer": ob.state_dict(), "params": [p.detach().cpu() for p in pb]},
               tmp_path / "D.pth")
    ck = torch.load(tmp_path / "D.pth", weights_only=True)
    pc = [p.to(device).requires_grad_(True) for p in ck["params"]]
    oc = FusedRAdam(pc, 1e-4, weight_decay=0.01)
    oc.load_state_dict(ck["optimizer"])
    assert float(oc.state[pc[0]]["step"]) == 3.0
    for gs in grads[3:]:
        for p, g in zip(pc, gs):
            p.grad = g.to(device)
        oc.step()
    ref = radam_ref(params, grads, wd=0.01)
    for a, c, r in zip(pa, pc, ref):
        assert torch.equal(a, c)
        assert (c.detach().cpu() - r).abs().max().item() <= 1e-6 * r.abs().max().item()
    assert float(oc.state[pc[0]]["step"]) == 6.0


def test_fused_radam_state_dict_leaves_live_counter(device):
    """state_dict() must not freeze the live step: save after 2
    steps, step 3 more, save again -> the second checkpoint holds step 5 and
    the live state still points at the device counter."""
    shapes = _shapes()
    params, grads = _seq(shapes, 5, 2)
    pa = [p.to(device).requires_grad_(True) for p in params]
    oa = FusedRAdam(pa, 1e-4)
    for i, gs in enumerate(grads):
        for p, g in zip(pa, gs):
            p.grad = g.to(device)
        oa.step()
        if i == 1:
            sd1 = oa.state_dict()
    sd2 = oa.state_dict()
    assert all(st["step"] == 2 for st in sd1["state"].values())
    assert all(st["step"] == 5 for st in sd2["state"].values())
    assert isinstance(oa.state[pa[0]]["step"], torch.Tensor)
    assert float(oa.state[pa[0]]["step"]) == 5.0


def test_fused_radam_loads_reference_int_step_state(device):
    """A reference D_*.pth holds radam.py's per-parameter int ``step``
    (radam.py:55): loaded into FusedRAdam it seeds the device counter."""
    from vits_amd.optim import RAdam

    shapes = _shapes()
    params, grads = _seq(shapes, 5, 2)
    pr = [p.clone().requires_grad_(True) for p in params]
    o_cpu = RAdam(pr, 1e-4)          # radam.py semantics on CPU, int steps
    for gs in grads[:2]:
        for p, g in zip(pr, gs):
            p.grad = g
        o_cpu.step()
    sd = o_cpu.state_dict()
    assert isinstance(sd["state"][0]["step"], int)
    pd = [p.detach().to(device).requires_grad_(True) for p in pr]
    od = FusedRAdam(pd, 1e-4)
    od.load_state_dict(sd)
    for gs in grads[2:]:
        for p, g in zip(pd, gs):
            p.grad = g.to(device)
        od.step()
    ref = radam_ref(params, grads)
    for p, r in zip(pd, ref):
        assert (p.detach().cpu() - r).abs().max().item() <= 1e-6 * r.abs().max().item()
    assert float(od.state[pd[0]]["step"]) == 5.0


def test_fused_radam_tensor_lr_reaches_captured_graph(device):
    """lr as a device tensor: a step captured in a hipGraph follows an
    ExponentialLR schedule (a float lr froze at capture)."""
    shapes = _shapes()
    params, grads = _seq(shapes, 4, 3)
    pd = [p.to(device).requires_grad_(True) for p in params]
    lr = torch.tensor(1e-3, device=device, dtype=torch.float64)
    opt = FusedRAdam(pd, lr)
    sched = torch.optim.lr_scheduler.ExponentialLR(opt, gamma=0.5)
    static = [torch.zeros_like(p) for p in pd]
    for p, s in zip(pd, static):
        p.grad = s
    # the first step runs eagerly (state allocation), the rest replay a graph
    for s, g in zip(static, grads[0]):
        s.copy_(g)
    opt.step()
    lrs = [1e-3]
    sched.step()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):  # records, does not run
        opt.step()
    for gs in grads[1:]:
        for s, g in zip(static, gs):
            s.copy_(g.to(device))
        lrs.append(float(opt.param_groups[0]["lr"]))
        graph.replay()
        sched.step()
    torch.cuda.synchronize()
    assert lrs == [1e-3, 5e-4, 2.5e-4, 1.25e-4]
    ref = radam_ref(params, grads, lr=lrs)
    for p, r in zip(pd, ref):
        assert (p.detach().cpu() - r).abs().max().item() <= 1e-6 * r.abs().max().item()


def test_capturable_adamw_tensor_lr_reaches_captured_graph(device):
    """The G optimizer under capture (torch AdamW fused+capturable, lr a
    device tensor): replays follow the schedule like eager float-lr steps."""
    shapes = _shapes()
    params, grads = _seq(shapes, 4, 4)
    lrs = [2e-4 * 0.5 ** i for i in range(4)]
    pe = [p.to(device).requires_grad_(True) for p in params]
    oe = torch.optim.AdamW(pe, 2e-4, betas=(0.8, 0.99), eps=1e-9, weight_decay=0.01, fused=True)
    for lr, gs in zip(lrs, grads):
        oe.param_groups[0]["lr"] = lr
        for p, g in zip(pe, gs):
            p.grad = g.to(device)
        oe.step()
    pc = [p.to(device).requires_grad_(True) for p in params]
    oc = torch.optim.AdamW(pc, torch.tensor(2e-4, device=device), betas=(0.8, 0.99), eps=1e-9,
                           weight_decay=0.01, fused=True, capturable=True)
    sched = torch.optim.lr_scheduler.ExponentialLR(oc, gamma=0.5)
    static = [torch.zeros_like(p) for p in pc]
    for p, s in zip(pc, static):
        p.grad = s
    for s, g in zip(static, grads[0]):
        s.copy_(g.to(device))
    oc.step()
    sched.step()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        oc.step()
    for gs in grads[1:]:
        for s, g in zip(static, gs):
            s.copy_(g.to(device))
        graph.replay()
        sched.step()
    torch.cuda.synchronize()
    for a, b in zip(pe, pc):
        assert (a - b).abs().max().item() <= 1e-6 * a.abs().max().item()
