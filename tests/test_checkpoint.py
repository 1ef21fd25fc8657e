"""Checkpoint I/O and the CPU optimizer as the reference's drivers use them.

``vits_amd.utils`` must serve train_stft.py's own unpacking pattern
(train_stft.py:117-122: ``_, _, epoch_str = utils.load_checkpoint(ckptG,
net_g, optim_g, adapt=hps.adapt)``) for a save/load round trip of G and D
(utils.py:19-57); ``vits_amd.optim.RAdam`` is radam.py's update on CPU.
"""
import os

import pytest
import torch

from common import radam_ref
from test_train import tiny_hps


def _nets_and_optims(seed):
    from vits_amd.optim import RAdam
    from vits_amd.train import build_models

    hps = tiny_hps()
    torch.manual_seed(seed)
    net_g, net_d = build_models(hps, torch.device("cpu"))
    optim_g = torch.optim.AdamW(net_g.parameters(), hps.train.learning_rate,
                                betas=hps.train.betas, eps=hps.train.eps)
    optim_d = RAdam(net_d.parameters(), 1e-4)
    return net_g, net_d, optim_g, optim_d


def _fake_step(net, opt, seed):
    gen = torch.Generator().manual_seed(seed)
    for p in net.parameters():
        p.grad = torch.randn(p.shape, generator=gen) * 1e-2
    opt.step()


def test_checkpoint_round_trip_reference_unpacking(tmp_path):
    from vits_amd import utils

    net_g, net_d, optim_g, optim_d = _nets_and_optims(0)
    _fake_step(net_g, optim_g, 1)
    _fake_step(net_d, optim_d, 2)
    g_path = os.path.join(tmp_path, "G_700.pth")
    d_path = os.path.join(tmp_path, "D_700.pth")
    utils.save_checkpoint(net_g, optim_g, 7, g_path)
    utils.save_checkpoint(net_d, optim_d, 7, d_path)
    assert utils.latest_checkpoint_path(str(tmp_path), "G_*.pth") == g_path

    g2, d2, og2, od2 = _nets_and_optims(5)
    # train_stft.py:117-122, exactly as the reference writes it
    _, _, epoch_str = utils.load_checkpoint(g_path, g2, og2, adapt=False)
    _, _, epoch_str = utils.load_checkpoint(d_path, d2, od2, adapt=False)
    assert epoch_str == 7
    for a, b in zip(net_g.state_dict().values(), g2.state_dict().values()):
        assert torch.equal(a, b)
    for a, b in zip(net_d.state_dict().values(), d2.state_dict().values()):
        assert torch.equal(a, b)
    # optimizer state travelled too: the next step is identical
    _fake_step(net_d, optim_d, 3)
    _fake_step(d2, od2, 3)
    for a, b in zip(net_d.parameters(), d2.parameters()):
        assert torch.equal(a, b)
    assert od2.state[next(iter(d2.parameters()))]["step"] == 2

    # -a/--adapt: weights only, iteration 1 (utils.py:22-27)
    g3, d3, og3, od3 = _nets_and_optims(6)
    _, _, epoch_str = utils.load_checkpoint(d_path, d3, od3, adapt=True)
    assert epoch_str == 1 and len(od3.state) == 0


def test_checkpoint_missing_key_keeps_init(tmp_path):
    """utils.py:33-39: a key absent from the checkpoint keeps the model's
    current value; everything else is loaded."""
    from vits_amd import utils

    net_g, _, optim_g, _ = _nets_and_optims(0)
    sd = net_g.state_dict()
    drop = "emb_g.weight"
    torch.save({"model": {k: v for k, v in sd.items() if k != drop}, "iteration": 3,
                "optimizer": None}, tmp_path / "G_3.pth")
    g2, _, og2, _ = _nets_and_optims(9)
    before = g2.state_dict()[drop].clone()
    _, _, it = utils.load_checkpoint(str(tmp_path / "G_3.pth"), g2, og2)
    assert it == 3
    assert torch.equal(g2.state_dict()[drop], before)
    k = "dec.conv_pre.bias"
    assert torch.equal(g2.state_dict()[k], sd[k])


def test_get_hparams_cli(tmp_path, monkeypatch):
    """utils.py:152-191 flags and the config copy into logs/<model>."""
    import json

    from vits_amd import utils

    cfg = tmp_path / "base.json"
    cfg.write_text(json.dumps({"train": {"seed": 1}, "model": {"n_flows": 4}}))
    monkeypatch.chdir(tmp_path)
    h = utils.get_hparams(argv=["-c", str(cfg), "-m", "exp", "-a"])
    assert h.train.seed == 1 and h.model.n_flows == 4 and h.adapt and not h.use_dur_dis
    assert os.path.isfile(tmp_path / "logs" / "exp" / "config.json")
    assert utils.get_hparams_from_dir(h.model_dir).model.n_flows == 4


@pytest.mark.parametrize("wd", [0.0, 0.01])
def test_cpu_radam_matches_radam_py(wd):
    """vits_amd.optim.RAdam (the CPU D optimizer of the train loop) is
    radam.py: warm-up branch (N_sma < 5 for t <= 5), rectified branch, and
    weight decay applied to the parameter.  torch.optim.RAdam is not (it
    rectifies only when rho > 5 and adds weight decay to the gradient)."""
    from vits_amd.optim import RAdam

    gen = torch.Generator().manual_seed(0)
    shapes = [(16, 8, 3), (5,), (1, 1, 1)]
    params = [torch.randn(*s, generator=gen) for s in shapes]
    grads = [[torch.randn(*s, generator=gen) * 0.1 for s in shapes] for _ in range(9)]
    ps = [p.clone().requires_grad_(True) for p in params]
    opt = RAdam(ps, 1e-3, weight_decay=wd)
    for gs in grads:
        for p, g in zip(ps, gs):
            p.grad = g
        opt.step()
    ref = radam_ref(params, grads, lr=1e-3, wd=wd)
    for p, r in zip(ps, ref):
        assert torch.allclose(p.detach(), r, rtol=0, atol=1e-7 * r.abs().max().item())


def test_tensor_lr_checkpoint_is_portable_and_loads_in_place(tmp_path):
    """a checkpoint written from an optimizer whose lr is a
    tensor (the graph-capturable TrainStep) stores floats, so a float-lr
    optimizer (the reference's) loads it; loading INTO a pinned tensor-lr
    optimizer keeps the lr / initial_lr / moment tensor objects (a captured
    graph reads them) and copies the loaded values in, and a scheduler
    step afterwards continues the loaded sequence in place."""
    from vits_amd import utils

    torch.manual_seed(0)
    w = torch.nn.Parameter(torch.randn(5, 3))
    lr_t = torch.tensor(2e-4)
    opt = torch.optim.AdamW([w], lr_t, betas=(0.8, 0.99), foreach=False)
    sched = torch.optim.lr_scheduler.ExponentialLR(opt, 0.5)
    w.grad = torch.randn(5, 3)
    opt.step()
    sched.step()  # lr 1e-4
    utils.save_checkpoint(torch.nn.Linear(1, 1), opt, 3, str(tmp_path / "G_3.pth"))
    sd = torch.load(tmp_path / "G_3.pth", weights_only=True)["optimizer"]
    assert isinstance(sd["param_groups"][0]["lr"], float)
    assert isinstance(sd["param_groups"][0]["initial_lr"], float)
    # a float-lr optimizer (the reference's AdamW, default foreach) consumes it
    w2 = torch.nn.Parameter(torch.randn(5, 3))
    ref = torch.optim.AdamW([w2], 2e-4, betas=(0.8, 0.99))
    ref.load_state_dict(sd)
    w2.grad = torch.randn(5, 3)
    ref.step()
    assert abs(ref.param_groups[0]["lr"] - 1e-4) < 1e-10  # an fp32 tensor lr, stored as float

    # loading into a pinned tensor-lr optimizer: objects kept, values copied
    w3 = torch.nn.Parameter(torch.randn(5, 3))
    lr3 = torch.tensor(7e-4)
    opt3 = utils.pin_optimizer_state(torch.optim.AdamW([w3], lr3, betas=(0.8, 0.99),
                                                       foreach=False))
    sched3 = torch.optim.lr_scheduler.ExponentialLR(opt3, 0.5)
    w3.grad = torch.randn(5, 3)
    opt3.step()  # creates the moments the "graph" would hold
    m_obj = opt3.state[w3]["exp_avg"]
    init_obj = opt3.param_groups[0]["initial_lr"]
    sd = torch.load(tmp_path / "G_3.pth", weights_only=True)["optimizer"]  # ref.step mutated it
    opt3.load_state_dict(sd)
    assert opt3.param_groups[0]["lr"] is lr3 and abs(float(lr3) - 1e-4) < 1e-10
    assert opt3.param_groups[0]["initial_lr"] is init_obj and abs(float(init_obj) - 2e-4) < 1e-10
    assert opt3.state[w3]["exp_avg"] is m_obj
    assert torch.equal(m_obj, opt.state[w]["exp_avg"])
    sched3.step()
    assert opt3.param_groups[0]["lr"] is lr3 and abs(float(lr3) - 5e-5) < 1e-10
