"""CPU checks of the host-side modules: drop-in state_dict contract, the
training forward (PyTorch ops under autograd) against the reference's own
outputs, and the no-fallback rule for the inference path."""
import json
import os

import numpy as np
import pytest
import torch

from common import BASE_DATA, BASE_MODEL, GOLDEN, build_model, golden, rel_err, tiny_cfg


class Replay:
    """Replays the reference's recorded randn_like / rand draws in order."""

    def __init__(self, draws):
        self.draws = list(draws)

    def __enter__(self):
        self._rl, self._r = torch.randn_like, torch.rand

        def nxt(kind, shape):
            k, t = self.draws.pop(0)
            assert k == kind and tuple(t.shape) == tuple(shape), (k, kind, t.shape, shape)
            return t.clone()

        torch.randn_like = lambda t, *a, **k: nxt("randn_like", t.shape).to(t.dtype)
        torch.rand = lambda *shape, **k: nxt("rand", shape[0] if len(shape) == 1 and isinstance(
            shape[0], (list, tuple, torch.Size)) else shape)
        return self

    def __exit__(self, *exc):
        torch.randn_like, torch.rand = self._rl, self._r
        return False


def test_state_dict_matches_reference_keys_and_shapes():
    with open(os.path.join(GOLDEN, "base_state_dict_shapes.json")) as f:
        ref = json.load(f)
    m = build_model(BASE_MODEL, BASE_DATA, fill=False)
    ours = {k: list(v.shape) for k, v in m.state_dict().items()}
    assert ours == ref
    assert len(ours) == 699


def _mas_oracle(neg_cent, mask):
    from oracle import mas as mas_oracle

    p = mas_oracle.maximum_path(neg_cent.detach().cpu().float().numpy(),
                                mask.detach().cpu().float().numpy())
    return torch.from_numpy(p).to(device=neg_cent.device, dtype=neg_cent.dtype)


def _neg_cent_oracle(z_p, m_p, logs_p):
    from oracle.vits_oracle import neg_cent

    return neg_cent(z_p.detach().float(), m_p.detach().float(), logs_p.detach().float())


def test_training_forward_matches_reference(monkeypatch):
    import vits_amd.models as vm

    monkeypatch.setattr(vm, "maximum_path", _mas_oracle)
    monkeypatch.setattr(vm, "neg_cent_scores", _neg_cent_oracle)
    c = tiny_cfg()
    m = build_model(c["model"], c["data"])
    gd = golden("tiny_forward.npz")
    t = {k: torch.from_numpy(v) for k, v in gd.items()}
    draws = [("randn_like", t["noise_q"]), ("randn_like", t["noise_align"]),
             ("rand", t["rand_slice"]), ("randn_like", t["noise_flow"])]
    # grad enabled: the training forward is the autograd path (no-grad decoder
    # calls are inference and go to the HIP engine)
    with Replay(draws):
        out = m(t["x"], t["x_lengths"], t["spec"], t["y_lengths"], t["emo"], t["sid"])
    o, l_length, attn, ids_slice, x_mask, y_mask, (z, z_p, m_p, logs_p, m_q, logs_q), z_q, \
        (xh, logw_, logw) = out
    assert np.array_equal(attn.numpy(), gd["attn"])
    assert np.array_equal(ids_slice.numpy(), gd["ids_slice"])
    for name, val in [("o", o), ("l_length", l_length), ("z", z), ("z_p", z_p), ("m_p", m_p),
                      ("logs_p", logs_p), ("m_q", m_q), ("logs_q", logs_q), ("z_q", z_q),
                      ("x_hidden", xh), ("logw_", logw_), ("logw", logw)]:
        assert rel_err(val.detach(), gd[name]) < 1e-5, name


def test_training_forward_backward_runs(monkeypatch):
    import vits_amd.models as vm

    monkeypatch.setattr(vm, "maximum_path", _mas_oracle)
    monkeypatch.setattr(vm, "neg_cent_scores", _neg_cent_oracle)
    c = tiny_cfg()
    m = build_model(c["model"], c["data"]).train()
    gd = golden("tiny_forward.npz")
    t = {k: torch.from_numpy(v) for k, v in gd.items()}
    out = m(t["x"], t["x_lengths"], t["spec"], t["y_lengths"], t["emo"], t["sid"])
    loss = out[0].pow(2).mean() + out[1].sum()
    loss.backward()
    grads = [p.grad for p in m.parameters() if p.grad is not None]
    assert len(grads) > 100 and all(torch.isfinite(g).all() for g in grads)


def test_inference_path_has_no_cpu_fallback():
    from vits_amd._lib import VitsAmdError

    c = tiny_cfg()
    m = build_model(c["model"], c["data"])
    x = torch.randn(1, 5, c["data"]["text_channels"])
    with pytest.raises(VitsAmdError):
        m.infer_p1(x, torch.randn(1, 1024), torch.tensor([1]))
    with pytest.raises(VitsAmdError):
        m.infer_p2(torch.zeros(1, 10, 5), torch.zeros(1, 16, 5), torch.ones(1, 16, 5),
                   torch.zeros(1, 32), torch.zeros(1, 16, 10))
    from vits_amd.monotonic_align import maximum_path

    with pytest.raises(VitsAmdError):
        maximum_path(torch.zeros(1, 4, 2), torch.ones(1, 4, 2))


def test_generator_no_grad_cpu_raises_but_grad_path_runs():
    """No-grad Generator calls are inference -> HIP only (raise off-GPU); the
    autograd (training) path runs PyTorch ops and must match the oracle."""
    from vits_amd._lib import VitsAmdError
    from oracle import vits_oracle as V
    from common import oracle_sd

    c = tiny_cfg()
    m = build_model(c["model"], c["data"])
    z = torch.randn(1, c["model"]["inter_channels"], 4)
    g = torch.randn(1, c["model"]["gin_channels"])
    with torch.no_grad(), pytest.raises(VitsAmdError):
        m.dec(z, g)
    got = m.dec(z, g)  # grad enabled, params require grad -> training path
    assert got.requires_grad
    with torch.no_grad():
        ref = V.generator(oracle_sd(m), z, g, c["model"])
    assert rel_err(got.detach(), ref) < 1e-5


def test_commons_paths():
    from vits_amd import commons

    d = torch.tensor([[[2.0, 1.0, 3.0]]])
    p = commons.infer_path(d, 3, 6)
    assert p.shape == (1, 6, 3)
    assert p[0].argmax(1).tolist() == [0, 0, 1, 2, 2, 2]
    mask = torch.ones(1, 6, 3)
    assert torch.equal(commons.generate_path(d, mask), p)
    x = torch.arange(2 * 3 * 10).float().view(2, 3, 10)
    seg = commons.slice_segments(x, torch.tensor([1, 5]), 4)
    assert torch.equal(seg[0], x[0, :, 1:5]) and torch.equal(seg[1], x[1, :, 5:9])
