"""Host-sync-free whole-utterance inference (SynthesizerTrn.infer_bucketed /
capture_infer_bucketed, EmoVITS graph mode) against the eager reference
sequence it replaces: infer_p1 -> w = exp(logw) * rate -> ceil -> y_len via
.item() (the host sync, models.py:547 / infer.py:171) -> infer_path
(commons.py:143-155) -> infer_p2 on exactly y_len frames.

The bucketed path computes durations, y_len and the expansion on the device
(vits_expand_durations), runs the flow and decoder over a static frame
bucket with every conv masked at y_len (and tiles past y_len + 64 skipped),
so each output sample is computed by the same kernels with the same
summation order as the exact-length eager run: the comparisons are
BITWISE (torch.equal on the first y_len * hop samples)."""
import math

import numpy as np
import pytest
import torch

from common import base_model

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def base(device):
    return base_model(device)


def _eager(model, x, emo, sid, noise_full, rate=1.0):
    """The reference's eager sequence (models.py:537-556 with infer_p2's
    pre-scaled noise), on exactly y_len frames."""
    from vits_amd.commons import infer_path

    m_p, s_p, logw, g = model.infer_p1(x, emo, sid)
    w = torch.exp(logw) * rate
    w_ceil = torch.ceil(w)
    y_len = int(torch.clamp_min(torch.sum(w_ceil), 1).item())
    attn = infer_path(w_ceil.float(), x.shape[1], y_len).to(m_p.dtype)
    return model.infer_p2(attn, m_p, s_p, g, noise_full[:, :, :y_len].to(m_p.dtype)), y_len


def _inputs(device, t_x, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(1, t_x, 256, generator=g).to(device)
    emo = torch.randn(1, 1024, generator=g).to(device)
    sid = torch.tensor([int(torch.randint(0, 2048, (1,), generator=g))], device=device)
    return x, emo, sid, g


@pytest.mark.parametrize("t_x,t_y,rate", [(37, 512, 1.0), (100, 1024, 1.3), (12, 256, 0.8)])
def test_infer_bucketed_bitwise_equals_eager(base, device, t_x, t_y, rate):
    x, emo, sid, g = _inputs(device, t_x, t_x)
    noise = (torch.randn(1, 192, t_y, generator=g) * 0.707).to(device)
    ref, y_len = _eager(base, x, emo, sid, noise, rate)
    assert y_len <= t_y
    wav, yl = base.infer_bucketed(x, emo, sid, noise, t_y, length_scale=rate)
    torch.cuda.synchronize()
    assert int(yl[0]) == y_len
    assert wav.shape == (1, 1, t_y * 192)
    assert torch.equal(wav[:, :, :y_len * 192], ref)


def test_infer_bucketed_graph_replay_and_padded_text(base, device):
    """One hipGraph for the whole utterance, text padded to a 64-token
    bucket (masked text encoder / duration predictor): bitwise the eager
    exact-length result, for a long then a short utterance replayed from
    the same graph (stale buffers past y_len must not leak in)."""
    run = base.capture_infer_bucketed(64, 1024, padded_text=True)
    for t_x, seed in ((60, 1), (23, 2)):
        x, emo, sid, g = _inputs(device, t_x, seed)
        noise = (torch.randn(1, 192, 1024, generator=g) * 0.707).to(device)
        ref, y_len = _eager(base, x, emo, sid, noise)
        wav, yl = run(x, emo, sid, noise, x_length=t_x)
        torch.cuda.synchronize()
        assert int(yl[0]) == y_len
        assert torch.equal(wav[:, :, :y_len * 192], ref), t_x


def test_emovits_graph_mode_equals_eager_mode(device, tmp_path):
    """EmoVITS (fp16 model, noise slices of its fixed buffer) in graph mode
    (one replay per utterance) vs its eager mode from the same numpy seed:
    bitwise equal waveforms, and numpy's generator ends in the same state
    (the device draws infer.py:173's randint(len - nl) from raw words of
    numpy's own generator, as numpy's legacy masked rejection does)."""
    from vits_amd.infer import EmoVITS
    from vits_amd.utils import get_hparams_from_dict

    from common import BASE_DATA, BASE_MODEL

    hps = get_hparams_from_dict({"data": {"sampling_rate": 16000, "hop_length": 192,
                                          "text_channels": 256, "n_speakers": 2048,
                                          "noise_scale": 0.707},
                                 "model": dict(BASE_MODEL)})
    model = base_model(device)
    ev = EmoVITS(str(tmp_path / "ckpt.pth"), device, hps=hps, model=model, graph=True)
    x, emo, sid, _ = _inputs(device, 41, 5)
    text = x[0].float().cpu().numpy()
    emo_h = emo.half()
    outs = []
    for graph in (True, False):
        ev.graph = graph
        for seed in (0, 11):
            np.random.seed(seed)
            wav, _ = ev.infer(int(sid), text, emo_h)
            outs.append((wav, np.random.randint(1 << 30)))
    for (wg, ng), (we, ne) in zip(outs[:2], outs[2:]):
        assert wg.shape == we.shape and np.isfinite(wg).all()
        assert np.array_equal(wg, we)
        assert ng == ne
    assert not np.array_equal(outs[0][0], outs[1][0])  # different seeds, different slices


@pytest.mark.gpu
def test_expand_durations_noise_slice_overflow_reads_nothing(device):
    """A y_len whose slice does not fit the flat noise buffer (C * y_len >
    numel; the reference's randint raises) writes z = 0 and flags -1 in the
    extra lens row instead of reading past the buffer."""
    from vits_amd import ops

    B, C, t_x, t_y = 2, 8, 6, 64
    logw = torch.full((B, 1, t_x), math.log(8.0), device=device)  # 48 frames each
    logw[1] = math.log(2.0)                                        # 12 frames
    m_p = torch.randn(B, C, t_x, device=device)
    s_p = torch.rand(B, C, t_x, device=device)
    noise = torch.randn(C * 40, device=device)  # room for 40 frames only
    pool = torch.from_numpy(np.stack([ops.numpy_draw_pool()[0] for _ in range(B)])).to(device)
    z, lens = ops.expand_durations(logw, m_p, s_p, noise, t_y, noise_start=pool,
                                   stage_mult=(1, 2))
    lens = lens.cpu()
    assert lens[0].tolist() == [48, 12] and lens[1].tolist() == [96, 24]
    assert int(lens[2, 0]) == -1 and int(lens[2, 1]) >= 1
    assert torch.count_nonzero(z[0]).item() == 0
    assert torch.count_nonzero(z[1, :, :12]).item() == C * 12
