"""Pin the CPU oracles: against the reference's own outputs (golden fixtures
generated from emotional-vits by tests/golden/make_golden.py) and, for the
absent monotonic_align package, against brute-force enumeration."""
import numpy as np
import pytest
import torch

from common import BASE_MODEL, base_model, golden, oracle_sd, rel_err
from oracle import mas as mas_oracle
from oracle import vits_oracle as V

# oracle vs reference on CPU fp32: same torch ops, same order -> ~bit-exact;
# the only differences are weight-norm folding placement (1 ulp level)
TOL = 2e-5


@pytest.fixture(scope="module")
def base_sd():
    torch.set_num_threads(8)
    return oracle_sd(base_model())


def test_mas_bruteforce_small():
    rng = np.random.default_rng(0)
    for _ in range(400):
        ty = int(rng.integers(1, 11))
        tx = int(rng.integers(1, min(ty, 6) + 1))
        v = rng.standard_normal((1, ty + 2, tx + 1)).astype(np.float32)
        p = mas_oracle.maximum_path_lengths(v, np.array([ty]), np.array([tx]))[0]
        # structure: exactly one 1 per valid frame, none outside
        assert (p[:ty].sum(1) == 1).all() and p[ty:].sum() == 0 and p[:, tx:].sum() == 0
        idx = p[:ty, :tx].argmax(1)
        assert idx[0] == 0 and idx[-1] == tx - 1
        assert np.all(np.diff(idx) >= 0) and np.all(np.diff(idx) <= 1)
        best, paths = mas_oracle.brute_force(v[0, :ty, :tx], ty, tx)
        s = float(np.sum(v[0, np.arange(ty), idx].astype(np.float64)))
        assert abs(s - best) < 1e-4


def test_mas_tie_rule():
    # all-equal scores: every monotone path ties; the strict '<' in the
    # backtrack keeps the index until forced (idx == y), so walking back from
    # the last frame the last token absorbs every spare frame: y -> min(y, t_x-1)
    ty, tx = 9, 4
    v = np.zeros((1, ty, tx), np.float32)
    p = mas_oracle.maximum_path_lengths(v, np.array([ty]), np.array([tx]))[0]
    idx = p.argmax(1)
    assert list(idx) == [0, 1, 2, 3, 3, 3, 3, 3, 3]


def test_mas_mask_lengths():
    rng = np.random.default_rng(3)
    nc = rng.standard_normal((3, 30, 8)).astype(np.float32)
    mask = np.zeros_like(nc)
    for b, (tt, ts) in enumerate([(30, 8), (17, 5), (8, 8)]):
        mask[b, :tt, :ts] = 1
    p1 = mas_oracle.maximum_path(nc, mask)
    p2 = mas_oracle.maximum_path_lengths(nc, np.array([30, 17, 8]), np.array([8, 5, 8]))
    assert np.array_equal(p1, p2)
    assert p1[1, 17:].sum() == 0 and p1[1, :, 5:].sum() == 0


def test_oracle_infer_p1_p2_vs_reference(base_sd):
    gd = golden("base_infer.npz")
    cfg = dict(BASE_MODEL)
    m_p, s_p, logw, g = V.infer_p1(base_sd, torch.from_numpy(gd["x"]), torch.from_numpy(gd["emo"]),
                                   torch.from_numpy(gd["sid"]), cfg)
    assert rel_err(m_p, gd["m_p"]) < TOL
    assert rel_err(s_p, gd["s_p"]) < TOL
    assert rel_err(logw, gd["logw"]) < TOL
    assert rel_err(g, gd["g"]) == 0
    wav = V.infer_p2(base_sd, torch.from_numpy(gd["attn"]), torch.from_numpy(gd["m_p"]),
                     torch.from_numpy(gd["s_p"]), torch.from_numpy(gd["g"]),
                     torch.from_numpy(gd["noise"]), cfg)
    assert rel_err(wav, gd["wav"]) < TOL


def test_oracle_inference_vs_reference(base_sd):
    gd = golden("base_inference.npz")
    o, attn, y_mask, (z, z_p, m_e, logs_e) = V.inference(
        base_sd, torch.from_numpy(gd["x"]), torch.from_numpy(gd["x_lengths"]),
        torch.from_numpy(gd["emo"]), torch.from_numpy(gd["sid"]), torch.from_numpy(gd["noise"]),
        dict(BASE_MODEL), noise_scale=float(gd["noise_scale"]))
    assert np.array_equal(attn.numpy(), gd["attn"])
    assert np.array_equal(y_mask.numpy(), gd["y_mask"])
    assert rel_err(z_p, gd["z_p"]) < TOL
    assert rel_err(z, gd["z"]) < TOL
    assert rel_err(o, gd["o"]) < TOL


def test_mel_filterbank_matches_transformers_slaney():
    """librosa is absent; cross-check our Slaney restatement against the
    independent implementation in transformers.audio_utils (parity otherwise
    unpinned: SURVEY.md §8(c) A21)."""
    tr = pytest.importorskip("transformers.audio_utils")
    from vits_amd.mel_processing import mel_filterbank

    ours = mel_filterbank(16000, 1024, 80, 0.0, None)
    theirs = tr.mel_filter_bank(num_frequency_bins=513, num_mel_filters=80, min_frequency=0.0,
                                max_frequency=8000.0, sampling_rate=16000, norm="slaney",
                                mel_scale="slaney").T
    assert ours.shape == theirs.shape == (80, 513)
    assert np.abs(ours - theirs).max() < 1e-6 * max(1.0, np.abs(theirs).max())
