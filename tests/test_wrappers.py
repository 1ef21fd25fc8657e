"""Inference wrappers: export.load_model (greedy soup), EmoVITS, VITSWrap."""
import json
import os

import numpy as np
import pytest
import torch

from common import build_model, tiny_cfg

HERE = os.path.dirname(os.path.abspath(__file__))


def _write_ckpts(tmp_path, n=3):
    c = tiny_cfg()
    hps = {"train": {"segment_size": c["data"]["segment_size"] * 192},
           "data": {"text_channels": c["data"]["text_channels"],
                    "filter_length": (c["data"]["spec_channels"] - 1) * 2, "hop_length": 192,
                    "n_speakers": c["data"]["n_speakers"], "sampling_rate": 16000,
                    "noise_scale": 0.707},
           "model": c["model"]}
    with open(tmp_path / "config.json", "w") as f:
        json.dump(hps, f)
    sds = []
    for i in range(n):
        m = build_model(c["model"], c["data"], fill=False)
        from vits_amd.utils import deterministic_fill_

        deterministic_fill_(m, seed=100 + i)
        torch.save({"model": m.state_dict(), "iteration": i}, tmp_path / f"G_{(i + 1) * 1000}.pth")
        sds.append(m.state_dict())
    return hps, sds


def test_load_model_greedy_soup(tmp_path):
    from vits_amd.export import load_model

    _, sds = _write_ckpts(tmp_path, 3)
    m = load_model(str(tmp_path), greedy=5)
    sd = m.state_dict()
    k = "dec.conv_pre.weight"
    want = (sds[0][k] + sds[1][k] + sds[2][k]) / 3
    # reference order: last file first, then the others in sorted order
    assert torch.allclose(sd[k], want, atol=1e-6)
    m1 = load_model(str(tmp_path / "G_3000.pth"))
    assert torch.equal(m1.state_dict()[k], sds[2][k])


def test_wav_header():
    from vits_amd.vits_wrap import _gen_wav_header

    h = _gen_wav_header(100, 16000, 16)
    assert len(h) == 44 and h[:4] == b"RIFF" and h[8:12] == b"WAVE" and h[36:40] == b"data"


@pytest.mark.gpu
def test_emovits_and_vitswrap(tmp_path, device):
    from vits_amd.infer import EmoVITS
    from vits_amd.vits_wrap import VITSWrap

    _write_ckpts(tmp_path, 1)
    c = tiny_cfg()
    np.random.seed(0)
    emo_bank = np.random.randn(3, 1024).astype(np.float32)
    emo_bank.tofile(tmp_path / "1.emo")
    with open(tmp_path / "spk.map", "w") as f:
        f.write("7 1\n")
    tts = EmoVITS(str(tmp_path / "G_1000.pth"), device)
    assert tts.spkid_mapping == {7: 1}
    text = np.random.randn(9, c["data"]["text_channels"]).astype(np.float32)
    wav, emo = tts.infer(7, text, None)
    assert wav.dtype == np.float32 and wav.ndim == 1 and len(wav) % 192 == 0 and len(wav) > 0
    assert np.isfinite(wav).all() and np.abs(wav).max() <= 1.0

    class Parser:
        max_utt_length = 10

        def __call__(self, utt_id, text):
            return utt_id, text, np.random.randn(max(1, len(text)), c["data"]["text_channels"]).astype(np.float32)

    wrap = VITSWrap(textparser=Parser(), speecher=tts)
    out = wrap.speaking({"text": "abcdefghij。klmnopq", "spkid": 1, "sampling_rate": 22050, "pitch": 1.2})
    assert out["sr"] == 22050 and out["wav"][:4] == b"RIFF"
    assert len(out["segment_info"]) == 2 and out["rtf"] > 0


@pytest.mark.gpu
def test_emovits_graph_cache_matches_eager(tmp_path, device):
    """EmoVITS(graph_cache>0) replays per-length hipGraphs of infer_p1: same
    waveform as the eager path for the same noise offset."""
    from vits_amd.infer import EmoVITS

    _write_ckpts(tmp_path, 1)
    c = tiny_cfg()
    text = np.random.RandomState(0).randn(11, c["data"]["text_channels"]).astype(np.float32)
    outs = []
    tts = EmoVITS(str(tmp_path / "G_1000.pth"), device, graph_cache=0)
    for gc in (0, 4):
        tts.graph_cache = gc  # same model and noise buffer, eager then graph
        np.random.seed(5)
        emo = torch.zeros(1, 1024)
        wav, _ = tts.infer(1, text, emo)
        outs.append(wav)
    assert outs[0].shape == outs[1].shape and np.array_equal(outs[0], outs[1])


def test_bench_gpus_flag_launches_ranks():
    """bench.py --gpus 2 outside torchrun starts two ranks itself (a child
    torch.distributed.run; gloo in --dry-run) and rank 0 reports the
    whole-job fields: n_gpus 2, global_batch 2 x batch, value over both."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(HERE)
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run",
                        "--steps", "3", "--warmup", "1", "--batch", "5"], capture_output=True,
                       text=True, timeout=300, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["rank_seen"] == 0
    assert line["config"]["global_batch"] == 10
    assert line["config"]["parallelism"] == "replicas x2"
    one = line["value"] / 2
    assert line["value"] == pytest.approx(3 * 5 * 500 * 192 * 2 / (line["ms_per_step"] * 3 / 1e3),
                                          rel=1e-2) and one > 0
