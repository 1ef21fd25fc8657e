"""The BASELINE.json configurations themselves, on the GPU.

* C1 (the headline utterance, Tx=100 -> Ty=500, 96,000 samples) against the
  reference's own outputs recorded by tests/golden/make_golden.py::make_c1:
  infer_p1 outputs, two 8192-sample windows + checksums of the waveform,
  per-block RMS, reverse-flow statistics; plus SynthesizerTrn.infer (the
  single-call API, models.py:537-556) with its recorded noise draw.
* C3 (train_stft step, batch 64, one GPU): the base-config step captured
  into one hipGraph and replayed.
* C5 (long-form, B=4, Tx=500, Ty=2500 = 30 s per utterance, bf16 model,
  hipGraph): against the fp32 HIP output of the same inputs.

Tolerances: fp32 paths as tests/test_models_gpu.py (rel 1e-4, SNR >= 60 dB);
C5 bf16 waveform SNR >= 35 dB vs fp32 (measured ~39 dB with 16-bit decoder
activations, ~41 dB with fp32 ones; bf16 operands round at 2^-8)."""
import numpy as np
import pytest
import torch

from common import base_model, golden, rel_err, snr_db

pytestmark = pytest.mark.gpu


def c1_inputs():
    """Same generator calls as make_golden.c1_inputs (checked by in_sums)."""
    g = torch.Generator().manual_seed(1234)
    x = torch.randn(1, 100, 256, generator=g)
    emo = torch.randn(1, 1024, generator=g)
    noise = torch.randn(1, 192, 500, generator=g) * 0.707
    return x, emo, torch.tensor([1]), noise


@pytest.fixture(scope="module")
def base(device):
    return base_model(device)


def test_c1_headline_utterance_vs_reference(base, device):
    from vits_amd.commons import infer_path

    gd = golden("base_c1.npz")
    x, emo, sid, noise = c1_inputs()
    sums = np.array([x.double().sum(), emo.double().sum(), noise.double().sum()])
    assert np.array_equal(sums, gd["in_sums"]), "input regeneration drifted"
    m_p, s_p, logw, g = base.infer_p1(x.to(device), emo.to(device), sid.to(device))
    assert rel_err(m_p, gd["m_p"]) < 1e-4
    assert rel_err(s_p, gd["s_p"]) < 1e-4
    assert rel_err(logw, gd["logw"]) < 1e-4
    attn = infer_path(torch.full((1, 1, 100), 5.0), 100, 500).to(device)
    wav = base.infer_p2(attn, m_p, s_p, g, noise.to(device)).cpu()
    assert wav.shape == (1, 1, 96000)
    for name, sl in (("wav_head", slice(0, 8192)), ("wav_mid", slice(48000, 48000 + 8192))):
        assert snr_db(wav[0, 0, sl], gd[name]) >= 60.0, name
        assert rel_err(wav[0, 0, sl], gd[name]) < 1e-4, name
    w = wav.double().flatten()
    ref = gd["wav_stats"]
    got = np.array([w.sum(), w.abs().sum(), (w * w).sum(), w.abs().max()])
    # sum of a zero-mean signal: compare on the abs-sum scale
    assert abs(got[0] - ref[0]) <= 1e-5 * ref[1]
    assert np.all(np.abs(got[1:] - ref[1:]) <= 1e-4 * np.abs(ref[1:]))
    rms = wav[0, 0].view(-1, 192).pow(2).mean(1).sqrt().numpy()
    assert np.abs(rms - gd["wav_block_rms"]).max() <= 1e-4 * gd["wav_block_rms"].max()


def test_c1_single_call_infer_vs_reference(base, device):
    gd = golden("base_c1.npz")
    o = base.infer(torch.from_numpy(gd["infer_x"]).to(device),
                   torch.from_numpy(gd["infer_emo"]).to(device),
                   torch.from_numpy(gd["infer_sid"]).to(device), noise_scale=0.707,
                   noise=torch.from_numpy(gd["infer_noise"]).to(device))
    assert o.shape == gd["infer_o"].shape
    assert snr_db(o, gd["infer_o"]) >= 60.0
    assert rel_err(o, gd["infer_o"]) < 1e-4


def test_c5_longform_bf16_vs_reference_bf16_model(base, device):
    """One C5 utterance (Tx=500, Ty=2500, 480,000 samples) against the
    REFERENCE's own bf16 model (models.py after model.to(torch.bfloat16),
    recorded on CPU: tests/golden/base_c5.npz) and its fp32 model.
    * fp32 HIP vs reference fp32: SNR >= 60 dB, as C1.
    * bf16 HIP vs reference fp32: no worse than the reference's own bf16
      model is (its SNR vs fp32, 37.6 dB, minus 3 dB).
    * bf16 HIP vs reference bf16: two independent bf16 roundings of the
      same network, each ~38 dB from fp32; their noise powers add, so the
      bar is the reference's SNR minus 6 dB.
    Windows: head / middle / tail, 16,384 samples each."""
    from bench import make_inputs

    gd = golden("base_c5.npz")
    inputs = make_inputs(1, 500, 2500, device, seed=4321)
    sums = np.array([inputs[i].double().sum().item() for i in (1, 2, 3, 4)])
    assert np.allclose(sums, gd["in_sums"], rtol=0, atol=1e-6 * np.abs(gd["in_sums"]).max()), \
        "input regeneration drifted"
    with torch.no_grad():
        w32 = base.infer_p2(*inputs).float().cpu()
        m16 = base_model(device).to(torch.bfloat16)
        run = m16.capture_infer_p2(1, 500, 2500)
        w16 = run(*inputs).float().cpu()
    torch.cuda.synchronize()
    ref_snr = float(gd["ref_snr_bf16_vs_fp32"])

    def cat(w):
        return torch.cat([w[0, 0, s:s + 16384] for s in (0, 240000, 480000 - 16384)])

    def cat_ref(tag):
        return torch.from_numpy(np.concatenate([gd[f"{tag}_{n}"] for n in ("head", "mid", "tail")]))

    s32 = snr_db(cat(w32), cat_ref("w32"))
    s16_32 = snr_db(cat(w16), cat_ref("w32"))
    s16_16 = snr_db(cat(w16), cat_ref("w16"))
    print(f"C5: fp32 vs ref fp32 {s32:.1f} dB; bf16 vs ref fp32 {s16_32:.1f} dB "
          f"(reference bf16: {ref_snr:.1f} dB); bf16 vs ref bf16 {s16_16:.1f} dB")
    assert s32 >= 60.0
    assert s16_32 >= ref_snr - 3.0
    assert s16_16 >= ref_snr - 6.0
    # loudness envelope (per 1920-sample block rms) of the bf16 waveform
    rms = w16[0, 0].view(-1, 1920).pow(2).mean(1).sqrt().numpy()
    assert np.abs(rms - gd["w16_block_rms"]).max() <= 0.05 * gd["w16_block_rms"].max()


def test_c5_longform_bf16_graph_vs_fp32(base, device):
    """BASELINE C5 shape: B=4, Tx=500, Ty=2500 (480,000 samples each), bf16
    model replayed from one hipGraph, vs the fp32 HIP output."""
    from bench import make_inputs

    B, Tx, Ty = 4, 500, 2500
    inputs = make_inputs(B, Tx, Ty, device, seed=4321)
    with torch.no_grad():
        ref = base.infer_p2(*inputs).float()
        m16 = base_model(device).to(torch.bfloat16)
        run = m16.capture_infer_p2(B, Tx, Ty)
        out = run(*inputs).float().clone()
        eager = m16.infer_p2(*inputs).float()
    torch.cuda.synchronize()
    assert out.shape == (B, 1, Ty * 192)
    assert torch.isfinite(out).all() and out.abs().max() <= 1.0
    assert torch.equal(out, eager)  # graph replay == eager, bit for bit
    for b in range(B):
        s = snr_db(out[b], ref[b])
        print(f"C5 utt {b}: bf16 vs fp32 SNR {s:.1f} dB")
        assert s >= 35.0


def test_c3_train_stft_step_batch64_captured(device):
    """BASELINE C3: the base-config train_stft step at batch 64 on one GPU,
    fp16 autocast, captured into one hipGraph and replayed: finite losses,
    both networks move, the replay repeats the captured step."""
    from vits_amd.train import TrainStep, build_models, default_hps, synthetic_batch

    hps = default_hps()
    torch.manual_seed(1234)
    net_g, net_d = build_models(hps, device)
    st = TrainStep(hps, net_g, net_d, device, capturable=True)
    st.scaler = torch.amp.GradScaler("cuda", init_scale=64.0)
    batch = [t.to(device) for t in synthetic_batch(hps, 64, seed=0)]
    st.capture(batch, warmup=1)
    g0 = [p.detach().clone() for p in list(net_g.parameters())[:60]]
    d0 = [p.detach().clone() for p in list(net_d.parameters())[:60]]
    outs = [{k: v.clone() for k, v in st.replay().items()} for _ in range(2)]
    torch.cuda.synchronize()
    for out in outs:
        for k in ("loss_disc", "loss_gen_all", "loss_stft", "loss_kl"):
            assert torch.isfinite(out[k]), k
    assert any(not torch.equal(a, b) for a, b in zip(g0, net_g.parameters()))
    assert any(not torch.equal(a, b) for a, b in zip(d0, net_d.parameters()))
    assert torch.cuda.max_memory_allocated(device) < 120 * 2 ** 30
