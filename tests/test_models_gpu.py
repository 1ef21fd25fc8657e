"""End-to-end parity of the HIP inference path against the reference's golden
outputs and the CPU oracle.

Tolerances (fp32 everywhere; the HIP convs are exact-f32 MFMA fmaf chains in
a different summation order than the CPU): per-tensor max error <= 1e-4 of
the tensor's max magnitude for intermediate tensors, and waveform SNR >= 60 dB
(SURVEY.md §7 step 4)."""
import numpy as np
import pytest
import torch

from common import (BASE_MODEL, base_model, golden, oracle_sd, rel_err, snr_db, tiny_cfg,
                    build_model)

pytestmark = pytest.mark.gpu

REL = 1e-4
SNR_DB = 60.0


@pytest.fixture(scope="module")
def base(device):
    return base_model(device)


def T(a, device):
    return torch.from_numpy(np.ascontiguousarray(a)).to(device)


def test_infer_p1_vs_reference(base, device):
    gd = golden("base_infer.npz")
    m_p, s_p, logw, g = base.infer_p1(T(gd["x"], device), T(gd["emo"], device),
                                      T(gd["sid"], device).long())
    assert rel_err(m_p, gd["m_p"]) < REL
    assert rel_err(s_p, gd["s_p"]) < REL
    assert rel_err(logw, gd["logw"]) < REL
    assert rel_err(g, gd["g"]) == 0


def test_infer_p2_vs_reference(base, device):
    gd = golden("base_infer.npz")
    wav = base.infer_p2(T(gd["attn"], device), T(gd["m_p"], device), T(gd["s_p"], device),
                        T(gd["g"], device), T(gd["noise"], device))
    assert wav.shape == gd["wav"].shape
    assert snr_db(wav, gd["wav"]) >= SNR_DB
    assert rel_err(wav, gd["wav"]) < REL
    # flow output on its own
    from vits_amd import engine, ops

    z = ops.expand_prior(T(gd["attn"], device), T(gd["m_p"], device), T(gd["s_p"], device),
                         T(gd["noise"], device))
    engine.get_plan(base.flow, engine.CouplingFlowPlan).run_(z, T(gd["g"], device))
    assert rel_err(z, gd["z"]) < REL


def test_inference_batched_masked_vs_reference(base, device):
    gd = golden("base_inference.npz")
    o, attn, y_mask, (z, z_p, m_e, logs_e) = base.inference(
        T(gd["x"], device), T(gd["x_lengths"], device).long(), T(gd["emo"], device),
        T(gd["sid"], device).long(), noise_scale=float(gd["noise_scale"]),
        noise=T(gd["noise"], device))
    assert torch.equal(attn.cpu(), torch.from_numpy(gd["attn"]))
    assert torch.equal(y_mask.cpu(), torch.from_numpy(gd["y_mask"]))
    assert rel_err(z_p, gd["z_p"]) < REL
    assert rel_err(z, gd["z"]) < REL
    assert snr_db(o, gd["o"]) >= SNR_DB


def test_infer_p2_vs_oracle_longer(base, device):
    """B=2, Tx=40, Ty=200 with ragged durations vs the CPU oracle."""
    from oracle import vits_oracle as V

    torch.manual_seed(0)
    B, Tx = 2, 40
    dur = torch.randint(1, 9, (B, 1, Tx)).float()
    Ty = int(dur.sum(-1).max())
    from vits_amd.commons import infer_path

    attn = torch.cat([infer_path(dur[b:b + 1], Tx, Ty) for b in range(B)], 0)
    m_p = torch.randn(B, 192, Tx)
    s_p = torch.rand(B, 192, Tx) + 0.3
    g = torch.randn(B, 1024) * 0.5
    noise = torch.randn(B, 192, Ty) * 0.7
    torch.set_num_threads(16)
    ref = V.infer_p2(oracle_sd(base), attn, m_p, s_p, g, noise, dict(BASE_MODEL))
    out = base.infer_p2(attn.to(device), m_p.to(device), s_p.to(device), g.to(device),
                        noise.to(device))
    assert snr_db(out, ref) >= SNR_DB
    assert rel_err(out, ref) < REL


def test_full_size_batch_properties(base, device):
    """BASELINE config 2 shape (B=16, Tx=100, Ty=500): size-independent
    properties — finite, |wav| <= 1, and every utterance equals the same
    utterance synthesised alone (batch independence)."""
    torch.manual_seed(1)
    B, Tx, Ty = 16, 100, 500
    from vits_amd.commons import infer_path

    attn = infer_path(torch.full((1, 1, Tx), 5.0), Tx, Ty).expand(B, Ty, Tx).contiguous()
    m_p = torch.randn(B, 192, Tx, device=device)
    s_p = torch.rand(B, 192, Tx, device=device) + 0.3
    g = torch.randn(B, 1024, device=device) * 0.5
    noise = torch.randn(B, 192, Ty, device=device) * 0.7
    attn = attn.to(device)
    out = base.infer_p2(attn, m_p, s_p, g, noise)
    assert out.shape == (B, 1, Ty * 192)
    assert torch.isfinite(out).all() and out.abs().max() <= 1.0
    for b in (0, 7, 15):
        one = base.infer_p2(attn[b:b + 1], m_p[b:b + 1], s_p[b:b + 1], g[b:b + 1], noise[b:b + 1])
        assert torch.equal(one, out[b:b + 1])


def test_hipgraph_replay_matches_eager(base, device):
    gd = golden("base_infer.npz")
    args = [T(gd[k], device) for k in ("attn", "m_p", "s_p", "g", "noise")]
    eager = base.infer_p2(*args)
    Ty, Tx = gd["attn"].shape[1], gd["attn"].shape[2]
    run = base.capture_infer_p2(1, Tx, Ty)
    out = run(*args)
    torch.cuda.synchronize()
    assert torch.equal(out, eager)


def test_mrstft_loss_vs_reference(device):
    from vits_amd.stft_loss import MultiResolutionSTFTLoss

    gd = golden("mrstft.npz")
    loss = MultiResolutionSTFTLoss().to(device)
    y = T(gd["y"], device)
    y_hat = T(gd["y_hat"], device).requires_grad_(True)
    sc, mag, ys, yhs = loss(y, y_hat)
    (sc + mag).backward()
    assert abs(sc.item() - float(gd["sc"])) <= 1e-5 * abs(float(gd["sc"]))
    assert abs(mag.item() - float(gd["mag"])) <= 1e-5 * abs(float(gd["mag"]))
    for i in range(5):
        assert abs(ys[i].double().sum().item() - float(gd[f"y_mag_sum{i}"])) <= 1e-5 * abs(
            float(gd[f"y_mag_sum{i}"]))
        assert abs(yhs[i].double().sum().item() - float(gd[f"y_hat_mag_sum{i}"])) <= 1e-5 * abs(
            float(gd[f"y_hat_mag_sum{i}"]))
    assert rel_err(ys[0][:1], gd["y_mag0"]) < 2e-5
    assert rel_err(yhs[4][:1], gd["y_hat_mag4"]) < 2e-5
    assert rel_err(y_hat.grad, gd["grad_y_hat"]) < 1e-4


def test_training_forward_gpu_vs_reference(device):
    """Tiny-config training forward on the GPU (torch ops + HIP MAS) with the
    reference's recorded noise draws passed explicitly."""
    c = tiny_cfg()
    m = build_model(c["model"], c["data"], device)
    gd = golden("tiny_forward.npz")
    t = {k: torch.from_numpy(v) for k, v in gd.items()}
    # rand_slice_segments draws torch.rand([b]) on the host generator
    orig_rand = torch.rand
    torch.rand = lambda *a, **k: t["rand_slice"].clone()
    try:
        out = m(t["x"].to(device), t["x_lengths"].to(device), t["spec"].to(device),
                t["y_lengths"].to(device), t["emo"].to(device), t["sid"].to(device),
                noise_q=t["noise_q"].to(device), noise_align=t["noise_align"].to(device),
                noise_flow=t["noise_flow"].to(device))
    finally:
        torch.rand = orig_rand
    o, l_length, attn, ids_slice = out[:4]
    assert torch.equal(attn.cpu(), t["attn"])
    assert torch.equal(ids_slice.cpu(), t["ids_slice"])
    assert rel_err(o.detach(), gd["o"]) < 1e-4
    assert rel_err(out[7].detach(), gd["z_q"]) < 1e-4


# --------------------------------------------------------------------------
# module-level parity (base.json shapes, deterministic weights) vs the oracle
# --------------------------------------------------------------------------

def test_posterior_infer_vs_oracle(base, device):
    from oracle import vits_oracle as V

    g = torch.Generator().manual_seed(7)
    spec = torch.rand(2, 513, 123, generator=g)
    n = torch.randn(2, 192, 123, generator=g)
    got = base.enc_q.infer(spec.to(device), n.to(device))
    ref = V.posterior_infer(oracle_sd(base), spec, n, BASE_MODEL["n_layers_q"], 256)
    assert rel_err(got, ref) < REL


def test_wn_infer_vs_oracle(base, device):
    """The flow's WN (cond from g, 4 layers, unmasked infer)."""
    from oracle import vits_oracle as V

    g = torch.Generator().manual_seed(8)
    x = torch.randn(2, 256, 77, generator=g) * 0.5
    gg = torch.randn(2, 1024, generator=g) * 0.5
    wn = base.flow.flows[0].enc
    got = wn.infer(x.to(device), gg.to(device))
    ref = V.wn(oracle_sd(base), "flow.flows.0.enc", x, None, gg, 4, 256, masked=False)
    assert rel_err(got, ref) < REL


@pytest.mark.parametrize("idx", [0, 4, 8, 11])
def test_resblock2_vs_oracle(base, device, idx):
    """ResBlock2 no-grad path (fused HIP convs) for the k=3/7/11 blocks of
    stages 0..3 (C=256..32)."""
    from oracle import vits_oracle as V

    rb = base.dec.resblocks[idx]
    C = rb.convs1[0].in_channels
    g = torch.Generator().manual_seed(idx)
    x = torch.randn(2, C, 301, generator=g) * 0.5
    gg = torch.randn(2, 1024, generator=g) * 0.5
    with torch.no_grad():
        got = rb(x.to(device), gg.to(device))
    ref = V.resblock2(oracle_sd(base), f"dec.resblocks.{idx}", x, gg, rb.kernel_size, rb.dilation)
    assert rel_err(got, ref) < REL


def test_generator_vs_oracle(base, device):
    from oracle import vits_oracle as V

    g = torch.Generator().manual_seed(9)
    z = torch.randn(2, 192, 37, generator=g) * 0.7
    gg = torch.randn(2, 1024, generator=g) * 0.5
    with torch.no_grad():
        got = base.dec(z.to(device), gg.to(device))
    ref = V.generator(oracle_sd(base), z, gg, BASE_MODEL)
    assert got.shape == ref.shape == (2, 1, 37 * 192)
    assert snr_db(got, ref) >= SNR_DB and rel_err(got, ref) < REL


@pytest.mark.parametrize("dt,min_snr", [(torch.bfloat16, 30.0), (torch.float16, 45.0)])
def test_lowp_model_infer_p2_vs_reference(device, dt, min_snr):
    """A bf16 / fp16 model runs its convs on the 16-bit-MFMA kernel variant of
    its type (fp32 activations / accumulation).  Tolerance: waveform SNR
    against the reference's fp32 golden output >= 30 dB for bf16 (measured
    ~40 dB; operands round at 2^-8) and >= 45 dB for fp16 (2^-11)."""
    m = base_model(device).to(dt)
    gd = golden("base_infer.npz")
    wav = m.infer_p2(T(gd["attn"], device), T(gd["m_p"], device), T(gd["s_p"], device),
                     T(gd["g"], device), T(gd["noise"], device))
    assert wav.shape == gd["wav"].shape
    snr = snr_db(wav.float(), gd["wav"])
    print(f"{dt}: SNR {snr:.1f} dB")
    assert snr >= min_snr
    plan = m.dec.__dict__.get("_vits_amd_plan")
    assert plan is not None and plan.conv_pre.wdtype == {torch.bfloat16: 1, torch.float16: 2}[dt]


def test_infer_p1_graph_matches_eager(base, device):
    """capture_infer_p1 (per-length hipGraph used by EmoVITS) replays the same
    kernels: bit-identical to eager infer_p1, also after new inputs."""
    g = torch.Generator().manual_seed(21)
    run = base.capture_infer_p1(37)
    for _ in range(2):
        x = torch.randn(1, 37, 256, generator=g).to(device)
        emo = torch.randn(1, 1024, generator=g).to(device)
        sid = torch.tensor([int(torch.randint(0, 2048, (1,), generator=g))], device=device)
        ref = base.infer_p1(x, emo, sid)
        got = run(x, emo, sid)
        for a, b in zip(got, ref):
            assert torch.equal(a, b)
