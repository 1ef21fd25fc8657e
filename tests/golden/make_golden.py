"""Generate the golden fixtures under tests/golden/ FROM THE REFERENCE ITSELF.

Runs only in the build container (it imports the read-only reference from
/root/reference/emotional-vits); the GPU box never runs it.  Weights come
from vits_amd.utils.deterministic_tensor (key-hashed, seed 1234) so no
checkpoint is shipped: tests rebuild the identical weights by key.

Fixtures (npz, float32 unless noted):
  base_infer.npz      configs/base.json model: infer_p1 outputs for
                      x[1,12,256]; infer_p2 with durations 5/token and given
                      noise; the reverse-flow output z.
  base_inference.npz  batched masked `inference` (B=2, x_lengths [12, 9]) with
                      the randn draw recorded.
  tiny_forward.npz    a small-config model (same topology) training `forward`
                      in eval mode (dropout off) with its four RNG draws
                      recorded; `monotonic_align` is supplied by the C oracle
                      (the external package is absent: SURVEY.md §8(c)).
  base_state_dict_shapes.json   reference state_dict keys -> shapes (drop-in
                      checkpoint contract).
  mpd.npz             models.MultiPeriodDiscriminator (train.py's D) on
                      y, y_hat [2, 1, 1201]: every score, per-feature-map
                      sums / abs-sums / shapes, discriminator / generator /
                      feature losses, d(loss_gen + loss_fm)/dy_hat;
                      mpd_state_dict_shapes.json its keys -> shapes.
  mrstft.npz          stft_loss.MultiResolutionSTFTLoss on x,y [2, 9216]:
                      sc, mag, magnitude maps of resolutions 0 and 4
                      (utterance 0), per-resolution sums, d(sc+mag)/dy_hat.
  mwsd.npz            mrd.MultiWaveSTFTDiscriminator (train_stft.py's D) on
                      y, y_hat [2, 1, 3072] and their MR-STFT magnitudes:
                      every score, dL_gen/dy_hat and d/dmag heads, parameter
                      gradient statistics (norm, sum, abs-sum, max) plus the
                      full gradients of the small tensors, the spectral-norm
                      u vectors after one train-mode forward;
                      mwsd_state_dict_shapes.json its keys -> shapes.
  train_step.npz      ONE train_stft.py step (lines 162-236) on a tiny config
                      (p_dropout 0, B=2, Tx 10, Ty 40, 16-frame segments):
                      every RNG draw recorded (rand_slice, align noise,
                      randn_like), losses, G / D gradient norms, per-parameter
                      gradient statistics and post-step parameter statistics
                      (RAdam for D, AdamW for G as the reference builds them);
                      train_step_config.json the config.
  train_step_base.npz the same step at configs/base.json widths (Tx 20,
                      Ty 100); train_step_base_config.json.
  train_step_adv.npz  the tiny step with c_stft = 0 (adversarial, duration
                      and KL losses only); train_step_adv_config.json.
  base_c5.npz         one C5 long-form utterance (Tx=500, Ty=2500) through
                      the reference's bf16 model and its fp32 model:
                      waveform windows / statistics, reference SNR
  base_c1.npz         the C1 headline utterance (configs/base.json, Tx=100,
                      Ty=500, models.py:568-575): infer_p1 / infer_p2 outputs,
                      waveform head / middle windows, per-block rms of the
                      decoder, z statistics; plus SynthesizerTrn.infer at
                      Tx=12 with its noise draw recorded.

Usage: python tests/golden/make_golden.py [mpd|mwsd|train_step|train_step_base|train_step_adv|c1 ...]
"""
from __future__ import annotations

import json
import os
import sys
import types
import warnings

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/emotional-vits"
sys.path.insert(0, ROOT)
warnings.filterwarnings("ignore")

from vits_amd.utils import deterministic_fill_  # noqa: E402

TINY = dict(inter_channels=16, hidden_channels=32, filter_channels=32, n_heads=2, n_layers=2,
            kernel_size=5, p_dropout=0.1, ffn="FFN2", resblock="2",
            resblock_kernel_sizes=[3, 7, 11], resblock_dilation_sizes=[[1, 3, 5]] * 3,
            upsample_rates=[8, 6, 2, 2], upsample_initial_channel=256,
            upsample_kernel_sizes=[16, 12, 4, 4], kernel_size_q=5, n_layers_q=2,
            hidden_size_d=32, kernel_size_d=5, p_dropout_d=0.5, act_func_d="ReLU",
            act_func_params_d={}, use_spectral_norm=False, dilation_rate=[1, 1, 1, 1], n_flows=4,
            gin_channels=32)
TINY_DATA = dict(text_channels=16, spec_channels=33, segment_size=4, n_speakers=4)


def base_cfg():
    with open(os.path.join(REF, "configs", "base.json")) as f:
        return json.load(f)


def _install_mas():
    from oracle import mas as mas_oracle

    mod = types.ModuleType("monotonic_align")

    def maximum_path(neg_cent, mask):
        p = mas_oracle.maximum_path(neg_cent.detach().cpu().float().numpy(),
                                    mask.detach().cpu().float().numpy())
        return torch.from_numpy(p).to(device=neg_cent.device, dtype=neg_cent.dtype)

    mod.maximum_path = maximum_path
    sys.modules["monotonic_align"] = mod


def _ref():
    sys.path.insert(0, REF)
    _install_mas()
    import commons  # noqa: F401
    import models
    import stft_loss

    return models, stft_loss


class RecordRNG:
    """Record every torch.randn_like / torch.rand draw the reference makes
    (randn_like keeps the strides of transposed inputs, so the draws cannot
    be reproduced by a plain torch.randn of the same shape)."""

    def __enter__(self):
        self.draws = []
        self._rl, self._r = torch.randn_like, torch.rand

        def rl(t, *a, **k):
            out = self._rl(t, *a, **k)
            self.draws.append(("randn_like", out.detach().clone().contiguous()))
            return out

        def r(*a, **k):
            out = self._r(*a, **k)
            self.draws.append(("rand", out.detach().clone().contiguous()))
            return out

        torch.randn_like, torch.rand = rl, r
        return self

    def __exit__(self, *exc):
        torch.randn_like, torch.rand = self._rl, self._r
        return False


def np32(t):
    return t.detach().cpu().float().numpy()


def make_base(models):
    cfg = base_cfg()
    m = models.SynthesizerTrn(cfg["data"]["text_channels"], cfg["data"]["filter_length"] // 2 + 1,
                              cfg["train"]["segment_size"] // cfg["data"]["hop_length"],
                              n_speakers=cfg["data"]["n_speakers"], **cfg["model"]).eval()
    deterministic_fill_(m)
    import commons

    g = torch.Generator().manual_seed(1234)
    Tx = 12
    x = torch.randn(1, Tx, 256, generator=g)
    emo = torch.randn(1, 1024, generator=g)
    sid = torch.tensor([7])
    with torch.no_grad():
        m_p, s_p, logw, gg = m.infer_p1(x, emo, sid)
        w = torch.full((1, 1, Tx), 5.0)
        Ty = 5 * Tx
        attn = commons.infer_path(w, Tx, Ty)
        noise = torch.randn(1, 192, Ty, generator=g) * 0.707
        wav = m.infer_p2(attn, m_p, s_p, gg, noise)
        mp_e = torch.matmul(attn, m_p.transpose(1, 2)).transpose(1, 2)
        sp_e = torch.matmul(attn, s_p.transpose(1, 2)).transpose(1, 2)
        z = m.flow.infer(mp_e + noise * sp_e, g=gg, reverse=True)
    with open(os.path.join(HERE, "base_state_dict_shapes.json"), "w") as f:
        json.dump({k: list(v.shape) for k, v in m.state_dict().items()}, f, indent=0)
    np.savez_compressed(os.path.join(HERE, "base_infer.npz"), x=np32(x), emo=np32(emo),
                        sid=sid.numpy(), m_p=np32(m_p), s_p=np32(s_p), logw=np32(logw), g=np32(gg),
                        attn=np32(attn), noise=np32(noise), z=np32(z), wav=np32(wav))

    # batched masked inference
    B, Tx2 = 2, 12
    xb = torch.randn(B, Tx2, 256, generator=g)
    emob = torch.randn(B, 1024, generator=g)
    sidb = torch.tensor([3, 1500])
    xl = torch.tensor([12, 9])
    torch.manual_seed(4321)
    with torch.no_grad(), RecordRNG() as rec:
        o, attn_b, y_mask, (zb, zpb, meb, lsb) = m.inference(xb, xl, emob, sidb, noise_scale=0.667,
                                                             length_scale=1.0)
    assert [k for k, _ in rec.draws] == ["randn_like"]
    noise_b = rec.draws[0][1]
    np.savez_compressed(os.path.join(HERE, "base_inference.npz"), x=np32(xb), emo=np32(emob),
                        sid=sidb.numpy(), x_lengths=xl.numpy(), noise=np32(noise_b), o=np32(o),
                        attn=np32(attn_b), y_mask=np32(y_mask), z=np32(zb), z_p=np32(zpb),
                        m_e=np32(meb), logs_e=np32(lsb), noise_scale=np.float32(0.667))
    return m


def make_tiny(models):
    m = models.SynthesizerTrn(TINY_DATA["text_channels"], TINY_DATA["spec_channels"],
                              TINY_DATA["segment_size"], n_speakers=TINY_DATA["n_speakers"],
                              **TINY).eval()
    deterministic_fill_(m)
    g = torch.Generator().manual_seed(99)
    B, Tx, Ty = 2, 7, 20
    x = torch.randn(B, Tx, TINY_DATA["text_channels"], generator=g)
    xl = torch.tensor([7, 5])
    spec = torch.rand(B, TINY_DATA["spec_channels"], Ty, generator=g)
    yl = torch.tensor([20, 16])
    emo = torch.randn(B, 1024, generator=g)
    sid = torch.tensor([1, 3])
    torch.manual_seed(2024)
    with torch.no_grad(), RecordRNG() as rec:
        out = m(x, xl, spec, yl, emo, sid)
    # the four RNG draws of forward in eval mode, in order
    assert [k for k, _ in rec.draws] == ["randn_like", "randn_like", "rand", "randn_like"]
    n_q, n_al, r_slice, n_fl = (t for _, t in rec.draws)
    o, l_length, attn, ids_slice, x_mask, y_mask, (z, z_p, m_p, logs_p, m_q, logs_q), z_q, \
        (xh, logw_, logw) = out
    np.savez_compressed(
        os.path.join(HERE, "tiny_forward.npz"), x=np32(x), x_lengths=xl.numpy(), spec=np32(spec),
        y_lengths=yl.numpy(), emo=np32(emo), sid=sid.numpy(), noise_q=np32(n_q),
        noise_align=np32(n_al), rand_slice=np32(r_slice), noise_flow=np32(n_fl), o=np32(o),
        l_length=np32(l_length), attn=np32(attn), ids_slice=ids_slice.numpy(), z=np32(z),
        z_p=np32(z_p), m_p=np32(m_p), logs_p=np32(logs_p), m_q=np32(m_q), logs_q=np32(logs_q),
        z_q=np32(z_q), x_hidden=np32(xh), logw_=np32(logw_), logw=np32(logw),
        align_noise=np.float32(0.01))
    return m


def make_mrstft(stft_loss):
    g = torch.Generator().manual_seed(5)
    y = (torch.randn(2, 9216, generator=g) * 0.3).clamp(-1, 1)
    y_hat = (torch.randn(2, 9216, generator=g) * 0.3).clamp(-1, 1).requires_grad_(True)
    loss = stft_loss.MultiResolutionSTFTLoss()
    # train_stft.py:195 calls mstft_loss(y, y_hat)
    sc, mag, ys, yhs = loss(y, y_hat)
    (sc + mag).backward()
    arrs = dict(y=np32(y), y_hat=np32(y_hat.detach()), sc=np32(sc), mag=np32(mag),
                grad_y_hat=np32(y_hat.grad))
    for i, (a, b) in enumerate(zip(ys, yhs)):
        if i in (0, 4):  # full maps for the smallest/largest resolution
            arrs[f"y_mag{i}"] = np32(a[:1])
            arrs[f"y_hat_mag{i}"] = np32(b[:1])
        arrs[f"y_mag_sum{i}"] = np.float64(a.double().sum())
        arrs[f"y_hat_mag_sum{i}"] = np.float64(b.double().sum())
    np.savez_compressed(os.path.join(HERE, "mrstft.npz"), **arrs)


def make_mpd(models):
    import losses

    d = models.MultiPeriodDiscriminator(False)
    deterministic_fill_(d)
    with open(os.path.join(HERE, "mpd_state_dict_shapes.json"), "w") as f:
        json.dump({k: list(v.shape) for k, v in d.state_dict().items()}, f, indent=0)
    g = torch.Generator().manual_seed(7)
    # 1201 samples: not a multiple of any period (reflect-pad path of every P)
    y = (torch.randn(2, 1, 1201, generator=g) * 0.3).clamp(-1, 1)
    y_hat = (torch.randn(2, 1, 1201, generator=g) * 0.3).clamp(-1, 1).requires_grad_(True)
    y_d_rs, y_d_gs, fmap_rs, fmap_gs = d(y, y_hat)
    loss_disc, _, _ = losses.discriminator_loss(y_d_rs, [t.detach() for t in y_d_gs])
    loss_fm = losses.feature_loss(fmap_rs, fmap_gs)
    loss_gen, _ = losses.generator_loss(y_d_gs)
    (loss_gen + loss_fm).backward()
    arrs = dict(y=np32(y), y_hat=np32(y_hat.detach()), loss_disc=np32(loss_disc),
                loss_fm=np32(loss_fm), loss_gen=np32(loss_gen), grad_y_hat=np32(y_hat.grad))
    for i in range(len(y_d_rs)):
        arrs[f"r{i}"] = np32(y_d_rs[i])
        arrs[f"g{i}"] = np32(y_d_gs[i])
        for j, (a, b) in enumerate(zip(fmap_rs[i], fmap_gs[i])):
            arrs[f"fr{i}_{j}_shape"] = np.array(a.shape, np.int64)
            arrs[f"fr{i}_{j}_sum"] = np.float64(a.double().sum())
            arrs[f"fr{i}_{j}_abs"] = np.float64(a.double().abs().sum())
            arrs[f"fg{i}_{j}_sum"] = np.float64(b.double().sum())
    np.savez_compressed(os.path.join(HERE, "mpd.npz"), **arrs)


def _sn_state(d, pre=""):
    """Every spectral-norm u vector (concatenated, in state_dict order) and
    v checksum of a module: {pre}sn_keys, {pre}sn_u, {pre}sn_vsum."""
    keys, us, vs = [], [], []
    sd = d.state_dict()
    for k, b in sd.items():
        if k.endswith("weight_u"):
            keys.append(k[:-len("_u")])
            us.append(np32(b))
            vs.append(float(sd[k[:-1] + "v"].double().sum()))
    return {pre + "sn_keys": np.array(keys), pre + "sn_u": np.concatenate(us),
            pre + "sn_vsum": np.array(vs, np.float64)}


def _param_stats(grads, params=None, before=None, pre="", full_max=64):
    """Per-parameter gradient statistics packed into a few arrays:
    {pre}keys, {pre}stats [n, 4] = (grad norm, grad sum, update sum, update
    abs-sum) in float64, and the full gradients of tensors with <= full_max
    elements concatenated ({pre}small_keys / {pre}small_grad)."""
    keys, stats, skeys, sgrads = [], [], [], []
    for k, gr in grads.items():
        keys.append(k)
        row = [gr.double().norm().item(), gr.double().sum().item(), 0.0, 0.0]
        if params is not None:
            delta = params[k].detach().double() - before[k].double()
            row[2], row[3] = delta.sum().item(), delta.abs().sum().item()
        stats.append(row)
        if gr.numel() <= full_max:
            skeys.append(k)
            sgrads.append(np32(gr).ravel())
    return {pre + "keys": np.array(keys), pre + "stats": np.array(stats, np.float64),
            pre + "small_keys": np.array(skeys), pre + "small_grad": np.concatenate(sgrads)}


MWSD_L = 3072  # 16 frames x hop 192: the shortest segment every MWSD branch accepts


def mwsd_inputs():
    """y [2, 1, 3072] and its five MR-STFT magnitudes (the D inputs of
    train_stft.py:198), from a seeded host generator."""
    g = torch.Generator().manual_seed(31)
    y = (torch.randn(2, 1, MWSD_L, generator=g) * 0.2).clamp(-1, 1)
    return y


def make_mwsd(stft_loss):
    """mrd.MultiWaveSTFTDiscriminator (mrd.py:200-236) in training mode: the
    ten scores, the spectral-norm state after the forward (one power
    iteration per layer), d(generator_loss)/d(input) for the waveform and
    every magnitude map, and every parameter gradient (norm, sum; full for
    the small ones)."""
    import losses
    import mrd

    from vits_amd.utils import deterministic_fill_sn_

    d = mrd.MultiWaveSTFTDiscriminator()
    deterministic_fill_(d)
    deterministic_fill_sn_(d)
    d.train()
    with open(os.path.join(HERE, "mwsd_state_dict_shapes.json"), "w") as f:
        json.dump({k: list(v.shape) for k, v in d.state_dict().items()}, f, indent=0)
    y = mwsd_inputs().requires_grad_(True)
    loss = stft_loss.MultiResolutionSTFTLoss()
    with torch.no_grad():
        _, _, mags, _ = loss(y.detach().squeeze(1), y.detach().squeeze(1))
    mags = [m.clone().requires_grad_(True) for m in mags]
    outs = d(y, mags)
    lg, _ = losses.generator_loss(outs)
    lg.backward()
    arrs = dict(y=np32(y.detach()), loss_gen=np32(lg), grad_y=np32(y.grad))
    for i, m in enumerate(mags):
        arrs[f"mag{i}"] = np32(m.detach())
        # the magnitude gradients: norm / sum and the first 4 frames in full
        arrs[f"grad_mag{i}_head"] = np32(m.grad[:, :, :4])
        arrs[f"grad_mag{i}_stats"] = np.array([m.grad.double().norm().item(),
                                               m.grad.double().sum().item()])
    for i, o in enumerate(outs):
        arrs[f"out{i}"] = np32(o.detach())
    arrs.update(_param_stats({k: p.grad for k, p in d.named_parameters()}, full_max=256))
    arrs.update(_sn_state(d))
    np.savez_compressed(os.path.join(HERE, "mwsd.npz"), **arrs)


# one train_stft.py step (train_stft.py:162-236) on the tiny generator + the
# real MWSD discriminator, fp32 (fp16_run off: no autocast, GradScaler
# disabled); dropout probabilities 0 so that train mode is deterministic apart
# from the four recorded RNG draws
TRAIN_STEP = dict(seg_frames=16, B=2, Tx=10, Ty=40, x_lengths=[10, 8], y_lengths=[40, 34],
                  sid=[1, 3], hop=192, lr_g=2e-4, betas=[0.8, 0.99], eps=1e-9, wd=0.01, lr_d=1e-4,
                  c_stft=25.0, c_dur=2.0, c_kl=1.0, c_kl_q=0.01, align_noise=1e-2,
                  align_noise_decay=1e-6)


# the same step at configs/base.json widths (B=2, Tx 20, Ty 100): every HIP
# training kernel at the benchmarked channel counts
TRAIN_STEP_BASE = dict(TRAIN_STEP, Tx=20, Ty=100, x_lengths=[20, 16], y_lengths=[100, 84])
# the tiny step with the MR-STFT loss weight 0 (train_stft.py:225, c_stft):
# the L1 of log STFT magnitudes weights every bin by 1 / |X|, and any
# waveform has near-zero bins, so under fp16 the waveform-path gradients are
# dominated by rounding noise (tools/chaos_probe.py); without it the fp16
# step's gradients are stable enough to be pinned per parameter
TRAIN_STEP_ADV = dict(TRAIN_STEP, c_stft=0.0)
TRAIN_VARIANTS = {
    "train_step": (TRAIN_STEP, "tiny"),
    "train_step_base": (TRAIN_STEP_BASE, "base"),
    "train_step_adv": (TRAIN_STEP_ADV, "tiny"),
}


def train_step_inputs(c=None, data=None):
    c = TRAIN_STEP if c is None else c
    data = TINY_DATA if data is None else data
    g = torch.Generator().manual_seed(404)
    B, Tx, Ty = c["B"], c["Tx"], c["Ty"]
    x = torch.randn(B, Tx, data["text_channels"], generator=g)
    spec = torch.rand(B, data["spec_channels"], Ty, generator=g)
    y = (torch.randn(B, 1, Ty * c["hop"], generator=g) * 0.2).clamp(-1, 1)
    emo = torch.randn(B, 1024, generator=g)
    xl, yl = torch.tensor(c["x_lengths"]), torch.tensor(c["y_lengths"])
    for b in range(B):  # zero padding beyond each length (as the collate pads)
        x[b, xl[b]:] = 0
        spec[b, :, yl[b]:] = 0
        y[b, :, yl[b] * c["hop"]:] = 0
    return x, xl, spec, yl, y, yl * c["hop"], emo, torch.tensor(c["sid"])


def make_train_step(models, stft_loss, name="train_step"):
    import commons
    import losses
    import mrd
    import radam

    from vits_amd.utils import deterministic_fill_sn_

    c, widths = TRAIN_VARIANTS[name]
    if widths == "tiny":
        cfg, data = dict(TINY, p_dropout=0.0, p_dropout_d=0.0), TINY_DATA
    else:
        bc = base_cfg()
        cfg = dict(bc["model"], p_dropout=0.0, p_dropout_d=0.0)
        data = dict(text_channels=bc["data"]["text_channels"],
                    spec_channels=bc["data"]["filter_length"] // 2 + 1, segment_size=c["seg_frames"],
                    n_speakers=bc["data"]["n_speakers"])
    net_g = models.SynthesizerTrn(data["text_channels"], data["spec_channels"],
                                  c["seg_frames"], n_speakers=data["n_speakers"],
                                  align_noise=c["align_noise"],
                                  align_noise_decay=c["align_noise_decay"], **cfg)
    deterministic_fill_(net_g)
    net_d = mrd.MultiWaveSTFTDiscriminator()
    deterministic_fill_(net_d)
    deterministic_fill_sn_(net_d)
    net_g.train()
    net_d.train()
    mstft = stft_loss.MultiResolutionSTFTLoss()
    optim_g = torch.optim.AdamW(net_g.parameters(), c["lr_g"], betas=c["betas"],
                                weight_decay=c["wd"], eps=c["eps"])
    optim_d = radam.RAdam(net_d.parameters(), c["lr_d"])
    g0 = {k: p.detach().clone() for k, p in net_g.named_parameters()}
    d0 = {k: p.detach().clone() for k, p in net_d.named_parameters()}
    x, xl, spec, sl, y, yl, emo, sid = train_step_inputs(c, data)
    seg = c["seg_frames"]
    torch.manual_seed(777)
    with RecordRNG() as rec:
        (y_hat, l_length, attn, ids_slice, x_mask, z_mask, (z, z_p, m_p, logs_p, m_q, logs_q),
         z_q, _) = net_g(x, xl, spec, sl, emo, sid)
    assert [k for k, _ in rec.draws] == ["randn_like", "randn_like", "rand", "randn_like"]
    # train_stft.py:193-215 (the logging mels of :173-191 change no loss)
    y_s = commons.slice_segments(y, ids_slice * c["hop"], seg * c["hop"])
    sc_loss, mag_loss, y_mag, y_hat_mag = mstft(y_s.squeeze(1), y_hat.squeeze(1))
    y_d_hat_r = net_d(y_s, y_mag)
    y_d_hat_g = net_d(y_hat.detach(), [t.detach() for t in y_hat_mag])
    loss_disc, losses_r, losses_g = losses.discriminator_loss(y_d_hat_r, y_d_hat_g)
    optim_d.zero_grad()
    loss_disc.backward()
    grad_norm_d = commons.clip_grad_value_(net_d.parameters(), None)
    d_grads = {k: p.grad.detach().clone() for k, p in net_d.named_parameters()}
    optim_d.step()
    # train_stft.py:217-236
    y_d_hat_g2 = net_d(y_hat, y_hat_mag)
    loss_dur = torch.sum(l_length.float()) * c["c_dur"]
    loss_stft = (sc_loss.float() + mag_loss.float()) * c["c_stft"]
    loss_kl = losses.kl_loss(z_p, logs_q, m_p, logs_p, z_mask) * c["c_kl"]
    loss_kl_q = losses.kl_loss(z_q, logs_p, m_q, logs_q, z_mask) * c["c_kl_q"]
    loss_gen, _ = losses.generator_loss(y_d_hat_g2)
    loss_gen_all = loss_gen + loss_stft + loss_dur + loss_kl + loss_kl_q
    optim_g.zero_grad()
    loss_gen_all.backward()
    grad_norm_g = commons.clip_grad_value_(net_g.parameters(), None)
    g_grads = {k: p.grad.detach().clone() for k, p in net_g.named_parameters()
               if p.grad is not None}
    optim_g.step()

    n_q, n_al, r_slice, n_fl = (t for _, t in rec.draws)
    arrs = dict(x=np32(x), x_lengths=xl.numpy(), spec=np32(spec), y_lengths=sl.numpy(),
                y=np32(y), wav_lengths=yl.numpy(), emo=np32(emo), sid=sid.numpy(),
                noise_q=np32(n_q), noise_align=np32(n_al), rand_slice=np32(r_slice),
                noise_flow=np32(n_fl), attn=np32(attn), ids_slice=ids_slice.numpy(),
                y_hat=np32(y_hat), l_length=np32(l_length), sc_loss=np32(sc_loss),
                mag_loss=np32(mag_loss), loss_disc=np32(loss_disc),
                losses_disc_r=np.array(losses_r, np.float64),
                losses_disc_g=np.array(losses_g, np.float64), loss_gen=np32(loss_gen),
                loss_stft=np32(loss_stft), loss_dur=np32(loss_dur), loss_kl=np32(loss_kl),
                loss_kl_q=np32(loss_kl_q), loss_gen_all=np32(loss_gen_all),
                grad_norm_d=np.float64(grad_norm_d), grad_norm_g=np.float64(grad_norm_g))
    for pre, grads, before, net in (("g_", g_grads, g0, net_g), ("d_", d_grads, d0, net_d)):
        arrs.update(_param_stats(grads, dict(net.named_parameters()), before, pre))
    arrs.update(_sn_state(net_d, "d_"))
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **arrs)
    with open(os.path.join(HERE, name + "_config.json"), "w") as f:
        json.dump(dict(step=c, model=cfg, data=data), f, indent=1)


def c1_inputs():
    """BASELINE C1: one utterance, Tx=100, 5 frames/token ->
    Ty=500 (96,000 samples), sid 1, noise randn * 0.707, seeded host
    generator 1234."""
    g = torch.Generator().manual_seed(1234)
    x = torch.randn(1, 100, 256, generator=g)
    emo = torch.randn(1, 1024, generator=g)
    noise = torch.randn(1, 192, 500, generator=g) * 0.707
    return x, emo, torch.tensor([1]), noise


def make_c1(models, m=None):
    """The headline utterance from the reference (models.py:558-575, the
    EmoVITS call pattern at Tx=100/Ty=500): full infer_p1 outputs, checksums
    and two 8192-sample windows of the 96,000-sample waveform, per-stage
    statistics of the reverse flow.  Inputs are regenerated from the seed
    (their checksums are stored to prove it).  Plus SynthesizerTrn.infer (the
    single-call API, models.py:537-556) at Tx=12 with its randn_like draw."""
    import commons

    if m is None:
        cfg = base_cfg()
        m = models.SynthesizerTrn(cfg["data"]["text_channels"],
                                  cfg["data"]["filter_length"] // 2 + 1,
                                  cfg["train"]["segment_size"] // cfg["data"]["hop_length"],
                                  n_speakers=cfg["data"]["n_speakers"], **cfg["model"]).eval()
        deterministic_fill_(m)
    x, emo, sid, noise = c1_inputs()
    with torch.no_grad():
        m_p, s_p, logw, gg = m.infer_p1(x, emo, sid)
        attn = commons.infer_path(torch.full((1, 1, 100), 5.0), 100, 500)
        wav = m.infer_p2(attn, m_p, s_p, gg, noise)
        mp_e = torch.matmul(attn, m_p.transpose(1, 2)).transpose(1, 2)
        sp_e = torch.matmul(attn, s_p.transpose(1, 2)).transpose(1, 2)
        z = m.flow.infer(mp_e + noise * sp_e, g=gg, reverse=True)
    w = wav.double().flatten()
    arrs = dict(in_sums=np.array([x.double().sum(), emo.double().sum(), noise.double().sum()]),
                m_p=np32(m_p), s_p=np32(s_p), logw=np32(logw),
                wav_head=np32(wav[0, 0, :8192]), wav_mid=np32(wav[0, 0, 48000:48000 + 8192]),
                wav_stats=np.array([w.sum(), w.abs().sum(), (w * w).sum(), w.abs().max()]),
                wav_block_rms=np32(wav[0, 0].view(-1, 192).pow(2).mean(1).sqrt()),
                z_stats=np.array([z.double().sum(), z.double().abs().sum(),
                                  (z.double() ** 2).sum()]),
                z_frame_rms=np32(z[0].pow(2).mean(0).sqrt()))
    # the single-call API with its noise draw
    g2 = torch.Generator().manual_seed(55)
    x2 = torch.randn(1, 12, 256, generator=g2)
    emo2 = torch.randn(1, 1024, generator=g2)
    torch.manual_seed(66)
    with torch.no_grad(), RecordRNG() as rec:
        o2 = m.infer(x2, emo2, torch.tensor([5]), noise_scale=0.707, length_scale=1.0)
    assert [k for k, _ in rec.draws] == ["randn_like"]
    arrs.update(infer_x=np32(x2), infer_emo=np32(emo2), infer_sid=np.array([5]),
                infer_noise=np32(rec.draws[0][1]), infer_o=np32(o2))
    np.savez_compressed(os.path.join(HERE, "base_c1.npz"), **arrs)


def c5_inputs():
    """One BASELINE C5 utterance (Tx=500, 5 frames per token -> Ty=2500,
    480,000 samples): bench.make_inputs(1, 500, 2500, seed=4321)."""
    g = torch.Generator().manual_seed(4321)
    Tx, Ty = 500, 2500
    dur = torch.full((1, 1, Tx), float(Ty // Tx))
    m_p = torch.randn(1, 192, Tx, generator=g)
    s_p = torch.rand(1, 192, Tx, generator=g) + 0.3
    gg = torch.randn(1, 1024, generator=g) * 0.5
    noise = torch.randn(1, 192, Ty, generator=g) * 0.707
    return dur, m_p, s_p, gg, noise


def make_c5(models):
    """The C5 long-form utterance through the reference's own bf16 model
    (models.py:568-575 after model.to(torch.bfloat16), torch-CPU bf16
    convolutions) and its fp32 model: windows, statistics and per-block rms
    of both waveforms, plus the reference's bf16-vs-fp32 SNR - the yardstick
    the HIP bf16 path is held to (tests/test_configs_gpu.py)."""
    import commons

    cfg = base_cfg()
    m = models.SynthesizerTrn(cfg["data"]["text_channels"],
                              cfg["data"]["filter_length"] // 2 + 1,
                              cfg["train"]["segment_size"] // cfg["data"]["hop_length"],
                              n_speakers=cfg["data"]["n_speakers"], **cfg["model"]).eval()
    deterministic_fill_(m)
    dur, m_p, s_p, gg, noise = c5_inputs()
    attn = commons.infer_path(dur, 500, 2500)
    with torch.no_grad():
        w32 = m.infer_p2(attn, m_p, s_p, gg, noise).float()
        m16 = m.to(torch.bfloat16)
        w16 = m16.infer_p2(*(t.to(torch.bfloat16) for t in (attn, m_p, s_p, gg, noise))).float()

    def snr(a, b):
        a, b = a.double().flatten(), b.double().flatten()
        return float(10 * torch.log10((b * b).sum() / ((a - b) ** 2).sum()))

    arrs = dict(in_sums=np.array([m_p.double().sum(), s_p.double().sum(), gg.double().sum(),
                                  noise.double().sum()]),
                ref_snr_bf16_vs_fp32=np.float64(snr(w16, w32)))
    for tag, w in (("w16", w16), ("w32", w32)):
        wd = w.double().flatten()
        arrs[tag + "_stats"] = np.array([wd.sum(), wd.abs().sum(), (wd * wd).sum(),
                                         wd.abs().max()])
        arrs[tag + "_block_rms"] = np32(w[0, 0].view(-1, 1920).pow(2).mean(1).sqrt())
        for name, start in (("head", 0), ("mid", 240000), ("tail", 480000 - 16384)):
            arrs[f"{tag}_{name}"] = np32(w[0, 0, start:start + 16384])
    np.savez_compressed(os.path.join(HERE, "base_c5.npz"), **arrs)
    print("C5 reference bf16 vs fp32 SNR %.2f dB" % arrs["ref_snr_bf16_vs_fp32"])


def main():
    torch.set_num_threads(8)
    models, stft_loss = _ref()
    if len(sys.argv) > 1:  # only the named fixtures
        for name in sys.argv[1:]:
            {"mpd": lambda: make_mpd(models), "mwsd": lambda: make_mwsd(stft_loss),
             "train_step": lambda: make_train_step(models, stft_loss),
             "train_step_base": lambda: make_train_step(models, stft_loss, "train_step_base"),
             "train_step_adv": lambda: make_train_step(models, stft_loss, "train_step_adv"),
             "c1": lambda: make_c1(models), "c5": lambda: make_c5(models)}[name]()
        return
    m = make_base(models)
    make_c1(models, m)
    make_c5(models)
    make_tiny(models)
    make_mrstft(stft_loss)
    make_mpd(models)
    make_mwsd(stft_loss)
    for name in TRAIN_VARIANTS:
        make_train_step(models, stft_loss, name)
    with open(os.path.join(HERE, "tiny_config.json"), "w") as f:
        json.dump(dict(model=TINY, data=TINY_DATA), f, indent=1)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
