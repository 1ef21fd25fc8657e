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

Usage: python tests/golden/make_golden.py
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


def main():
    torch.set_num_threads(8)
    models, stft_loss = _ref()
    if len(sys.argv) > 1 and sys.argv[1] == "mpd":  # only the MPD fixture
        make_mpd(models)
        return
    make_base(models)
    make_tiny(models)
    make_mrstft(stft_loss)
    make_mpd(models)
    with open(os.path.join(HERE, "tiny_config.json"), "w") as f:
        json.dump(dict(model=TINY, data=TINY_DATA), f, indent=1)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
