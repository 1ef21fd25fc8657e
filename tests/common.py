"""Shared helpers for the test suite (configs, fixtures, model builders)."""
import json
import math
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")

# configs/base.json "model" section + data fields used to build SynthesizerTrn
BASE_MODEL = dict(inter_channels=192, hidden_channels=256, filter_channels=512, n_heads=2,
                  n_layers=6, kernel_size=5, p_dropout=0.1, ffn="FFN2", resblock="2",
                  resblock_kernel_sizes=[3, 7, 11],
                  resblock_dilation_sizes=[[1, 3, 5], [1, 3, 5], [1, 3, 5]],
                  upsample_rates=[8, 6, 2, 2], upsample_initial_channel=512,
                  upsample_kernel_sizes=[16, 12, 4, 4], kernel_size_q=5, n_layers_q=16,
                  hidden_size_d=256, kernel_size_d=5, p_dropout_d=0.5, act_func_d="ReLU",
                  act_func_params_d={}, use_spectral_norm=False, dilation_rate=[1, 1, 1, 1],
                  n_flows=4, gin_channels=1024)
BASE_DATA = dict(text_channels=256, spec_channels=513, segment_size=48, n_speakers=2048)


def golden(name):
    return dict(np.load(os.path.join(GOLDEN, name), allow_pickle=False))


def tiny_cfg():
    with open(os.path.join(GOLDEN, "tiny_config.json")) as f:
        return json.load(f)


def build_model(cfg_model, cfg_data, device="cpu", fill=True):
    from vits_amd.models import SynthesizerTrn
    from vits_amd.utils import deterministic_fill_

    m = SynthesizerTrn(cfg_data["text_channels"], cfg_data["spec_channels"],
                       cfg_data["segment_size"], n_speakers=cfg_data["n_speakers"], **cfg_model)
    m = m.eval()
    if fill:
        deterministic_fill_(m)
    return m.to(device)


def base_model(device="cpu"):
    return build_model(BASE_MODEL, BASE_DATA, device)


def tiny_model(device="cpu"):
    c = tiny_cfg()
    return build_model(c["model"], c["data"], device)


def oracle_sd(model):
    from oracle.vits_oracle import SD

    return SD({k: v.detach().cpu() for k, v in model.state_dict().items()})


def rel_err(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return ((a - b).abs().max() / (b.abs().max() + 1e-30)).item()


def snr_db(a, ref):
    a = torch.as_tensor(a).double().cpu().flatten()
    ref = torch.as_tensor(ref).double().cpu().flatten()
    noise = ((a - ref) ** 2).sum().item()
    sig = (ref ** 2).sum().item()
    if noise == 0:
        return float("inf")
    return 10 * np.log10(sig / noise)


def radam_ref(params, grads_seq, lr=1e-4, b1=0.9, b2=0.999, eps=1e-8, wd=0.0, t0=0, state=None):
    """radam.py:35-99 restated in the reference's arithmetic (fp32 tensors,
    Python-double scalars).  ``lr`` may be a list (one value per step, an
    lr scheduler's sequence); ``t0``/``state`` continue from a saved step."""
    ps = [p.float().clone() for p in params]
    if state is None:
        m = [torch.zeros_like(p) for p in ps]
        v = [torch.zeros_like(p) for p in ps]
    else:
        m, v = [x.clone() for x in state[0]], [x.clone() for x in state[1]]
    for i_step, grads in enumerate(grads_seq):
        t = t0 + i_step + 1
        lr_t = lr[i_step] if isinstance(lr, (list, tuple)) else lr
        b2t = b2 ** t
        nmax = 2 / (1 - b2) - 1
        n = nmax - 2 * t * b2t / (1 - b2t)
        if n >= 5:
            step = math.sqrt((1 - b2t) * (n - 4) / (nmax - 4) * (n - 2) / n * nmax
                             / (nmax - 2)) / (1 - b1 ** t)
        else:
            step = 1.0 / (1 - b1 ** t)
        for i, g in enumerate(grads):
            g = g.float()
            v[i].mul_(b2).addcmul_(g, g, value=1 - b2)
            m[i].mul_(b1).add_(g, alpha=1 - b1)
            if wd:
                ps[i].add_(ps[i], alpha=-wd * lr_t)
            if n >= 5:
                ps[i].addcdiv_(m[i], v[i].sqrt().add_(eps), value=-step * lr_t)
            else:
                ps[i].add_(m[i], alpha=-step * lr_t)
    return ps
