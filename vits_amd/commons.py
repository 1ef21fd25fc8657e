"""Path / mask / segment helpers (reference ``commons.py``).

Host-side torch code: these run on whatever device their inputs live on and
are not the hot path (the inference engine replaces the one-hot path GEMMs
by ``vits_expand_prior``).  Each function states the reference lines whose
semantics it keeps.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn


def init_weights(m, mean=0.0, std=0.01):
    """commons.py:8-10: N(mean, std) for Conv1d/Linear weights."""
    if isinstance(m, (nn.Conv1d, nn.Linear)):
        m.weight.data.normal_(mean, std)


def get_padding(kernel_size: int, dilation: int = 1) -> int:
    """commons.py:13-14 — 'same' padding of a dilated odd kernel."""
    return int((kernel_size * dilation - dilation) / 2)


def kl_divergence(m_p, logs_p, m_q, logs_q):
    """KL(P||Q) of diagonal Gaussians (commons.py:29-33)."""
    kl = (logs_q - logs_p) - 0.5
    kl = kl + 0.5 * (torch.exp(2.0 * logs_p) + (m_p - m_q) ** 2) * torch.exp(-2.0 * logs_q)
    return kl


def sequence_mask(length: torch.Tensor, max_length=None) -> torch.Tensor:
    """[b] lengths -> bool [b, max_length] (commons.py:120-124)."""
    if max_length is None:
        max_length = length.max()
    pos = torch.arange(int(max_length), dtype=length.dtype, device=length.device)
    return pos.unsqueeze(0) < length.unsqueeze(1)


def _cum_path(duration: torch.Tensor, t_y: int, dtype) -> torch.Tensor:
    """One-hot path [b, t_x, t_y] from durations [b, 1, t_x]: frame y belongs
    to token x iff cum[x-1] <= y < cum[x]."""
    b, _, t_x = duration.shape
    cum = torch.cumsum(duration, -1).reshape(b * t_x)
    upto = sequence_mask(cum, t_y).to(dtype).reshape(b, t_x, t_y)
    prev = F.pad(upto, (0, 0, 1, 0))[:, :-1]
    return upto - prev


def generate_path(duration: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    """duration [b,1,t_x], mask [b,t_y,t_x] -> path [b,t_y,t_x] (commons.py:127-140)."""
    _, t_y, _ = mask.shape
    path = _cum_path(duration, t_y, mask.dtype)
    return path.transpose(1, 2) * mask


def infer_path(duration: torch.Tensor, t_x: int, t_y: int, dtype=torch.float) -> torch.Tensor:
    """Unmasked variant used by EmoVITS.infer (commons.py:143-155)."""
    return _cum_path(duration, int(t_y), dtype).transpose(1, 2)


def slice_segments(x: torch.Tensor, ids_str: torch.Tensor, segment_size: int = 4) -> torch.Tensor:
    """x[i, :, ids[i]:ids[i]+seg] per row (commons.py:47-53), as one gather
    instead of a Python loop over the batch."""
    b, d, t = x.shape
    idx = ids_str.to(device=x.device, dtype=torch.long).view(b, 1, 1) + torch.arange(
        segment_size, device=x.device).view(1, 1, segment_size)
    idx = idx.clamp_(0, max(t - 1, 0)).expand(b, d, segment_size)
    return torch.gather(x, 2, idx)


def rand_slice_segments(x: torch.Tensor, x_lengths=None, segment_size: int = 4,
                        device_rng: bool = False):
    """Random window per row (commons.py:56-63); same RNG draw as the
    reference (one torch.rand([b]) on the host generator).  ``device_rng``
    (set per model by vits_amd.train.TrainStep.capture, for the hipGraph-
    captured step) draws the window starts on the device instead."""
    b, d, t = x.size()
    if x_lengths is None:
        x_lengths = t
    ids_str_max = x_lengths - segment_size + 1
    if device_rng:
        # graph-captured training step: the draw must come from the device
        # generator so every replay re-draws
        r = torch.rand([b], device=x.device)
    else:
        r = torch.rand([b]).to(device=x.device)
    ids_str = (r * ids_str_max).to(dtype=torch.long)
    return slice_segments(x, ids_str, segment_size), ids_str


def gen_sin_table(max_len: int, d_model: int, padding_idx=None) -> torch.Tensor:
    """Sinusoid table [1, max_len, d_model] (commons.py:176-190)."""
    pe = torch.zeros(max_len, d_model)
    position = torch.arange(0, max_len, dtype=torch.float32).unsqueeze(1)
    div_term = torch.exp(
        torch.arange(0, d_model, 2, dtype=torch.float32) * -(np.log(10000.0) / d_model))
    pe[:, 0::2] = torch.sin(position * div_term)
    pe[:, 1::2] = torch.cos(position * div_term)
    if padding_idx is not None:
        pe[padding_idx] = 0.0
    return pe.unsqueeze_(0)


def clip_grad_value_(parameters, clip_value, norm_type=2, as_tensor=False):
    """Clamp grads to +-clip_value and return the total grad norm
    (commons.py:158-173).  The reference syncs the host once per parameter
    (.item() in the loop); here the norm is reduced on the device and read
    back once."""
    if isinstance(parameters, torch.Tensor):
        parameters = [parameters]
    parameters = [p for p in parameters if p.grad is not None]
    norm_type = float(norm_type)
    if not parameters:
        return torch.zeros(()) if as_tensor else 0.0
    grads = [p.grad.detach() for p in parameters]
    if norm_type == 2.0 and grads[0].is_cuda:
        # one multi-tensor launch per dtype/device group instead of one per parameter
        norms = torch.stack([n.float() for n in torch._foreach_norm(grads, 2.0)])
    else:
        norms = torch.stack([g.norm(norm_type).float() for g in grads])
    total = torch.sum(norms ** norm_type) ** (1.0 / norm_type)
    if clip_value is not None:
        cv = float(clip_value)
        torch._foreach_clamp_min_(grads, -cv)
        torch._foreach_clamp_max_(grads, cv)
    # as_tensor: stay on the device (no host sync: the graph-captured step)
    return total if as_tensor else float(total.item())


def subsequent_mask(length: int) -> torch.Tensor:
    return torch.tril(torch.ones(length, length)).unsqueeze(0).unsqueeze(0)


def convert_pad_shape(pad_shape):
    layers = pad_shape[::-1]
    return [item for sublist in layers for item in sublist]


def intersperse(lst, item):
    result = [item] * (len(lst) * 2 + 1)
    result[1::2] = lst
    return result


__all__ = [
    "init_weights", "get_padding", "kl_divergence", "sequence_mask", "generate_path", "infer_path",
    "slice_segments", "rand_slice_segments", "gen_sin_table", "clip_grad_value_", "subsequent_mask",
    "convert_pad_shape", "intersperse", "math",
]
