"""Building blocks of the VITS generator (reference ``modules.py``).

Parameter names and shapes are the reference's (legacy weight-norm
``weight_g``/``weight_v``), so reference checkpoints load unchanged.

Two execution modes per block:
* ``forward`` — the training path: PyTorch-ROCm ops under autograd (the
  fused HIP kernels are forward-only; backward kernels are a §8(f) "next"
  item).  Semantics follow the cited reference lines exactly.
* ``infer`` — the inference path: lowered to libvits_amd kernels through
  ``vits_amd.engine`` (see there); no torch compute op runs.
"""
from __future__ import annotations

import torch
from torch import nn
from torch.nn import functional as F
from torch.nn.utils import weight_norm, remove_weight_norm  # noqa: F401  (legacy names)

from . import train_ops
from .commons import get_padding, init_weights

LRELU_SLOPE = 0.1


class LayerNorm(nn.Module):
    """Channel LayerNorm on [B, C, T] (modules.py:33-44)."""

    def __init__(self, channels, eps=1e-5):
        super().__init__()
        self.channels = channels
        self.eps = eps
        self.gamma = nn.Parameter(torch.ones(channels))
        self.beta = nn.Parameter(torch.zeros(channels))

    def forward(self, x):
        y = F.layer_norm(x.transpose(1, -1), (self.channels,), self.gamma, self.beta, self.eps)
        return y.transpose(1, -1)


class WN(nn.Module):
    """Gated dilated-conv stack (modules.py:93-182)."""

    def __init__(self, hidden_channels, kernel_size, dilation_rate, n_layers, gin_channels=0,
                 p_dropout=0):
        super().__init__()
        assert kernel_size % 2 == 1
        self.hidden_channels = hidden_channels
        self.kernel_size = (kernel_size,)
        self.dilation_rate = dilation_rate
        self.n_layers = n_layers
        self.gin_channels = gin_channels
        self.p_dropout = p_dropout
        self.in_layers = nn.ModuleList()
        self.res_skip_layers = nn.ModuleList()
        self.drop = nn.Dropout(p_dropout)
        if gin_channels != 0:
            self.cond_layer = weight_norm(nn.Linear(gin_channels, 2 * hidden_channels * n_layers))
        for i in range(n_layers):
            dilation = dilation_rate ** i
            padding = int((kernel_size * dilation - dilation) / 2)
            self.in_layers.append(weight_norm(
                nn.Conv1d(hidden_channels, 2 * hidden_channels, kernel_size, dilation=dilation,
                          padding=padding)))
            self.in_layers[-1]._vits_gate = True  # feeds only the gate (train_ops.conv1d_gate)
            rs = 2 * hidden_channels if i < n_layers - 1 else hidden_channels
            self.res_skip_layers.append(weight_norm(nn.Conv1d(hidden_channels, rs, 1)))

    def _gate(self, x_in, g, i):
        H = self.hidden_channels
        return train_ops.gate(x_in, None if g is None else g[:, i * 2 * H:(i + 1) * 2 * H])

    def forward(self, x, x_mask, g=None, out16=False, x16=None, **kwargs):
        """out16: return the output rounded to the 16-bit autocast type when
        the fused path applies (for a caller whose only use of it is an
        autocast conv, which would round it there); x16: x already rounded
        (train_ops.mask_cast), the first in_layer's input."""
        H = self.hidden_channels
        output = None  # zeros_like(x), materialised on first use
        g32 = None
        H2 = 2 * H
        if self.gin_channels != 0:
            g = train_ops.linear(self.cond_layer, g)
            g32 = train_ops.cond_f32(g)  # one cast for every layer's fused gate
            if g32 is not None:  # the layers' slices, with a one-launch backward
                g32 = train_ops.split_cols(g32, self.n_layers, H2)
        # x rounded to the conv dtype (by the caller, then by WNUpdate16)
        x16 = x16 if x16 is not None and x16.shape == x.shape else None
        for i in range(self.n_layers):
            xi = x if x16 is None else x16
            g_l = g[:, i * H2:(i + 1) * H2] if self.gin_channels else None
            # in_layer conv + gate as one launch on the fp16 training path
            if g32 is not None:
                acts = train_ops.conv1d_gate(self.in_layers[i], xi, g32[i], g16=g_l)
            else:
                acts = train_ops.conv1d_gate(self.in_layers[i], xi, g_l)
            if acts is None:
                acts = self._gate(train_ops.conv1d(self.in_layers[i], xi),
                                  g if self.gin_channels else None, i)
            acts = self.drop(acts)
            rs = train_ops.conv1d(self.res_skip_layers[i], acts)
            if i < self.n_layers - 1:
                # x = (x + rs[:, :H]) * x_mask ; output = output + rs[:, H:]
                # (one kernel each way on the fp16 training path)
                upd = train_ops.wn_update(x, rs, x_mask, output)
                if upd is not None:
                    x, x16, output = upd
                else:
                    x16 = None
                    x = (x + rs[:, :H]) * x_mask
                    output = (torch.zeros_like(x) if output is None else output) + rs[:, H:]
            else:
                if out16:
                    # (output + rs) * x_mask, rounded for the consuming conv
                    o16 = train_ops.wn_final(output, rs, x_mask)
                    if o16 is not None:
                        return o16
                output = (torch.zeros_like(x) if output is None else output) + rs
        return output * x_mask

    def infer(self, x, g=None, **kwargs):
        from .engine import wn_infer

        return wn_infer(self, x, g)


class ResBlock2(nn.Module):
    """Speaker-conditioned gated residual block (modules.py:223-260)."""

    def __init__(self, channels, kernel_size=3, dilation=(1, 3, 5), gin_channels=0):
        super().__init__()
        inter = (channels // 16) * 16
        self.kernel_size = kernel_size
        self.dilation = tuple(dilation)
        self.convs1 = nn.ModuleList([
            weight_norm(nn.Conv1d(channels, inter, kernel_size, 1, dilation=d,
                                  padding=get_padding(kernel_size, d))) for d in dilation])
        for c in self.convs1:
            c._vits_gate = True  # feeds only the gate (train_ops.conv1d_gate)
        self.convs2 = nn.ModuleList([
            weight_norm(nn.Conv1d(inter // 2, channels, kernel_size, 1, dilation=1,
                                  padding=get_padding(kernel_size, 1))) for _ in dilation])
        self.conds = nn.ModuleList([
            weight_norm(nn.Linear(gin_channels, inter)) for _ in dilation])
        self.apply(init_weights)

    def forward(self, x, g=None, conds=None):
        """conds: the conditioning Linears' outputs when the caller computed
        them (Generator._resblock_conds: all resblocks in one GEMM)."""
        if not (torch.is_grad_enabled() and (x.requires_grad or any(
                p.requires_grad for p in self.parameters()))):
            from .engine import resblock_infer

            return resblock_infer(self, x, g)
        for i, (c1, c2, cs) in enumerate(zip(self.convs1, self.convs2, self.conds)):
            gc = train_ops.linear(cs, g) if conds is None else conds[i]
            gc32 = None
            if isinstance(gc, tuple):  # (16-bit cond, its fp32 copy): Generator._resblock_conds
                gc, gc32 = gc
            # c1 + gate as one launch on the fp16 training path
            if gc32 is not None:
                xt = train_ops.conv1d_gate(c1, x, gc32, in_slope=LRELU_SLOPE, g16=gc)
            else:
                xt = train_ops.conv1d_gate(c1, x, gc, in_slope=LRELU_SLOPE)
            if xt is None:
                xt = train_ops.gate(train_ops.conv1d(c1, x, in_slope=LRELU_SLOPE), gc)
            # modules.py:258-259 (xt = c2(xt); x = xt + x): the add in the
            # conv epilogue on the fp16 training path
            x = train_ops.conv1d(c2, xt, residual=x)
        return x

    def infer(self, x, g=None):
        return self.forward(x, g)


class Flip(nn.Module):
    """Channel reversal between couplings (modules.py:278-289)."""

    def forward(self, x, *args, reverse=False, **kwargs):
        x = torch.flip(x, [1])
        if not reverse:
            return x, torch.zeros(x.size(0), dtype=x.dtype, device=x.device)
        return x

    def infer(self, x, *args, reverse=True, **kwargs):
        return torch.flip(x, [1])


class ResidualCouplingLayer(nn.Module):
    """Mean-only affine coupling (modules.py:314-375)."""

    def __init__(self, channels, hidden_channels, kernel_size, dilation_rate, n_layers,
                 p_dropout=0, gin_channels=0, mean_only=False):
        assert channels % 2 == 0, "channels should be divisible by 2"
        super().__init__()
        self.channels = channels
        self.hidden_channels = hidden_channels
        self.kernel_size = kernel_size
        self.dilation_rate = dilation_rate
        self.n_layers = n_layers
        self.half_channels = channels // 2
        self.mean_only = mean_only
        self.pre = nn.Conv1d(self.half_channels, hidden_channels, 1)
        self.enc = WN(hidden_channels, kernel_size, dilation_rate, n_layers, p_dropout=p_dropout,
                      gin_channels=gin_channels)
        self.post = nn.Conv1d(hidden_channels, self.half_channels * (2 - mean_only), 1)
        self.post.weight.data.zero_()
        self.post.bias.data.zero_()

    def _stats(self, x0, x_mask, g):
        h = train_ops.conv1d(self.pre, x0) * x_mask
        h = self.enc(h, x_mask, g=g)
        stats = train_ops.conv1d(self.post, h) * x_mask
        if not self.mean_only:
            m, logs = torch.split(stats, [self.half_channels] * 2, 1)
        else:
            m, logs = stats, torch.zeros_like(stats)
        return m, logs

    def _fused(self, x, x_mask, g, reverse, flip):
        """The mean-only coupling on the fused fp16 training path: pre conv ->
        mask_cast (h and the first in_layer's 16-bit input) -> WN (16-bit
        output) -> post conv -> one coupling-update kernel (+ the Flip that
        follows, when ``flip``).  None where it does not apply."""
        if not (self.mean_only and train_ops.coupling_fused_ok(x, x_mask)):
            return None
        x0 = x[:, :self.half_channels]
        y = train_ops.conv1d(self.pre, x0)
        mc = train_ops.mask_cast(y, x_mask)
        if mc is None:
            return None
        h, h16 = mc
        o = self.enc(h, x_mask, g=g, out16=True, x16=h16)
        p = train_ops.conv1d(self.post, o)
        return train_ops.coupling_update(x, p, x_mask, reverse, flip)

    def forward(self, x, x_mask, g=None, reverse=False, flip=False):
        """flip: apply the following Flip module's channel reversal to the
        result (ResidualCouplingBlock folds it into the update kernel)."""
        out = self._fused(x, x_mask, g, reverse, flip)
        if out is not None:
            if reverse:
                return out
            return out, torch.zeros(x.shape[0], device=x.device, dtype=x.dtype)
        x0, x1 = torch.split(x, [self.half_channels] * 2, 1)
        m, logs = self._stats(x0, x_mask, g)
        if not reverse:
            x1 = m + x1 * torch.exp(logs) * x_mask
            out, logdet = torch.cat([x0, x1], 1), torch.sum(logs, [1, 2])
            return (torch.flip(out, [1]) if flip else out), logdet
        x1 = (x1 - m) * torch.exp(-logs) * x_mask
        out = torch.cat([x0, x1], 1)
        return torch.flip(out, [1]) if flip else out

    def infer(self, x, g, reverse=True):
        from .engine import coupling_infer

        return coupling_infer(self, x, g)


class TorchSTFT(nn.Module):
    """STFT front of the MR-STFT loss (modules.py:378-400).  ``stft`` returns
    (re, im) like the reference; the loss itself goes through the fused HIP
    magnitude kernel (vits_amd.stft_loss)."""

    def __init__(self, fft_size, hop_size, win_size=None):
        super().__init__()
        self.fft_size = fft_size
        self.hop_size = hop_size
        self.win_size = win_size if win_size is not None else fft_size
        self.register_buffer("window", torch.hann_window(self.win_size), persistent=False)

    def stft(self, x):
        spec = torch.stft(x, n_fft=self.fft_size, hop_length=self.hop_size,
                          win_length=self.win_size, window=self.window, center=True,
                          pad_mode="reflect", return_complex=True)
        return spec.real, spec.imag

    def istft(self, real, imag):
        return torch.istft(torch.complex(real, imag), n_fft=self.fft_size,
                           hop_length=self.hop_size, win_length=self.win_size,
                           window=self.window, center=True, return_complex=False)

    def mag(self, x, eps=1e-7):
        from .ops import stft_mag

        return stft_mag(x, self.window, self.fft_size, self.hop_size, self.win_size, eps=eps)
