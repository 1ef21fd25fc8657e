"""Post-LN transformer text encoder (reference ``attentions.py``).

``forward`` is the masked training path (PyTorch-ROCm ops under autograd);
``infer`` runs through the HIP kernels (MFMA conv projections, the fused
flash-style attention kernel, channel LayerNorm) via ``vits_amd.engine``.
"""
from __future__ import annotations

import math

import torch
from torch import nn
from torch.nn import functional as F

from . import train_ops
from .modules import LayerNorm


# self-attention's q / k / v projections as one HIP conv under autocast
# (train_ops.conv1d_cat); False (tests) keeps three
QKV_CAT = True


class MultiHeadAttention(nn.Module):
    """1x1-conv QKV + scaled dot-product attention (attentions.py:57-100).
    Plain (absolute-position) attention: no relative windows in this fork."""

    def __init__(self, channels, out_channels, n_heads, p_dropout=0):
        super().__init__()
        assert channels % n_heads == 0
        self.channels = channels
        self.out_channels = out_channels
        self.n_heads = n_heads
        self.p_dropout = p_dropout
        self.k_channels = channels // n_heads
        self.conv_q = nn.Conv1d(channels, channels, 1)
        self.conv_k = nn.Conv1d(channels, channels, 1)
        self.conv_v = nn.Conv1d(channels, channels, 1)
        self.conv_o = nn.Conv1d(channels, out_channels, 1)
        self.drop = nn.Dropout(p_dropout)
        nn.init.xavier_uniform_(self.conv_q.weight)
        nn.init.xavier_uniform_(self.conv_k.weight)
        nn.init.xavier_uniform_(self.conv_v.weight)
        # (served by train_ops.conv1d_cat in self-attention, which packs the
        # concatenated weight: train_ops.prepacked skips them)
        for m in (self.conv_q, self.conv_k, self.conv_v):
            m._vits_cat = True

    def forward(self, x, c, attn_mask=None, lengths=None):
        """lengths (int [B], optional): the key / query lengths attn_mask was
        built from (Encoder: x_mask outer product); unused in training, where
        the attention core is the reference's batched matmul / softmax
        (hipBLASLt; the inference plans run csrc/attention.hip instead)."""
        # 1x1 projections on the HIP training conv under autocast (torch otherwise)
        conv = train_ops.conv1d
        qkv = (train_ops.conv1d_cat((self.conv_q, self.conv_k, self.conv_v), x)
               if c is x and QKV_CAT else None)
        if qkv is not None:  # self-attention: q, k, v as one conv launch
            q, k, v = qkv
        else:
            q, k, v = conv(self.conv_q, x), conv(self.conv_k, c), conv(self.conv_v, c)
        y = self.attention(q, k, v, mask=attn_mask)[0]
        return conv(self.conv_o, y)

    def attention(self, query, key, value, mask=None):
        b, d, t_s = key.size()
        t_t = query.size(2)
        H, D = self.n_heads, self.k_channels
        q = query.view(b, H, D, t_t).transpose(2, 3)
        k = key.view(b, H, D, t_s).transpose(2, 3)
        v = value.view(b, H, D, t_s).transpose(2, 3)
        scores = torch.matmul(q / math.sqrt(D), k.transpose(-2, -1))
        if mask is not None:
            scores = scores.masked_fill(mask == 0, -1e4)
        p = self.drop(F.softmax(scores, dim=-1))
        out = torch.matmul(p, v).transpose(2, 3).contiguous().view(b, d, t_t)
        return out, p


class FFN2(nn.Module):
    """k-conv -> speaker-conditioned tanh*sigmoid gate -> k-conv (attentions.py:129-166)."""

    def __init__(self, in_channels, out_channels, filter_channels, kernel_size, p_dropout=0,
                 gin_channels=0):
        super().__init__()
        assert kernel_size % 2 == 1, f"{kernel_size}"
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.filter_channels = filter_channels
        self.kernel_size = kernel_size
        self.p_dropout = p_dropout
        self.conv_1 = nn.Conv1d(in_channels, filter_channels * 2, kernel_size, padding=kernel_size // 2)
        self.conv_2 = nn.Conv1d(filter_channels, out_channels, kernel_size, padding=kernel_size // 2)
        self.drop = nn.Dropout(p_dropout)
        self.cond = nn.Linear(gin_channels, filter_channels * 2)
        nn.init.xavier_uniform_(self.conv_1.weight)
        nn.init.xavier_uniform_(self.conv_2.weight)
        nn.init.xavier_uniform_(self.cond.weight)

    def _gate(self, x, g):
        xa, xb = torch.chunk(x, 2, dim=1)
        sa, sb = torch.chunk(self.cond(g), 2, dim=1)
        return torch.tanh(xa + sa.unsqueeze(-1)) * torch.sigmoid(xb + sb.unsqueeze(-1))

    def forward(self, x, x_mask, g):
        # HIP conv + fused gate under autocast; the reference's ops otherwise
        x = train_ops.gate(self.drop(train_ops.conv1d(self.conv_1, x)), self.cond(g))
        return train_ops.conv1d(self.conv_2, x * x_mask) * x_mask

    def infer(self, x, g):
        return self.conv_2(self._gate(self.conv_1(x), g))


class Encoder(nn.Module):
    """n_layers x [x = LN(x + MHA(x)); x = LN(x + FFN2(x, g))] (attentions.py:12-54)."""

    def __init__(self, hidden_channels, filter_channels, n_heads, n_layers, kernel_size=1,
                 p_dropout=0.0, ffn="FFN2", gin_channels=0, **kwargs):
        super().__init__()
        if ffn != "FFN2":
            raise NotImplementedError("only ffn='FFN2' (configs/base.json) is on the hot path")
        self.hidden_channels = hidden_channels
        self.filter_channels = filter_channels
        self.n_heads = n_heads
        self.n_layers = n_layers
        self.kernel_size = kernel_size
        self.p_dropout = p_dropout
        self.gin_channels = gin_channels
        self.drop = nn.Dropout(p_dropout)
        self.attn_layers = nn.ModuleList()
        self.norm_layers_1 = nn.ModuleList()
        self.ffn_layers = nn.ModuleList()
        self.norm_layers_2 = nn.ModuleList()
        for _ in range(n_layers):
            self.attn_layers.append(MultiHeadAttention(hidden_channels, hidden_channels, n_heads,
                                                       p_dropout=p_dropout))
            self.norm_layers_1.append(LayerNorm(hidden_channels))
            self.ffn_layers.append(FFN2(hidden_channels, hidden_channels, filter_channels,
                                        kernel_size, p_dropout=p_dropout, gin_channels=gin_channels))
            self.norm_layers_2.append(LayerNorm(hidden_channels))

    def forward(self, x, x_mask, g):
        attn_mask = x_mask.unsqueeze(2) * x_mask.unsqueeze(-1)
        # (x_mask is a length mask, commons.sequence_mask: its row sums are
        # the lengths the HIP attention masks with)
        lengths = x_mask[:, 0].sum(-1).to(torch.int32) if x_mask.is_cuda else None
        x = x * x_mask
        for i in range(self.n_layers):
            y = self.drop(self.attn_layers[i](x, x, attn_mask, lengths=lengths))
            x = self.norm_layers_1[i](x + y)
            y = self.drop(self.ffn_layers[i](x, x_mask, g=g))
            x = self.norm_layers_2[i](x + y)
        return x * x_mask

    def infer(self, x, g):
        from .engine import encoder_infer

        return encoder_infer(self, x, g)
