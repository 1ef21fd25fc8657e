"""TEST INFRASTRUCTURE ONLY — functional CPU fp32 restatement of the reference
VITS forward/inference path, driven by a plain state_dict (reference key
names).  Used as the parity checker for the HIP path (tests/, smoke()) and
as bench.py's ``cpu_baseline`` ("port").  Pinned against golden vectors
generated from the reference itself (tests/golden/make_golden.py).

Every function cites the reference lines it restates (paths relative to
emotional-vits/).  Weight norm is folded the way torch.nn.utils.weight_norm
does (g * v / ||v||, norm over all dims but 0).
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

LRELU = 0.1


class SD:
    """state_dict accessor with weight-norm folding."""

    def __init__(self, sd):
        self.sd = {k: v.detach().float().cpu() for k, v in sd.items()}

    def w(self, name):
        if name + ".weight_g" in self.sd:
            return torch._weight_norm(self.sd[name + ".weight_v"], self.sd[name + ".weight_g"], 0)
        return self.sd[name + ".weight"]

    def b(self, name):
        return self.sd.get(name + ".bias")

    def __getitem__(self, k):
        return self.sd[k]

    def has(self, k):
        return k in self.sd


def conv1d(sd: SD, name, x, dilation=1, padding=None):
    w = sd.w(name)
    k = w.shape[-1]
    if padding is None:
        padding = (k * dilation - dilation) // 2
    return F.conv1d(x, w, sd.b(name), padding=padding, dilation=dilation)


def linear(sd: SD, name, x):
    return F.linear(x, sd.w(name), sd.b(name))


def layer_norm_ch(sd: SD, name, x, eps=1e-5):
    """modules.LayerNorm (modules.py:41-44)."""
    C = x.shape[1]
    return F.layer_norm(x.transpose(1, -1), (C,), sd[name + ".gamma"], sd[name + ".beta"],
                        eps).transpose(1, -1)


def sequence_mask(length, max_length):
    """commons.py:120-124."""
    return torch.arange(max_length)[None, :] < length[:, None]


# ---------------------------------------------------------------------------
# WN / coupling / flow
# ---------------------------------------------------------------------------

def wn(sd: SD, pre, x, x_mask, g, n_layers, H, masked=True):
    """WN.forward (modules.py:130-155) / WN.infer (modules.py:157-182)."""
    if sd.has(pre + ".cond_layer.weight_g") or sd.has(pre + ".cond_layer.weight"):
        g = linear(sd, pre + ".cond_layer", g)
        has_cond = True
    else:
        has_cond = False
    output = torch.zeros_like(x)
    for i in range(n_layers):
        x_in = conv1d(sd, f"{pre}.in_layers.{i}", x)
        if has_cond:
            x_in = x_in + g[:, i * 2 * H:(i + 1) * 2 * H].unsqueeze(-1)
        acts = torch.tanh(x_in[:, :H]) * torch.sigmoid(x_in[:, H:])
        rs = conv1d(sd, f"{pre}.res_skip_layers.{i}", acts)
        if i < n_layers - 1:
            x = x + rs[:, :H]
            if masked:
                x = x * x_mask
            output = output + rs[:, H:]
        else:
            output = output + rs
    return output * x_mask if masked else output


def coupling_reverse(sd: SD, pre, x, x_mask, g, n_layers, H, masked):
    """ResidualCouplingLayer reverse (modules.py:357-360) / infer (modules.py:362-375), mean-only."""
    half = x.shape[1] // 2
    x0, x1 = x[:, :half], x[:, half:]
    h = conv1d(sd, pre + ".pre", x0)
    if masked:
        h = h * x_mask
    h = wn(sd, pre + ".enc", h, x_mask, g, n_layers, H, masked=masked)
    m = conv1d(sd, pre + ".post", h)
    if masked:
        m = m * x_mask
        x1 = (x1 - m) * torch.exp(-torch.zeros_like(m)) * x_mask
    else:
        x1 = x1 - m
    return torch.cat([x0, x1], 1)


def flow_reverse(sd: SD, z, g, n_flows=4, n_layers=4, H=256, x_mask=None):
    """ResidualCouplingBlock reversed (models.py:223-226 masked, 228-235 infer)."""
    masked = x_mask is not None
    if not masked:
        x_mask = torch.ones(z.shape[0], 1, z.shape[2])
    x = z
    for i in reversed(range(n_flows)):
        x = torch.flip(x, [1])  # Flip (modules.py:278-289) comes after coupling i
        x = coupling_reverse(sd, f"flow.flows.{2 * i}", x, x_mask, g, n_layers, H, masked)
    return x


# ---------------------------------------------------------------------------
# decoder
# ---------------------------------------------------------------------------

def resblock2(sd: SD, pre, x, g, k, dils):
    """ResBlock2.forward (modules.py:250-260)."""
    for p, d in enumerate(dils):
        xt = F.leaky_relu(x, LRELU)
        xt = conv1d(sd, f"{pre}.convs1.{p}", xt, dilation=d)
        gs = linear(sd, f"{pre}.conds.{p}", g)
        xa, xb = torch.chunk(xt, 2, dim=1)
        sa, sb = torch.chunk(gs, 2, dim=1)
        xt = torch.tanh(xa + sa.unsqueeze(-1)) * torch.sigmoid(xb + sb.unsqueeze(-1))
        xt = conv1d(sd, f"{pre}.convs2.{p}", xt)
        x = xt + x
    return x


def generator(sd: SD, x, g, cfg):
    """Generator.forward (models.py:306-318)."""
    rk = cfg["resblock_kernel_sizes"]
    rd = cfg["resblock_dilation_sizes"]
    ur = cfg["upsample_rates"]
    uk = cfg["upsample_kernel_sizes"]
    x = conv1d(sd, "dec.conv_pre", x, padding=3)
    nk = len(rk)
    for i, (u, k) in enumerate(zip(ur, uk)):
        x = F.leaky_relu(x, LRELU)
        x = F.conv_transpose1d(x, sd.w(f"dec.ups.{i}"), sd.b(f"dec.ups.{i}"), stride=u,
                               padding=(k - u) // 2)
        xs = 0
        for j in range(nk):
            xs += resblock2(sd, f"dec.resblocks.{i * nk + j}", x, g, rk[j], rd[j])
        x = xs / nk
    x = F.leaky_relu(x)
    x = F.conv1d(x, sd["dec.conv_post.weight"], None, padding=3)
    return torch.tanh(x)


# ---------------------------------------------------------------------------
# text encoder / duration predictor
# ---------------------------------------------------------------------------

def gen_sin_table(max_len, d_model):
    """commons.py:176-190."""
    pe = torch.zeros(max_len, d_model)
    position = torch.arange(0, max_len, dtype=torch.float32).unsqueeze(1)
    div_term = torch.exp(torch.arange(0, d_model, 2, dtype=torch.float32) *
                         -(np.log(10000.0) / d_model))
    pe[:, 0::2] = torch.sin(position * div_term)
    pe[:, 1::2] = torch.cos(position * div_term)
    return pe.unsqueeze_(0)


def mha(sd: SD, pre, x, n_heads, mask=None):
    """MultiHeadAttention (attentions.py:78-100)."""
    q = conv1d(sd, pre + ".conv_q", x)
    k = conv1d(sd, pre + ".conv_k", x)
    v = conv1d(sd, pre + ".conv_v", x)
    b, d, t = k.shape
    D = d // n_heads
    q = q.view(b, n_heads, D, t).transpose(2, 3)
    k = k.view(b, n_heads, D, t).transpose(2, 3)
    v = v.view(b, n_heads, D, t).transpose(2, 3)
    scores = torch.matmul(q / math.sqrt(D), k.transpose(-2, -1))
    if mask is not None:
        scores = scores.masked_fill(mask == 0, -1e4)
    p = F.softmax(scores, dim=-1)
    out = torch.matmul(p, v).transpose(2, 3).contiguous().view(b, d, t)
    return conv1d(sd, pre + ".conv_o", out)


def ffn2(sd: SD, pre, x, g, x_mask=None):
    """FFN2.forward / infer (attentions.py:149-166)."""
    x = conv1d(sd, pre + ".conv_1", x)
    gg = linear(sd, pre + ".cond", g)
    xa, xb = torch.chunk(x, 2, dim=1)
    sa, sb = torch.chunk(gg, 2, dim=1)
    x = torch.tanh(xa + sa.unsqueeze(-1)) * torch.sigmoid(xb + sb.unsqueeze(-1))
    if x_mask is not None:
        x = x * x_mask
    x = conv1d(sd, pre + ".conv_2", x)
    return x * x_mask if x_mask is not None else x


def text_encoder(sd: SD, x, emo, g, n_layers, n_heads, out_channels, x_lengths=None):
    """TextEncoder.forward (models.py:167-178) when x_lengths is given, else
    TextEncoder.infer (models.py:180-189)."""
    H = sd["enc_p.emb.0.weight"].shape[0]
    x = F.linear(x, sd["enc_p.emb.0.weight"], sd["enc_p.emb.0.bias"])
    x = F.layer_norm(x, (H,), sd["enc_p.emb.1.weight"], sd["enc_p.emb.1.bias"], 1e-5)
    x = x + linear(sd, "enc_p.emo_proj", emo).unsqueeze(1)
    T = x.shape[1]
    pe = gen_sin_table(max(T, 384), H)[:, :T] if T > 384 else gen_sin_table(384, H)[:, :T]
    x = x * math.sqrt(H) + pe * sd["enc_p.alpha"]
    x = x.transpose(1, -1)
    if x_lengths is not None:
        x_mask = sequence_mask(x_lengths, T).unsqueeze(1).float()
        attn_mask = x_mask.unsqueeze(2) * x_mask.unsqueeze(-1)
        x = x * x_mask
        x = x * x_mask
    else:
        x_mask, attn_mask = None, None
    for i in range(n_layers):
        y = mha(sd, f"enc_p.encoder.attn_layers.{i}", x, n_heads, attn_mask)
        x = layer_norm_ch(sd, f"enc_p.encoder.norm_layers_1.{i}", x + y)
        y = ffn2(sd, f"enc_p.encoder.ffn_layers.{i}", x, g, x_mask)
        x = layer_norm_ch(sd, f"enc_p.encoder.norm_layers_2.{i}", x + y)
    if x_mask is not None:
        x = x * x_mask
    stats = conv1d(sd, "enc_p.proj", x)
    if x_mask is not None:
        stats = stats * x_mask
    m, logs = torch.split(stats, out_channels, dim=1)
    return x, m, logs, x_mask


def duration_predictor(sd: SD, x, g, x_mask=None):
    """DurationPredictor.forward (models.py:47-57) / infer (models.py:59-67), ReLU."""
    msk = (lambda t: t * x_mask) if x_mask is not None else (lambda t: t)
    x = conv1d(sd, "dp.pre", x) + linear(sd, "dp.cond1", g).unsqueeze(-1)
    x = conv1d(sd, "dp.conv_1", msk(x))
    x = layer_norm_ch(sd, "dp.norm_1", F.relu(x))
    x = x + linear(sd, "dp.cond2", g).unsqueeze(-1)
    x = conv1d(sd, "dp.conv_2", msk(x))
    x = layer_norm_ch(sd, "dp.norm_2", F.relu(x))
    x = conv1d(sd, "dp.proj", msk(x))
    return msk(x)


# ---------------------------------------------------------------------------
# synthesizer entry points
# ---------------------------------------------------------------------------

def infer_path(duration, t_x, t_y):
    """commons.py:143-155."""
    b = duration.size(0)
    cum = torch.cumsum(duration, -1).view(b * t_x)
    path = sequence_mask(cum, t_y).float().view(b, t_x, t_y)
    path = path - F.pad(path, (0, 0, 1, 0))[:, :-1]
    return path.transpose(1, 2)


def infer_p1(sd: SD, x, emo, sid, cfg):
    """SynthesizerTrn.infer_p1 (models.py:558-566)."""
    g = F.embedding(sid, sd["emb_g.weight"])
    h, m_p, logs_p, _ = text_encoder(sd, x, emo, g, cfg["n_layers"], cfg["n_heads"],
                                     cfg["inter_channels"])
    s_p = torch.exp(logs_p)
    logw = duration_predictor(sd, h, g)
    return m_p, s_p, logw, g


def infer_p2(sd: SD, attn, m_p, s_p, g, noise, cfg):
    """SynthesizerTrn.infer_p2 (models.py:568-575)."""
    m_p = torch.matmul(attn, m_p.transpose(1, 2)).transpose(1, 2)
    s_p = torch.matmul(attn, s_p.transpose(1, 2)).transpose(1, 2)
    z_p = m_p + noise * s_p
    z = flow_reverse(sd, z_p, g, cfg.get("n_flows", 4), 4, cfg["hidden_channels"])
    return generator(sd, z, g, cfg)


def inference(sd: SD, x, x_lengths, emo, sid, noise, cfg, noise_scale=1.0, length_scale=1.0,
              max_len=None):
    """SynthesizerTrn.inference (models.py:517-535) with the randn draw given."""
    g = F.embedding(sid, sd["emb_g.weight"])
    h, m_p, logs_p, x_mask = text_encoder(sd, x, emo, g, cfg["n_layers"], cfg["n_heads"],
                                          cfg["inter_channels"], x_lengths=x_lengths)
    logw = duration_predictor(sd, h, g, x_mask)
    w = torch.exp(logw) * x_mask * length_scale
    w_ceil = torch.ceil(w)
    y_lengths = torch.clamp_min(torch.sum(w_ceil, [1, 2]), 1).long()
    t_y = int(y_lengths.max())
    y_mask = sequence_mask(y_lengths, t_y).unsqueeze(1).float()
    attn_mask = x_mask.unsqueeze(2) * y_mask.unsqueeze(-1)
    b, _, t_x = w_ceil.shape
    cum = torch.cumsum(w_ceil, -1).view(b * t_x)
    path = sequence_mask(cum, t_y).float().view(b, t_x, t_y)
    path = path - F.pad(path, (0, 0, 1, 0))[:, :-1]
    attn = path.transpose(1, 2) * attn_mask.squeeze(1)
    m_e = torch.matmul(attn, m_p.transpose(1, 2)).transpose(1, 2)
    logs_e = torch.matmul(attn, logs_p.transpose(1, 2)).transpose(1, 2)
    z_p = m_e + noise[:, :, :t_y] * torch.exp(logs_e) * noise_scale
    z = flow_reverse(sd, z_p, g, cfg.get("n_flows", 4), 4, cfg["hidden_channels"], x_mask=y_mask)
    o = generator(sd, (z * y_mask)[:, :, :max_len], g, cfg)
    return o, attn, y_mask, (z, z_p, m_e, logs_e)


def posterior_infer(sd: SD, spec, n, n_layers_q, H):
    """PosteriorEncoder.infer (models.py:273-279)."""
    x = conv1d(sd, "enc_q.pre.0", spec)
    x = layer_norm_ch(sd, "enc_q.pre.1", x)
    x = wn(sd, "enc_q.enc", x, None, None, n_layers_q, H, masked=False)
    stats = conv1d(sd, "enc_q.proj", x)
    C = stats.shape[1] // 2
    m, logs = stats[:, :C], stats[:, C:]
    return m + n * torch.exp(logs)


def neg_cent(z_p, m_p, logs_p):
    """MAS scores, models.py:483-489 (fp32, the four terms summed in the
    reference's order)."""
    s_p_sq_r = torch.exp(-2 * logs_p)
    nc1 = torch.sum(-0.5 * math.log(2 * math.pi) - logs_p, [1], keepdim=True)
    nc2 = torch.matmul(-0.5 * (z_p ** 2).transpose(1, 2), s_p_sq_r)
    nc3 = torch.matmul(z_p.transpose(1, 2), (m_p * s_p_sq_r))
    nc4 = torch.sum(-0.5 * (m_p ** 2) * s_p_sq_r, [1], keepdim=True)
    return nc1 + nc2 + nc3 + nc4
