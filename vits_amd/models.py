"""VITS synthesizer (reference ``models.py``), MI355X-native inference path.

Constructor signatures, attribute names and state_dict keys match the
reference (``models.py:20-575``), so checkpoints, ``train*.py``-style drivers,
``export.load_model`` and ``EmoVITS`` consume this module unchanged.

Execution:
* ``infer`` / ``infer_p1`` / ``infer_p2`` / ``inference`` and any no-grad
  ``Generator`` call run on libvits_amd kernels (``vits_amd.engine``); they
  require a ROCm GPU and raise otherwise (no CPU fallback).
* ``forward`` (training) runs PyTorch-ROCm ops under autograd; its
  monotonic-alignment search is the HIP ``maximum_path`` kernel
  (models.py:498 call contract).
"""
from __future__ import annotations

import math
from typing import Optional

import torch
from torch import nn
from torch.nn import Conv1d, ConvTranspose1d
from torch.nn import functional as F
from torch.nn.utils import remove_weight_norm, weight_norm

from . import attentions, commons, engine, modules, train_ops
from .commons import gen_sin_table, get_padding, init_weights
from .monotonic_align import maximum_path
from .ops import neg_cent as neg_cent_scores


def _needs_grad(module: nn.Module, *tensors) -> bool:
    if not torch.is_grad_enabled():
        return False
    if any(t is not None and t.requires_grad for t in tensors):
        return True
    return any(p.requires_grad for p in module.parameters())


class DurationPredictor(nn.Module):
    """L1-log duration predictor with speaker conditioning (models.py:20-67)."""

    def __init__(self, in_channels, filter_channels, kernel_size=5, p_dropout=0.25, act_func="ReLU",
                 act_func_params={}, gin_channels=0):
        super().__init__()
        self.in_channels = in_channels
        self.filter_channels = filter_channels
        self.kernel_size = kernel_size
        self.p_dropout = p_dropout
        self.gin_channels = gin_channels
        self.drop = nn.Dropout(p_dropout)
        self.pre = nn.Conv1d(in_channels, filter_channels, 1)
        self.conv_1 = nn.Conv1d(filter_channels, filter_channels, kernel_size, padding=kernel_size // 2)
        self.norm_1 = modules.LayerNorm(filter_channels)
        self.conv_2 = nn.Conv1d(filter_channels, filter_channels, kernel_size, padding=kernel_size // 2)
        self.norm_2 = modules.LayerNorm(filter_channels)
        self.proj = nn.Conv1d(filter_channels, 1, 1)
        self.cond1 = nn.Linear(gin_channels, filter_channels)
        self.cond2 = nn.Linear(gin_channels, filter_channels)
        if act_func.lower() == "swish":
            raise NotImplementedError("act_func_d='swish' is not selected by configs/base.json")
        self.act_1 = getattr(nn, act_func)(**act_func_params)
        self.act_2 = getattr(nn, act_func)(**act_func_params)

    def forward(self, x, x_mask, g):
        x, g = torch.detach(x), torch.detach(g)
        conv = train_ops.conv1d  # HIP under autocast on the GPU, torch otherwise
        x = conv(self.pre, x) + self.cond1(g).unsqueeze(-1)
        x = conv(self.conv_1, x * x_mask)
        x = self.drop(self.norm_1(self.act_1(x)))
        x = x + self.cond2(g).unsqueeze(-1)
        x = conv(self.conv_2, x * x_mask)
        x = self.drop(self.norm_2(self.act_2(x)))
        x = conv(self.proj, x * x_mask)
        return x * x_mask

    @torch.no_grad()
    def infer(self, x, g):
        engine._check_gpu(x, "DurationPredictor.infer")
        plan = engine.get_plan(self, engine.DurationPlan)
        return plan.run(engine._f32(x), g).to(x.dtype)


class TextEncoder(nn.Module):
    """Linear+LN text-vector embedding, emotion projection, scaled sinusoid
    positions, post-LN transformer, 1x1 projection (models.py:103-189)."""

    def __init__(self, in_channels, out_channels, hidden_channels, filter_channels, n_heads, n_layers,
                 kernel_size, p_dropout, ffn="FFN2", gin_channels=0):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.hidden_channels = hidden_channels
        self.filter_channels = filter_channels
        self.n_heads = n_heads
        self.n_layers = n_layers
        self.kernel_size = kernel_size
        self.p_dropout = p_dropout
        self.emb = nn.Sequential(nn.Linear(in_channels, hidden_channels), nn.LayerNorm(hidden_channels))
        self.emo_proj = nn.Linear(1024, hidden_channels)
        self.register_buffer("sin_table", gen_sin_table(256 + 128, hidden_channels), persistent=False)
        self.xscale = math.sqrt(hidden_channels)
        self.alpha = nn.Parameter(torch.tensor(1.0))
        self.encoder = attentions.Encoder(hidden_channels, filter_channels, n_heads, n_layers,
                                          kernel_size, p_dropout, ffn=ffn, gin_channels=gin_channels)
        self.proj = nn.Conv1d(hidden_channels, out_channels * 2, 1)
        nn.init.xavier_uniform_(self.emo_proj.weight)
        nn.init.xavier_uniform_(self.proj.weight)

    def positional_encoding(self, x, alpha):
        T, max_len = x.size(1), self.sin_table.size(1)
        assert not self.training or T < max_len, f"The input T={T} > max_len{max_len}, pls resolve it!"
        pe = self.sin_table[:, :T] if T <= max_len else gen_sin_table(T, x.size(2)).to(x.device)
        return x * self.xscale + pe * alpha

    def forward(self, x, x_lengths, emo, g):
        x = self.emb(x) + self.emo_proj(emo).unsqueeze(1)
        x = self.positional_encoding(x, self.alpha).transpose(1, -1)
        x_mask = torch.unsqueeze(commons.sequence_mask(x_lengths, x.size(2)), 1).to(x.dtype)
        x = self.encoder(x * x_mask, x_mask, g=g)
        stats = train_ops.conv1d(self.proj, x) * x_mask
        m, logs = torch.split(stats, self.out_channels, dim=1)
        return x, m, logs, x_mask

    @torch.no_grad()
    def infer(self, x, emo, g):
        engine._check_gpu(x, "TextEncoder.infer")
        plan = engine.get_plan(self, engine.TextEncoderPlan)
        h, m, logs = plan.run(x, emo, g)
        return h.to(x.dtype), m.to(x.dtype), logs.to(x.dtype)

    @torch.no_grad()
    def forward_masked_hip(self, x, x_lengths, emo, g, exp_logs=False, pad_exact=False):
        """Masked TextEncoder.forward on the HIP path (used by ``inference``);
        pad_exact: TextEncoder.infer of each unpadded utterance instead
        (engine.TextEncoderPlan.run)."""
        plan = engine.get_plan(self, engine.TextEncoderPlan)
        lengths = x_lengths.to(device=x.device, dtype=torch.int32).contiguous()
        return plan.run(x, emo, g, lengths=lengths, exp_logs=exp_logs, pad_exact=pad_exact)


class ResidualCouplingBlock(nn.Module):
    """4 mean-only couplings with channel flips (models.py:192-235)."""

    def __init__(self, channels, hidden_channels, kernel_size, dilation_rate, n_layers, n_flows=4,
                 gin_channels=0):
        super().__init__()
        assert len(dilation_rate) == n_flows
        self.channels = channels
        self.hidden_channels = hidden_channels
        self.kernel_size = kernel_size
        self.dilation_rate = dilation_rate
        self.n_layers = n_layers
        self.n_flows = n_flows
        self.gin_channels = gin_channels
        self.flows = nn.ModuleList()
        for i in range(n_flows):
            self.flows.append(modules.ResidualCouplingLayer(
                channels, hidden_channels, kernel_size, dilation_rate[i], n_layers,
                gin_channels=gin_channels, mean_only=True))
            self.flows.append(modules.Flip())

    @property
    def flows_reversed(self):
        return list(self.flows)[::-1]

    def forward(self, x, x_mask, g=None, reverse=False):
        flows = list(self.flows) if not reverse else list(self.flows)[::-1]
        i = 0
        while i < len(flows):
            f = flows[i]
            # a coupling followed by a Flip: the flip folded into the coupling
            flip = (isinstance(f, modules.ResidualCouplingLayer) and i + 1 < len(flows)
                    and isinstance(flows[i + 1], modules.Flip))
            kw = dict(flip=True) if flip else {}
            if not reverse:
                x, _ = f(x, x_mask, g=g, reverse=reverse, **kw)
            else:
                x = f(x, x_mask, g=g, reverse=reverse, **kw)
            i += 2 if flip else 1
        return x

    @torch.no_grad()
    def infer(self, x, g, reverse=True):
        if not reverse:
            raise NotImplementedError("infer() runs the reverse (generation) direction only")
        return engine.flow_infer(self, x, g)


class PosteriorEncoder(nn.Module):
    """Linear-spectrogram encoder q(z|x) (models.py:238-279)."""

    def __init__(self, in_channels, out_channels, hidden_channels, kernel_size, dilation_rate,
                 n_layers, gin_channels=0):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.hidden_channels = hidden_channels
        self.kernel_size = kernel_size
        self.dilation_rate = dilation_rate
        self.n_layers = n_layers
        self.gin_channels = gin_channels
        self.pre = nn.Sequential(nn.Conv1d(in_channels, hidden_channels, 1),
                                 modules.LayerNorm(hidden_channels))
        self.enc = modules.WN(hidden_channels, kernel_size, dilation_rate, n_layers,
                              gin_channels=gin_channels)
        self.proj = nn.Conv1d(hidden_channels, out_channels * 2, 1)

    def forward(self, x, x_lengths, g=None, noise=None):
        x_mask = torch.unsqueeze(commons.sequence_mask(x_lengths, x.size(2)), 1).to(x.dtype)
        x = self.pre[1](train_ops.conv1d(self.pre[0], x)) * x_mask
        x = self.enc(x, x_mask, g=g)
        stats = train_ops.conv1d(self.proj, x) * x_mask
        m, logs = torch.split(stats, self.out_channels, dim=1)
        if noise is None:
            noise = torch.randn_like(m)
        z = (m + noise * torch.exp(logs)) * x_mask
        return z, m, logs, x_mask

    @torch.no_grad()
    def infer(self, x, n, g=None):
        engine._check_gpu(x, "PosteriorEncoder.infer")
        plan = engine.get_plan(self, engine.PosteriorPlan)
        return plan.run(x, n, g).to(x.dtype)


class Generator(nn.Module):
    """HiFi-GAN-style decoder with gated, speaker-conditioned ResBlock2
    (models.py:282-318).  Without autograd it runs the fused HIP plan (ROCm
    only); with autograd it runs PyTorch-ROCm ops (training)."""

    def __init__(self, initial_channel, resblock, resblock_kernel_sizes, resblock_dilation_sizes,
                 upsample_rates, upsample_initial_channel, upsample_kernel_sizes, gin_channels=0):
        super().__init__()
        if str(resblock) != "2":
            raise NotImplementedError("only resblock='2' (configs/base.json) is on the hot path")
        self.num_kernels = len(resblock_kernel_sizes)
        self.num_upsamples = len(upsample_rates)
        self.conv_pre = Conv1d(initial_channel, upsample_initial_channel, 7, 1, padding=3)
        self.ups = nn.ModuleList()
        for i, (u, k) in enumerate(zip(upsample_rates, upsample_kernel_sizes)):
            self.ups.append(weight_norm(ConvTranspose1d(
                upsample_initial_channel // (2 ** i), upsample_initial_channel // (2 ** (i + 1)),
                k, u, padding=(k - u) // 2)))
        self.resblocks = nn.ModuleList()
        for i in range(len(self.ups)):
            ch = upsample_initial_channel // (2 ** (i + 1))
            for k, d in zip(resblock_kernel_sizes, resblock_dilation_sizes):
                self.resblocks.append(modules.ResBlock2(ch, k, d, gin_channels))
        self.conv_post = Conv1d(ch, 1, 7, 1, padding=3, bias=False)
        self.ups.apply(init_weights)

    def forward(self, x, g):
        if not _needs_grad(self, x, g):
            # inference: HIP plan only (raises off-GPU; there is no CPU path)
            return engine.generator_forward(self, x, g)
        x = train_ops.conv1d(self.conv_pre, x)
        conds, y16, y32 = self._resblock_conds(g)
        col0 = 0
        for i in range(self.num_upsamples):
            # polyphase on the HIP training conv under autocast (torch otherwise)
            x = train_ops.conv_transpose1d(self.ups[i], x, in_slope=modules.LRELU_SLOPE)
            rbs = self.resblocks[i * self.num_kernels:(i + 1) * self.num_kernels]
            # the stage's branches as grouped launches (fp16 autocast on the GPU)
            xs = train_ops.resblock_stage(x, rbs, y16, y32, col0)
            if xs is None:
                xs = 0
                for j in range(self.num_kernels):
                    rb = i * self.num_kernels + j
                    xs = xs + self.resblocks[rb](x, g=g, conds=None if conds is None else conds[rb])
                xs = xs / self.num_kernels
            x = xs
            col0 += sum(cs.out_features for rb in rbs for cs in rb.conds)
        x = train_ops.conv1d(self.conv_post, x, in_slope=0.01)  # F.leaky_relu default slope
        return torch.tanh(x)

    def _resblock_conds(self, g):
        """Every ResBlock2 conditioning Linear (modules.py:250-255: one per
        dilation pair, 36 at the base config, all applied to the same g) as
        ONE GEMM over the concatenated weights, split back per resblock:
        the same products, one launch instead of 36 (each with its own
        autocast casts and backward GEMMs).  Returns (per-resblock conds,
        the GEMM's output y, its fp32 copy y32 or None), or (None, None,
        None) without a speaker vector."""
        if g is None or not g.is_cuda:
            return None, None, None
        mods = [cs for rb in self.resblocks for cs in rb.conds]
        if not all(isinstance(m, nn.Linear) and m.bias is not None for m in mods):
            return None, None, None
        ws = [train_ops.module_weight(m) for m in mods]
        y = F.linear(g, torch.cat(ws, 0), torch.cat([m.bias for m in mods]))
        sizes = [w.shape[0] for w in ws]
        parts = torch.split(y, sizes, dim=1)
        y32 = train_ops.cond_f32(y)  # one cast for every pair's fused gate
        if y32 is not None:
            parts = list(zip(parts, torch.split(y32, sizes, dim=1)))
        k = len(self.resblocks[0].conds)
        return [parts[i * k:(i + 1) * k] for i in range(len(self.resblocks))], y, y32

    def infer(self, x, g):
        return self.forward(x, g)


class SynthesizerTrn(nn.Module):
    """Synthesizer for training and inference (models.py:411-575)."""

    def __init__(self, text_channels, spec_channels, segment_size, inter_channels, hidden_channels,
                 filter_channels, n_heads, n_layers, kernel_size, p_dropout,
                 resblock_kernel_sizes=None, resblock_dilation_sizes=None, upsample_rates=None,
                 upsample_initial_channel=None, upsample_kernel_sizes=None, resblock="2",
                 ffn="FFN2", kernel_size_q=5, n_layers_q=16, hidden_size_d=256, kernel_size_d=5,
                 p_dropout_d=0.5, act_func_d="ReLU", act_func_params_d={}, dilation_rate=[1, 1, 1, 1],
                 n_flows=4, n_speakers=0, gin_channels=0, align_noise=0.01, align_noise_decay=1e-6,
                 align_noise_min=0, **kwargs):
        super().__init__()
        assert len(dilation_rate) == n_flows
        assert n_speakers > 1
        self.segment_size = segment_size
        self.text_channels = text_channels
        self.inter_channels = inter_channels
        self.align_noise = align_noise
        self.align_noise_decay = align_noise_decay
        self.align_noise_min = align_noise_min
        self.dec = Generator(inter_channels, resblock, resblock_kernel_sizes, resblock_dilation_sizes,
                             upsample_rates, upsample_initial_channel, upsample_kernel_sizes,
                             gin_channels=gin_channels)
        self.enc_p = TextEncoder(text_channels, inter_channels, hidden_channels, filter_channels,
                                 n_heads, n_layers, kernel_size, p_dropout, ffn=ffn,
                                 gin_channels=gin_channels)
        self.enc_q = PosteriorEncoder(spec_channels, inter_channels, hidden_channels, kernel_size_q,
                                      1, n_layers_q, gin_channels=0)
        self.flow = ResidualCouplingBlock(inter_channels, hidden_channels, 5,
                                          dilation_rate=dilation_rate, n_layers=4, n_flows=n_flows,
                                          gin_channels=gin_channels)
        self.dp = DurationPredictor(hidden_channels, hidden_size_d, kernel_size_d,
                                    p_dropout=p_dropout_d, act_func=act_func_d,
                                    act_func_params=act_func_params_d, gin_channels=gin_channels)
        self.emb_g = nn.Embedding(n_speakers, gin_channels)
        self.hop_total = 1
        for u in upsample_rates:
            self.hop_total *= u
        self._graphs = {}

    # ------------------------------------------------------------------ utils
    def remove_weight_norm(self):
        """Fold weight norm into plain weights (models.py:467-474)."""
        def _remove(m):
            try:
                remove_weight_norm(m)
            except ValueError:
                return
        self.apply(_remove)
        engine.drop_plans(self)
        self._graphs.clear()

    def _apply(self, fn, *args, **kwargs):
        self._graphs = {}
        out = super()._apply(fn, *args, **kwargs)
        engine.drop_plans(self)
        return out

    # --------------------------------------------------------------- training
    def forward(self, x, x_lengths, y, y_lengths, emo, sid=None, noise_q=None, noise_align=None,
                noise_flow=None):
        """Training forward (models.py:476-515).  The optional noise tensors
        replace the three in-graph randn draws (posterior sample, alignment
        noise, reverse-flow sample) for reproducible parity runs."""
        g = self.emb_g(sid)
        x, m_p, logs_p, x_mask = self.enc_p(x, x_lengths, emo, g=g)
        z, m_q, logs_q, y_mask = self.enc_q(y, y_lengths, g=None, noise=noise_q)
        z_p = self.flow(z, y_mask, g=g)

        with torch.no_grad():
            # one fp32 MFMA kernel for the exp / 2 matmuls / 2 sums of
            # models.py:484-489 (vits_neg_cent)
            neg_cent = neg_cent_scores(z_p, m_p, logs_p)
            if self.align_noise > 0:
                eps = noise_align if noise_align is not None else torch.randn_like(neg_cent)
                an = self.__dict__.get("_align_noise_t")
                if an is not None:
                    # graph-captured step: the decaying scale lives on the device
                    # and decays inside the graph (one step per replay)
                    neg_cent = neg_cent + torch.std(neg_cent) * eps * an
                    an.sub_(self.align_noise_decay).clamp_(min=self.align_noise_min)
                else:
                    neg_cent = neg_cent + torch.std(neg_cent) * eps * self.align_noise
                self.align_noise -= self.align_noise_decay
                self.align_noise = max(self.align_noise, self.align_noise_min)
            attn_mask = torch.unsqueeze(x_mask, 2) * torch.unsqueeze(y_mask, -1)
            attn = maximum_path(neg_cent, attn_mask.squeeze(1)).detach()

        w = attn.sum(1, keepdim=True)
        logw_ = torch.log(w + 1e-6) * x_mask
        logw = self.dp(x, x_mask, g=g)
        l_length = torch.sum(torch.abs(logw - logw_), [1, 2]) / torch.sum(x_mask)

        m_p = torch.matmul(attn, m_p.transpose(1, 2)).transpose(1, 2)
        logs_p = torch.matmul(attn, logs_p.transpose(1, 2)).transpose(1, 2)

        z_slice, ids_slice = commons.rand_slice_segments(
            z, y_lengths, self.segment_size,
            device_rng=self.__dict__.get("_device_slice_rng", False))
        o = self.dec(z_slice, g=g)

        if noise_flow is None:
            noise_flow = torch.randn_like(m_p)
        z_q = self.flow(m_p + noise_flow * torch.exp(logs_p), y_mask, g=g, reverse=True)
        return (o, l_length, attn, ids_slice, x_mask, y_mask, (z, z_p, m_p, logs_p, m_q, logs_q),
                z_q, (x, logw_.detach(), logw))

    # -------------------------------------------------------------- inference
    @torch.no_grad()
    def inference(self, x, x_lengths, emo, sid=None, noise_scale=1, length_scale=1, max_len=None,
                  noise=None):
        """Batched, masked inference (models.py:517-535) on the HIP path.
        ``noise`` (optional, [B, C, T_y] ~ N(0,1)) replaces randn_like(m_p)."""
        engine._check_gpu(x, "SynthesizerTrn.inference")
        g = self.emb_g(sid)
        h, m_p, logs_p = self.enc_p.forward_masked_hip(x, x_lengths, emo, g)
        lengths = x_lengths.to(device=x.device, dtype=torch.int32).contiguous()
        logw = engine.get_plan(self.dp, engine.DurationPlan).run(h, g, lengths=lengths)
        x_mask = torch.unsqueeze(commons.sequence_mask(x_lengths, h.size(2)), 1).to(torch.float32)
        # duration -> path: host-visible lengths (the reference syncs here too)
        w = torch.exp(logw) * x_mask * length_scale
        w_ceil = torch.ceil(w)
        y_lengths = torch.clamp_min(torch.sum(w_ceil, [1, 2]), 1).long()
        y_mask = torch.unsqueeze(commons.sequence_mask(y_lengths, None), 1).to(x_mask.dtype)
        attn_mask = torch.unsqueeze(x_mask, 2) * torch.unsqueeze(y_mask, -1)
        attn = commons.generate_path(w_ceil, attn_mask.squeeze(1))
        if noise is None:
            noise = torch.randn(m_p.shape[0], m_p.shape[1], attn.shape[1], device=x.device)
        z_p = engine.ops.expand_prior(attn, m_p, logs_p, noise, exp_s=True,
                                      noise_scale=float(noise_scale))
        ylen32 = y_lengths.to(torch.int32).contiguous()
        z = engine.flow_reverse_masked(self.flow, z_p, ylen32, g)
        zm = z * y_mask
        o = self.dec(zm[:, :, :max_len].contiguous(), g=g)
        # returned expansions follow the reference: attn @ m_p / attn @ logs_p
        m_e = torch.matmul(attn, m_p.transpose(1, 2)).transpose(1, 2)
        logs_e = torch.matmul(attn, logs_p.transpose(1, 2)).transpose(1, 2)
        return o.to(x.dtype), attn, y_mask, (z, z_p, m_e, logs_e)

    @torch.no_grad()
    def infer(self, x, emo, sid, noise_scale=0.707, length_scale=1.0, noise=None):
        """Single-utterance inference (models.py:537-556)."""
        assert x.size(0) == 1
        m_p, s_p, logw, g = self.infer_p1(x, emo, sid)
        w = torch.exp(logw) * length_scale
        w_ceil = torch.ceil(w)
        y_len = int(torch.clamp_min(torch.sum(w_ceil), 1).item())
        attn = commons.infer_path(w_ceil, x.size(1), y_len, dtype=torch.float32)
        if noise is None:
            noise = torch.randn(1, m_p.shape[1], y_len, device=x.device)
        # reference: z_p = m + randn * exp(logs) * noise_scale with exp taken after
        # the (one-hot) expansion; infer_p1 already returns s = exp(logs)
        return self.infer_p2(attn, m_p, s_p, g, noise * noise_scale)

    @torch.no_grad()
    def infer_p1(self, x, emo, sid):
        """Text side (models.py:558-566): returns m_p, s_p = exp(logs_p), logw, g."""
        assert x.size(0) == 1
        engine._check_gpu(x, "SynthesizerTrn.infer_p1")
        g = self.emb_g(sid)
        plan = engine.get_plan(self.enc_p, engine.TextEncoderPlan)
        h, m_p, s_p = plan.run(x, emo, g, exp_logs=True)
        logw = engine.get_plan(self.dp, engine.DurationPlan).run(h, g)
        dt = x.dtype
        return m_p.to(dt), s_p.to(dt), logw.to(dt), g

    @torch.no_grad()
    def infer_p2(self, attn, m_p, s_p, g, noise):
        """Acoustic side (models.py:568-575): prior expansion + noise, reverse
        flow, decoder — all libvits_amd kernels."""
        engine._check_gpu(m_p, "SynthesizerTrn.infer_p2")
        z = engine.ops.expand_prior(attn, m_p, s_p, noise)
        fplan = engine.get_plan(self.flow, engine.CouplingFlowPlan)
        gf = engine._f32(g)
        fplan.run_(z, gf)
        gplan = engine.get_plan(self.dec, engine.GeneratorPlan)
        o = gplan.run(z, gf)
        return o.to(m_p.dtype)

    # stage multipliers of the lengths the bucketed infer hands to the flow,
    # conv_pre and the upsample stages (frames -> samples after each ups)
    def _stage_mult(self):
        mult, u = [1, 1], 1
        for up in self.dec.ups:
            u *= up.stride[0]
            mult.append(u)
        return tuple(mult)

    @torch.no_grad()
    def infer_bucketed(self, x, emo, sid, noise, t_y, *, x_lengths=None, length_scale=1.0,
                       noise_start=None):
        """infer (models.py:537-556) / EmoVITS.infer (infer.py:160-182) with
        NO host synchronisation, over a static bucket of t_y frames - the
        whole utterance can be captured into one hipGraph
        (capture_infer_bucketed).  The durations, y_len and the path are
        computed on the device (ops.expand_durations: the exp / ceil / sum /
        .item() / infer_path / expansion of models.py:544-553); the reverse
        flow and the decoder run masked at y_len (every conv output is zero
        past it, i.e. the zero padding the reference's decoder sees at the
        utterance end) and tiles past y_len + 64 are skipped
        (ops.length_skip), so the work follows y_len, not t_y.

        ``noise``: pre-scaled like infer_p2's (z = m + noise * s): [B, C,
        t_y], or a flat buffer sliced as EmoVITS slices it at
        np.random.randint(numel - C * y_len), drawn on the device from
        ``noise_start`` = int32 [B, ops.ED_DRAWS] raw MT19937 words
        (ops.numpy_draw_pool); the returned y_len is then int32 [2, B]:
        (y_len, generator words consumed; -1 when the slice does not
        fit, -2 when every word of the pool was rejected: the caller
        advances numpy's generator past the pool and runs again).  ``x_lengths`` (int32 [B]): padded text, encoded
        as TextEncoder.infer of each unpadded utterance (every layer masked,
        engine.TextEncoderPlan pad_exact); None: the exact-length infer_p1
        path (B = 1).  Returns (wav [B, 1, t_y * hop], y_len int32 [B]);
        samples past y_len * hop are not meaningful (crop on the host)."""
        engine._check_gpu(x, "SynthesizerTrn.infer_bucketed")
        dt = x.dtype
        if x_lengths is None:
            m_p, s_p, logw, g = self.infer_p1(x, emo, sid)
            xl = None
        else:
            g = self.emb_g(sid)
            xl = x_lengths.to(device=x.device, dtype=torch.int32).contiguous()
            h, m_p, s_p = self.enc_p.forward_masked_hip(x, xl, emo, g, exp_logs=True,
                                                        pad_exact=True)
            logw = engine.get_plan(self.dp, engine.DurationPlan).run(h, g, lengths=xl)
            m_p, s_p, logw = m_p.to(dt), s_p.to(dt), logw.to(dt)
        z, lens = engine.ops.expand_durations(
            logw, m_p, s_p, noise, int(t_y), rate=float(length_scale), x_len=xl,
            noise_start=noise_start, half_round=dt == torch.float16,
            stage_mult=self._stage_mult())
        gf = engine._f32(g)
        with engine.ops.length_skip(64):
            engine.get_plan(self.flow, engine.CouplingFlowPlan).run_(z, gf, lengths=lens[0])
            o = engine.get_plan(self.dec, engine.GeneratorPlan).run(z, gf, lengths=lens[1:])
        if noise_start is not None:
            return o.to(m_p.dtype), lens[0::len(lens) - 1]
        return o.to(m_p.dtype), lens[0]

    @torch.no_grad()
    def capture_infer_bucketed(self, t_x, t_y, *, noise_len=None, padded_text=False,
                               length_scale=1.0, warmup=2):
        """One hipGraph for a whole utterance (infer_bucketed) of t_x tokens
        (padded_text: up to t_x, x_lengths given at replay) into a t_y-frame
        bucket.  noise_len: replay reads a flat noise buffer of that many
        elements at a per-call start offset (EmoVITS); else noise [1, C,
        t_y].  Returns run(x, emo, sid, noise, noise_start=None,
        x_length=None) -> (wav, y_len) views of static buffers; with
        noise_len, noise_start is the [ops.ED_DRAWS] raw-word pool of
        ops.numpy_draw_pool and y_len is [2, 1] (y_len, words consumed)."""
        dev = next(self.parameters()).device
        dt = next(self.parameters()).dtype
        C = self.inter_channels
        static = dict(x=torch.zeros(1, t_x, self.text_channels, device=dev, dtype=dt),
                      emo=torch.zeros(1, 1024, device=dev, dtype=dt),
                      sid=torch.zeros(1, device=dev, dtype=torch.long),
                      start=torch.zeros(1, engine.ops.ED_DRAWS, device=dev, dtype=torch.int32),
                      xl=torch.full((1,), t_x, device=dev, dtype=torch.int32),
                      noise=torch.zeros(noise_len if noise_len else C * t_y, device=dev))

        def body():
            noise = static["noise"] if noise_len else static["noise"].view(1, C, t_y)
            return self.infer_bucketed(static["x"], static["emo"], static["sid"], noise, t_y,
                                       x_lengths=static["xl"] if padded_text else None,
                                       length_scale=length_scale,
                                       noise_start=static["start"] if noise_len else None)

        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            for _ in range(warmup):
                body()
        torch.cuda.current_stream(dev).wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            out = body()

        def run(x, emo, sid, noise=None, noise_start=None, x_length=None):
            if padded_text:
                n = x.shape[1] if x_length is None else int(x_length)
                static["x"].zero_()
                static["x"][:, :x.shape[1]].copy_(x)
                static["xl"].fill_(n)
            else:
                static["x"].copy_(x)
            static["emo"].copy_(emo)
            static["sid"].copy_(sid)
            if noise is not None:
                static["noise"].copy_(noise.reshape(-1))
            if noise_start is not None:
                static["start"].copy_(torch.as_tensor(noise_start, dtype=torch.int32).view(1, -1))
            graph.replay()
            return out

        run.graph = graph
        run.static = static
        run.t_y = t_y
        return run

    # ------------------------------------------------------------ hipGraphs
    @torch.no_grad()
    def capture_infer_p1(self, t_x, warmup=2):
        """Capture infer_p1 for one utterance of t_x tokens into a hipGraph
        (the text side is ~55 small launches whose host-side descriptor
        building dominates its B=1 latency).  Returns a callable(x, emo, sid)
        -> (m_p, s_p, logw, g) reading / returning static buffers."""
        dev = next(self.parameters()).device
        dt = next(self.parameters()).dtype
        static = dict(x=torch.zeros(1, t_x, self.text_channels, device=dev, dtype=dt),
                      emo=torch.zeros(1, 1024, device=dev, dtype=dt),
                      sid=torch.zeros(1, device=dev, dtype=torch.long))

        def body():
            return self.infer_p1(static["x"], static["emo"], static["sid"])

        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            for _ in range(warmup):
                body()
        torch.cuda.current_stream(dev).wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            out = body()

        def run(x, emo, sid):
            static["x"].copy_(x)
            static["emo"].copy_(emo)
            static["sid"].copy_(sid)
            graph.replay()
            return out

        run.graph = graph
        run.static = static
        return run

    @torch.no_grad()
    def capture_infer_p2(self, batch, t_x, t_y, warmup=2):
        """Capture infer_p2 for a static shape into a hipGraph (torch.cuda.CUDAGraph
        is HIP graphs on ROCm).  Returns a callable(attn, m_p, s_p, g, noise) -> wav
        that copies inputs into static buffers and replays the graph."""
        dev = next(self.parameters()).device
        C = self.inter_channels
        gin = self.emb_g.embedding_dim
        static = dict(
            attn=torch.zeros(batch, t_y, t_x, device=dev), m=torch.zeros(batch, C, t_x, device=dev),
            s=torch.ones(batch, C, t_x, device=dev), g=torch.zeros(batch, gin, device=dev),
            n=torch.zeros(batch, C, t_y, device=dev))
        fplan = engine.get_plan(self.flow, engine.CouplingFlowPlan)
        gplan = engine.get_plan(self.dec, engine.GeneratorPlan)

        def body():
            z = engine.ops.expand_prior(static["attn"], static["m"], static["s"], static["n"])
            fplan.run_(z, static["g"])
            return gplan.run(z, static["g"])

        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            for _ in range(warmup):
                body()
        torch.cuda.current_stream(dev).wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            out = body()

        def run(attn, m_p, s_p, g, noise):
            static["attn"].copy_(attn)
            static["m"].copy_(m_p)
            static["s"].copy_(s_p)
            static["g"].copy_(g)
            static["n"].copy_(noise)
            graph.replay()
            return out

        run.graph = graph
        run.static = static
        run.output = out
        return run


# train.py's discriminator lives beside the generator in the reference's
# models.py (models.py:321-408); the implementation is in discriminators.py
from .discriminators import DiscriminatorP, DiscriminatorS, MultiPeriodDiscriminator  # noqa: E402,F401
