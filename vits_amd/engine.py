"""Inference engine: lowers the VITS modules onto libvits_amd kernels.

A *plan* is built once per module (weight-norm folded, weights packed into
MFMA-friendly slabs, every per-utterance conditioning Linear stacked into one
GEMV) and cached on the module; it is rebuilt automatically when any
parameter changes (optimizer step, load_state_dict, .to()).  Running a plan
issues only HIP kernels on the current torch stream — no torch compute op, no
host sync — so a whole call can be captured in a hipGraph (see
``SynthesizerTrn.capture_infer_p2``).

Reference semantics followed per plan (paths in emotional-vits/):
  GeneratorPlan      models.py:306-318 + modules.py:250-260
  CouplingFlowPlan   models.py:228-235 (flows_reversed) + modules.py:362-375
                     + modules.py:157-182 (WN.infer); also the masked
                     reverse flow of models.py:219-226 / modules.py:341-360
  TextEncoderPlan    models.py:167-189 + attentions.py:12-54,57-100,129-166
  DurationPlan       models.py:49-67
  PosteriorPlan      models.py:264-279 + modules.py:130-182

Data layout in HBM: activations [B][C][T] fp32 exactly as the reference holds
them (the Generator of a 16-bit model: [B][C][T] of that 16-bit type, ACT16);
per-call intermediates come from the torch caching allocator.
"""
from __future__ import annotations

import os

import math
from typing import Optional

import torch

from . import ops
from ._lib import ACT_EXP, ACT_NONE, ACT_RELU, EPI_GATE
from .ops import PackedConv, make_desc, make_out, pack_conv, pack_conv_transpose

_PLAN_ATTR = "_vits_amd_plan"


def _param_signature(module: torch.nn.Module):
    ver = 0
    first = None
    n = 0
    for p in module.parameters():
        ver += p._version
        if first is None:
            first = (p.data_ptr(), p.device, p.dtype)
        n += 1
    return (first, ver, n)


# How fp32 models run their convs: "split" (default) = fp32 operands split
# exactly into three bf16 terms on the bf16 MFMA (VITS_WDT_F32S, fp32-level
# error, see csrc/conv1d_impl.h split3_bf16), "exact" = the f32-input MFMA
# (v_mfma_f32_32x32x2_f32, bitwise an fp32 fma chain).  Non-finite
# activations: split fp32 computes x - hi for an inf x as inf - inf, so an
# output the reference's fp32 conv gives as +-inf comes out NaN; outputs stay
# non-finite in exactly the reference's non-finite columns
# (tests/test_kernels_gpu.py::test_conv1d_nonfinite_inputs_stay_nonfinite).
# Weights are split on the host with mid = lo = 0 for non-finite values.
FP32_MODE = os.environ.get("VITS_FP32_MODE", "split")
if FP32_MODE not in ("split", "exact"):
    raise ValueError(f"VITS_FP32_MODE={FP32_MODE!r}: expected 'split' or 'exact'")
FP32_WDTYPE = ops.WDT_F32S if FP32_MODE == "split" else ops.WDT_F32


def get_plan(module: torch.nn.Module, builder):
    sig = _param_signature(module)
    plan = module.__dict__.get(_PLAN_ATTR)
    if plan is None or plan.signature != sig:
        # a bf16 / fp16 model (`model.to(torch.bfloat16)`, `model.half()` as
        # infer.py deploys) runs its convs on the 16-bit-MFMA kernel variant of
        # its own type (fp32 activations, fp32 accumulation); fp32 models run
        # exact fp32
        dt = sig[0][2] if sig[0] is not None else torch.float32
        wdt = {torch.bfloat16: ops.WDT_BF16, torch.float16: ops.WDT_F16}.get(dt, FP32_WDTYPE)
        with torch.no_grad(), ops.pack_lowp(wdt):
            plan = builder(module)
        plan.signature = sig
        module.__dict__[_PLAN_ATTR] = plan
    return plan


def drop_plans(module: torch.nn.Module):
    for m in module.modules():
        m.__dict__.pop(_PLAN_ATTR, None)


def _f32(t: torch.Tensor) -> torch.Tensor:
    return t.detach().to(torch.float32).contiguous()


def _device_of(module):
    return next(module.parameters()).device


class _CondStack:
    """Collects per-utterance Linear layers (weight [n, gin]) into one matrix."""

    def __init__(self):
        self.w, self.b, self.n = [], [], 0

    def add(self, weight: torch.Tensor, bias: Optional[torch.Tensor]) -> int:
        off = self.n
        self.w.append(_f32(weight))
        self.b.append(_f32(bias) if bias is not None else torch.zeros(
            weight.shape[0], device=weight.device))
        self.n += weight.shape[0]
        return off

    def finish(self):
        if not self.w:
            return None, None
        return torch.cat(self.w, 0).contiguous(), torch.cat(self.b, 0).contiguous()


def _linear_eff(lin: torch.nn.Module):
    return ops.weight_norm_effective(lin), lin.bias


def _conv_eff(conv: torch.nn.Module):
    return ops.weight_norm_effective(conv), conv.bias


# ---------------------------------------------------------------------------
# Generator (HiFi-GAN style decoder with gated ResBlock2)
# ---------------------------------------------------------------------------
# grouped launches of the ResBlock2 branches (False: one launch per conv,
# for A/B timing in tools/)
_GROUP_BRANCHES = True
# fused ResBlock2 pairs on the 32/64-channel stages (False: the two-conv
# path, for A/B timing and the parity test of both)
_FUSED_PAIRS = True
# 16-bit models: the last pairs of a stage's branches as one branch-mean
# launch (vits_resblock_pair16_mean_forward); 0 = one accumulating launch each.
# Used on the 32-channel stage (C5: 0.47 -> 0.41 ms); on the 64-channel one
# the summing kernel reaches 256 VGPRs and lost (0.61 -> 0.69 ms)
MEAN_PAIRS16 = True
# 16-bit models keep the decoder's activations 16-bit in HBM (as the
# reference's .half() model holds them): every conv of the Generator reads and
# writes its own 16-bit type (io16), halving the stage traffic.  C5 (B=4,
# Ty=2500, bf16, MI355X): conv time 12.9 -> 12.2 ms/step, SNR vs the fp32
# model 40.9 -> 39.0 dB (fp16: 56.2 dB).  The convs there are epilogue /
# issue-bound rather than HBM-bound, so most of the gain is the global-memory
# weight path these groups can take (conv1d.hip ga16, io16 = 2).
# False: fp32 activations (the 16-bit MFMA on fp32 I/O), for A/B.
ACT16 = True


class GeneratorPlan:
    def __init__(self, gen):
        self.signature = None
        dev = _device_of(gen)
        self.num_kernels = gen.num_kernels
        w, b = _conv_eff(gen.conv_pre)
        self.conv_pre = pack_conv(w, b)
        self.ups = []
        self.stages = []
        conds = _CondStack()
        for i, up in enumerate(gen.ups):
            w, b = _conv_eff(up)
            self.ups.append(pack_conv_transpose(w, b, up.stride[0], up.padding[0]))
            blocks = []
            for j in range(gen.num_kernels):
                rb = gen.resblocks[i * gen.num_kernels + j]
                pairs = []
                for c1, c2, cs in zip(rb.convs1, rb.convs2, rb.conds):
                    w1, b1 = _conv_eff(c1)
                    w2, b2 = _conv_eff(c2)
                    wc, bc = _linear_eff(cs)
                    p1 = pack_conv(w1, b1, dilation=c1.dilation[0], padding=c1.padding[0],
                                   gate=True)
                    p2 = pack_conv(w2, b2, dilation=c2.dilation[0], padding=c2.padding[0])
                    alt = None
                    if (ops.PACK_PRECISION.wdtype == ops.WDT_F32S and p1.wdtype == ops.WDT_F32
                            and p2.wdtype == ops.WDT_F32):
                        # a split-fp32 model's 32-row convs stay exact fp32 as
                        # single convs; the fused split pair takes them too
                        alt = (ops.to_lowp(p1, ops.WDT_F32S, min_rows=0),
                               ops.to_lowp(p2, ops.WDT_F32S, min_rows=0))
                    pairs.append((p1, p2, conds.add(wc, bc), alt))
                blocks.append(pairs)
            self.stages.append(blocks)
        self.cond_w, self.cond_b = conds.finish()
        self.n_cond = conds.n
        self.post_w = _f32(gen.conv_post.weight)
        self.device = dev
        lowp = {ops.WDT_BF16: torch.bfloat16, ops.WDT_F16: torch.float16}
        self.act_dtype = lowp.get(self.conv_pre.wdtype, torch.float32) if ACT16 else torch.float32
        if self.act_dtype != torch.float32:  # 16-bit X staging: wider K-chunks
            layers = [self.conv_pre] + self.ups + [c for blocks in self.stages
                                                   for pairs in blocks for pr in pairs
                                                   for c in pr[:2]]
            for layer in layers:
                layer.kc = ops.io16_kc(layer)

    def conds(self, g: torch.Tensor) -> Optional[torch.Tensor]:
        if self.cond_w is None:
            return None
        return ops.linear_rows(g, self.cond_w, self.cond_b)

    def run(self, x: torch.Tensor, g: torch.Tensor, cond: Optional[torch.Tensor] = None,
            out: Optional[torch.Tensor] = None,
            lengths: Optional[torch.Tensor] = None) -> torch.Tensor:
        """x [B, C_in, T] fp32 -> wav [B, 1, T * prod(u)].  ``lengths``
        (int32 [1 + n_stages, B], device): utterance b ends at lengths[0][b]
        frames (conv_pre) and lengths[i + 1][b] samples after upsampler i -
        every conv output is zero past it, so each utterance sees the zero
        padding of its own end, exactly as the reference's unmasked decoder
        on that many frames (models.py:306-318)."""
        B = x.shape[0]
        if cond is None:
            cond = self.conds(g)
        dev = x.device
        L = (lambda i: None) if lengths is None else (lambda i: lengths[i])
        # (16-bit activations: the conv rounds its input to the operand type
        # anyway, so casting z first leaves conv_pre unchanged)
        h = ops.conv1d(x.to(self.act_dtype), self.conv_pre, lengths=L(0))
        for i, (up, blocks) in enumerate(zip(self.ups, self.stages)):
            xu = ops.conv1d(h, up, in_slope=0.1, lengths=L(i + 1))
            C, T = xu.shape[1], xu.shape[2]
            xs = torch.empty(B, C, T, device=dev, dtype=xu.dtype)
            self._run_stage(blocks, xu, xs, cond, B, dev, L(i + 1))
            h = xs
        return ops.conv_post_tanh(h, self.post_w, out=out)

    @staticmethod
    def _run_stage(blocks, xu, xs, cond, B, dev, lengths=None):
        """The nk ResBlock2 branches of one stage (models.py:311-313) on xu,
        their mean into xs.  Branches are independent until the mean: each
        keeps its own buffers, and the work of one dilation index of all
        branches shares launches - fused pairs (csrc/resblock.hip, where
        ops.resblock_pair_supported) as one launch, the other branches' c1
        (gate epilogue) and c2 (residual epilogue) convs as one grouped
        launch each.  The last pairs accumulate the mean into xs in branch
        order (separate launches)."""
        nk = len(blocks)
        npairs = len(blocks[0])
        if any(len(pairs) != npairs for pairs in blocks):
            raise NotImplementedError("ResBlock2 branches with different dilation counts")
        C, T = xu.shape[1], xu.shape[2]
        io16 = 2 if xu.dtype != torch.float32 else 0  # (2: inference decoder, conv1d.hip ga16)

        def fused_layers(pr):
            """(c1, c2) the fused pair kernel runs for this pair, or None."""
            if io16:  # 16-bit model, 16-bit activations: csrc/resblock16.hip
                return pr[:2] if ops.resblock_pair16_supported(pr[0], pr[1], xu) else None
            if not _FUSED_PAIRS:
                return None
            # split fp32 (resblock_f32p.hip) first: on the 32-channel stage it
            # beats the exact pair (k=7 -30 %, k=11 -35 %, tools/rbp_bench.py)
            for c1, c2 in ((pr[0], pr[1]),) + ((pr[3],) if pr[3] is not None else ()):
                if ops.resblock_pair_f32p_supported(c1, c2, xu):
                    return c1, c2
            return pr[:2] if ops.resblock_pair_supported(pr[0], pr[1], T) else None

        fused = [[fused_layers(pr) for pr in pairs] for pairs in blocks]

        def pair_desc(j, p, dst, **kw):
            fn = ops.resblock_pair16_desc if io16 else ops.resblock_pair_desc
            c1, c2 = fused[j][p]
            return fn(c1, c2, cur[j], dst, cond=cond, cond_offset=blocks[j][p][2],
                      lengths=lengths, **kw)

        def pair_launch(js, p, dsts, **kw):
            """The fused pairs of branches js (one launch per weight type)."""
            if io16:
                ops.resblock_pair16_launch(tuple(pair_desc(j, p, d, **kw) for j, d in zip(js, dsts)),
                                           B, dev, blocks[0][0][0].wdtype)
                return
            for wdt in sorted({fused[j][p][0].wdtype for j in js}):
                sel = [(j, d) for j, d in zip(js, dsts) if fused[j][p][0].wdtype == wdt]
                ops.resblock_pair_launch(tuple(pair_desc(j, p, d, **kw) for j, d in sel), B, dev,
                                         wdt)
        tmp = [[torch.empty_like(xs), torch.empty_like(xs)] for _ in range(nk)]
        gbuf = [None if all(fused[j]) else
                torch.empty(B, C // 2, T, device=dev, dtype=xu.dtype) for j in range(nk)]
        cur = [xu] * nk

        def c1_desc(j, p):
            return make_desc(blocks[j][p][0], cur[j], make_out(gbuf[j]), in_slope=0.1, cond=cond,
                             cond_offset=blocks[j][p][2], lengths=lengths, io16=io16)

        def grouped(ds):
            return [tuple(ds)] if _GROUP_BRANCHES else list(ds)

        for p in range(npairs):
            fj = [j for j in range(nk) if fused[j][p]]
            cj = [j for j in range(nk) if not fused[j][p]]
            if p < npairs - 1:
                dst = [tmp[j][p & 1] for j in range(nk)]
                if fj:
                    pair_launch(fj, p, [dst[j] for j in fj])
                if cj:
                    descs = grouped(c1_desc(j, p) for j in cj)
                    descs += grouped(make_desc(blocks[j][p][1], gbuf[j],
                                               make_out(dst[j], res=cur[j]), lengths=lengths,
                                               io16=io16)
                                     for j in cj)
                    ops.conv1d_launch_seq(descs, B, dev)
                cur = dst
                continue
            # last pair of every branch: accumulate the mean, in branch order
            if io16 and not cj and 1 < nk <= 3 and MEAN_PAIRS16 and C == 32:
                # every branch fused: one launch sums them in registers
                ops.resblock_pair16_launch(tuple(pair_desc(j, p, xs) for j in range(nk)), B,
                                           dev, blocks[0][0][0].wdtype, mean=True)
                continue
            if cj:  # (an empty group would be an empty launch)
                ops.conv1d_launch_seq(grouped(c1_desc(j, p) for j in cj), B, dev)
            for j in range(nk):
                kw = dict(accumulate=j > 0, post_div=float(nk) if j == nk - 1 else 1.0)
                if fused[j][p]:
                    pair_launch([j], p, [xs], **kw)
                else:
                    ops.conv1d_launch_seq([make_desc(blocks[j][p][1], gbuf[j],
                                                     make_out(xs, res=cur[j], **kw),
                                                     lengths=lengths, io16=io16)], B, dev)


# ---------------------------------------------------------------------------
# WN stack (shared by coupling layers and the posterior encoder)
# ---------------------------------------------------------------------------
class WNPlan:
    def __init__(self, wn, conds: Optional[_CondStack]):
        self.H = wn.hidden_channels
        self.n_layers = wn.n_layers
        self.cond_off = None
        if wn.gin_channels != 0:
            wc, bc = _linear_eff(wn.cond_layer)
            self.cond_off = conds.add(wc, bc)
        self.in_layers = []
        self.res_skip = []
        for i in range(wn.n_layers):
            w, b = _conv_eff(wn.in_layers[i])
            self.in_layers.append(pack_conv(w, b, dilation=wn.in_layers[i].dilation[0],
                                            padding=wn.in_layers[i].padding[0], gate=True))
            w, b = _conv_eff(wn.res_skip_layers[i])
            self.res_skip.append(pack_conv(w, b))

    def descs(self, h: torch.Tensor, skip: torch.Tensor, abuf: torch.Tensor,
              cond: Optional[torch.Tensor], lengths: Optional[torch.Tensor]):
        """h [B,H,T] is updated in place (residual stream), skip receives the
        WN output (masked at the last layer when lengths are given)."""
        H = self.H
        out = []
        for i in range(self.n_layers):
            coff = 0 if self.cond_off is None else self.cond_off + 2 * H * i
            out.append(make_desc(self.in_layers[i], h, make_out(abuf),
                                 cond=cond if self.cond_off is not None else None,
                                 cond_offset=coff))
            last = i == self.n_layers - 1
            if not last:
                out.append(make_desc(self.res_skip[i], abuf, make_out(h, res=h),
                                     out1=make_out(skip, accumulate=i > 0), split=H,
                                     lengths=lengths))
            else:
                # only the final skip write is masked: (output + rs) * mask
                out.append(make_desc(self.res_skip[i], abuf,
                                     make_out(skip, accumulate=i > 0), lengths=lengths))
        return out


# ---------------------------------------------------------------------------
# reverse flow (ResidualCouplingBlock) — the Flip modules are folded away
# ---------------------------------------------------------------------------
class CouplingFlowPlan:
    """Runs ``flows_reversed`` in place on one [B, 2*half, T] buffer.

    Every Flip is absorbed into the weights: after an odd number of flips the
    logical first half lives reversed in the physical second half, so that
    coupling reads physical channels [half, 2*half) with its ``pre`` input
    channels reversed and updates physical [0, half) with its ``post`` output
    channels reversed.  The number of flips is even, so the buffer ends in
    the reference's channel order."""

    def __init__(self, block):
        self.signature = None
        conds = _CondStack()
        self.layers = []
        flipped = False
        for f in block.flows_reversed:
            if f.__class__.__name__ == "Flip":
                flipped = not flipped
                continue
            assert f.mean_only, "only mean-only couplings are on the hot path"
            half = f.half_channels
            wp, bp = _conv_eff(f.pre)
            wq, bq = _conv_eff(f.post)
            if flipped:
                wp = wp.flip(1)
                wq, bq = wq.flip(0), bq.flip(0)
            self.layers.append(dict(
                half=half, flipped=flipped,
                pre=pack_conv(wp, bp), post=pack_conv(wq, bq),
                wn=WNPlan(f.enc, conds)))
        assert not flipped, "odd number of Flip modules"
        self.cond_w, self.cond_b = conds.finish()
        self.H = self.layers[0]["wn"].H if self.layers else 0

    def conds(self, g):
        if self.cond_w is None:
            return None
        return ops.linear_rows(g, self.cond_w, self.cond_b)

    def run_(self, z: torch.Tensor, g: torch.Tensor, cond: Optional[torch.Tensor] = None,
             lengths: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Reverse flow in place on z [B, 2*half, T] (fp32 contiguous)."""
        B, _, T = z.shape
        if cond is None:
            cond = self.conds(g)
        dev = z.device
        H = self.H
        h = torch.empty(B, H, T, device=dev, dtype=torch.float32)
        skip = torch.empty_like(h)
        abuf = torch.empty_like(h)
        descs = []
        for L in self.layers:
            half = L["half"]
            src_off, dst_off = (half, 0) if L["flipped"] else (0, half)
            descs.append(make_desc(L["pre"], z, make_out(h), x_channel_offset=src_off,
                                   lengths=lengths))
            descs += L["wn"].descs(h, skip, abuf, cond, lengths)
            descs.append(make_desc(L["post"], skip, make_out(
                z, res=z, res_scale=-1.0, channel_offset=dst_off), lengths=lengths))
        ops.conv1d_launch_seq(descs, B, dev)
        return z


# ---------------------------------------------------------------------------
# Text encoder (+ projection) and duration predictor
# ---------------------------------------------------------------------------
class TextEncoderPlan:
    def __init__(self, enc):
        self.signature = None
        dev = _device_of(enc)
        self.hidden = enc.hidden_channels
        self.out_channels = enc.out_channels
        self.n_heads = enc.n_heads
        lin = enc.emb[0]
        self.emb = pack_conv(lin.weight.unsqueeze(-1), lin.bias)  # Linear as 1x1 conv
        ln = enc.emb[1]
        self.emb_ln = (_f32(ln.weight), _f32(ln.bias), ln.eps)
        self.emo_w, self.emo_b = _f32(enc.emo_proj.weight), _f32(enc.emo_proj.bias)
        self.xscale = float(enc.xscale)
        self.alpha = enc.alpha  # device scalar, read in-kernel
        self.sin_table = enc.sin_table
        conds = _CondStack()
        self.layers = []
        E = enc.encoder
        for i in range(E.n_layers):
            a = E.attn_layers[i]
            wqkv = torch.cat([a.conv_q.weight, a.conv_k.weight, a.conv_v.weight], 0)
            bqkv = torch.cat([a.conv_q.bias, a.conv_k.bias, a.conv_v.bias], 0)
            f = E.ffn_layers[i]
            n1, n2 = E.norm_layers_1[i], E.norm_layers_2[i]
            self.layers.append(dict(
                qkv=pack_conv(wqkv, bqkv), o=pack_conv(a.conv_o.weight, a.conv_o.bias),
                n1=(_f32(n1.gamma), _f32(n1.beta), n1.eps),
                ffn1=pack_conv(f.conv_1.weight, f.conv_1.bias, gate=True),
                ffn2=pack_conv(f.conv_2.weight, f.conv_2.bias),
                cond_off=conds.add(f.cond.weight, f.cond.bias),
                n2=(_f32(n2.gamma), _f32(n2.beta), n2.eps),
                filt=f.filter_channels))
        self.cond_w, self.cond_b = conds.finish()
        self.proj = pack_conv(enc.proj.weight, enc.proj.bias)
        self.device = dev

    def _pe(self, T, dev):
        if T <= self.sin_table.size(1):
            return self.sin_table[0, :T].to(dev, torch.float32).contiguous()
        from .commons import gen_sin_table

        return gen_sin_table(T, self.hidden)[0].to(dev).contiguous()

    def run(self, x: torch.Tensor, emo: torch.Tensor, g: torch.Tensor,
            lengths: Optional[torch.Tensor] = None, exp_logs: bool = False,
            pad_exact: bool = False):
        """x [B, T, text_channels] (time-major, as the reference takes it).
        Returns (h [B,H,T], m [B,C,T], logs_or_s [B,C,T]).

        lengths: TextEncoder.forward's masking (models.py:167-178,
        attentions.py:34-46: keys masked, FFN2's conv_2 input masked, but its
        conv_1 reads the unmasked post-LN activations of padded positions).
        pad_exact (with lengths): every LayerNorm output is zeroed past the
        length as well, so each utterance computes exactly what
        TextEncoder.infer computes on its unpadded tokens (models.py:180-189:
        the convs see zero padding at the utterance end) - the padded-text
        buckets of SynthesizerTrn.infer_bucketed."""
        x = _f32(x)
        B, T, _ = x.shape
        dev = x.device
        Hc = self.hidden
        xt = x.transpose(1, 2)  # view [B, C, T] with time stride C: read in place
        e = torch.empty(B, Hc, T, device=dev, dtype=torch.float32)
        ops.conv1d_launch(make_desc(self.emb, xt, make_out(e)), B, dev)
        emo_v = ops.linear_rows(_f32(emo), self.emo_w, self.emo_b)
        gam, bet, eps = self.emb_ln
        h = torch.empty_like(e)
        ops.layer_norm_channels(e, gam, bet, eps, out=h, post_add=emo_v, scale=self.xscale,
                                pos=self._pe(T, dev), pos_alpha=self.alpha.detach().float(),
                                lengths=lengths)
        cond = ops.linear_rows(_f32(g), self.cond_w, self.cond_b)
        qkv = torch.empty(B, 3 * Hc, T, device=dev, dtype=torch.float32)
        att = torch.empty(B, Hc, T, device=dev, dtype=torch.float32)
        y = torch.empty_like(att)
        for li, L in enumerate(self.layers):
            last = li == len(self.layers) - 1
            ops.conv1d_launch(make_desc(L["qkv"], h, make_out(qkv)), B, dev)
            _attention_into(qkv, Hc, self.n_heads, lengths, att)
            ops.conv1d_launch(make_desc(L["o"], att, make_out(y)), B, dev)
            g1, b1, e1 = L["n1"]
            ops.layer_norm_channels(h, g1, b1, e1, residual=y, out=h,
                                    lengths=lengths if pad_exact else None)
            gb = torch.empty(B, L["filt"], T, device=dev, dtype=torch.float32)
            ops.conv1d_launch(make_desc(L["ffn1"], h, make_out(gb), cond=cond,
                                        cond_offset=L["cond_off"], lengths=lengths), B, dev)
            ops.conv1d_launch(make_desc(L["ffn2"], gb, make_out(y), lengths=lengths), B, dev)
            g2, b2, e2 = L["n2"]
            # Encoder.forward ends with x * x_mask (attentions.py:46): the last
            # LayerNorm zeroes t >= length in its epilogue
            ops.layer_norm_channels(h, g2, b2, e2, residual=y, out=h,
                                    lengths=lengths if (last or pad_exact) else None)
        Cc = self.out_channels
        m = torch.empty(B, Cc, T, device=dev, dtype=torch.float32)
        s = torch.empty_like(m)
        ops.conv1d_launch(make_desc(self.proj, h, make_out(m), out1=make_out(
            s, act=ACT_EXP if exp_logs else ACT_NONE), split=Cc, lengths=lengths), B, dev)
        return h, m, s


def _attention_into(qkv, Hc, n_heads, lengths, out):
    """Attention over the fused [B, 3H, T] q|k|v projection output."""
    from . import _lib

    B, _, T = qkv.shape
    D = Hc // n_heads
    ops.require_device(qkv)
    lib = _lib.load()
    base = qkv.data_ptr()
    step = 4 * Hc * qkv.stride(1)
    _lib.check(lib.vits_attention_forward(base, base + step, base + 2 * step, out.data_ptr(), B,
                                          n_heads, D, T, qkv.stride(0), out.stride(0),
                                          None if lengths is None else lengths.data_ptr(),
                                          ops._stream_ptr(qkv.device)), "vits_attention_forward")
    return out


class DurationPlan:
    def __init__(self, dp):
        self.signature = None
        self.pre = pack_conv(dp.pre.weight, dp.pre.bias)
        self.conv_1 = pack_conv(dp.conv_1.weight, dp.conv_1.bias)
        self.conv_2 = pack_conv(dp.conv_2.weight, dp.conv_2.bias)
        self.proj = pack_conv(dp.proj.weight, dp.proj.bias)
        self.n1 = (_f32(dp.norm_1.gamma), _f32(dp.norm_1.beta), dp.norm_1.eps)
        self.n2 = (_f32(dp.norm_2.gamma), _f32(dp.norm_2.beta), dp.norm_2.eps)
        conds = _CondStack()
        self.c1 = conds.add(dp.cond1.weight, dp.cond1.bias)
        self.c2 = conds.add(dp.cond2.weight, dp.cond2.bias)
        self.cond_w, self.cond_b = conds.finish()
        self.F = dp.filter_channels
        act = dp.act_1.__class__.__name__
        if act != "ReLU":
            raise NotImplementedError("DurationPredictor HIP path implements act_func_d='ReLU'")

    def run(self, x: torch.Tensor, g: torch.Tensor, lengths: Optional[torch.Tensor] = None):
        B, _, T = x.shape
        dev = x.device
        cond = ops.linear_rows(_f32(g), self.cond_w, self.cond_b)
        a = torch.empty(B, self.F, T, device=dev, dtype=torch.float32)
        b = torch.empty_like(a)
        # x = pre(x) + cond1(g); masked before conv_1 (models.py:49-50)
        ops.conv1d_launch(make_desc(self.pre, x, make_out(a), cond=cond, cond_offset=self.c1,
                                    lengths=lengths), B, dev)
        ops.conv1d_launch(make_desc(self.conv_1, a, make_out(b, act=ACT_RELU)), B, dev)
        g1, b1, e1 = self.n1
        ops.layer_norm_channels(b, g1, b1, e1, out=a, post_add=cond[:, self.c2:self.c2 + self.F],
                                lengths=lengths)
        ops.conv1d_launch(make_desc(self.conv_2, a, make_out(b, act=ACT_RELU)), B, dev)
        g2, b2, e2 = self.n2
        ops.layer_norm_channels(b, g2, b2, e2, out=a, lengths=lengths)
        logw = torch.empty(B, 1, T, device=dev, dtype=torch.float32)
        ops.conv1d_launch(make_desc(self.proj, a, make_out(logw), lengths=lengths), B, dev)
        return logw


class PosteriorPlan:
    def __init__(self, enc_q):
        self.signature = None
        self.pre = pack_conv(enc_q.pre[0].weight, enc_q.pre[0].bias)
        ln = enc_q.pre[1]
        self.ln = (_f32(ln.gamma), _f32(ln.beta), ln.eps)
        conds = _CondStack()
        self.wn = WNPlan(enc_q.enc, conds)
        self.cond_w, self.cond_b = conds.finish()
        self.proj = pack_conv(enc_q.proj.weight, enc_q.proj.bias)
        self.out_channels = enc_q.out_channels
        self.H = enc_q.hidden_channels

    def run(self, spec: torch.Tensor, noise: torch.Tensor, g=None, lengths=None):
        """PosteriorEncoder.infer (models.py:273-279): z = m + n * exp(logs)."""
        B, _, T = spec.shape
        dev = spec.device
        h0 = torch.empty(B, self.H, T, device=dev, dtype=torch.float32)
        ops.conv1d_launch(make_desc(self.pre, _f32(spec), make_out(h0)), B, dev)
        g1, b1, e1 = self.ln
        h = torch.empty_like(h0)
        ops.layer_norm_channels(h0, g1, b1, e1, out=h, lengths=lengths)
        cond = None if self.cond_w is None else ops.linear_rows(_f32(g), self.cond_w, self.cond_b)
        skip = torch.empty_like(h)
        ops.conv1d_launch_seq(self.wn.descs(h, skip, h0, cond, lengths), B, dev)
        Cc = self.out_channels
        m = torch.empty(B, Cc, T, device=dev, dtype=torch.float32)
        s = torch.empty_like(m)
        ops.conv1d_launch(make_desc(self.proj, skip, make_out(m), out1=make_out(s, act=ACT_EXP),
                                    split=Cc, lengths=lengths), B, dev)
        z = torch.empty_like(m)
        z.copy_(m).addcmul_(_f32(noise), s)
        return z


# ---------------------------------------------------------------------------
# module-level entry points used by modules.py / attentions.py / models.py
# ---------------------------------------------------------------------------

def _check_gpu(x: torch.Tensor, what: str):
    if x.device.type != "cuda":
        raise ops._lib.VitsAmdError(
            f"{what}: the vits_amd inference path runs on a ROCm GPU only (got {x.device})")


def generator_forward(gen, x: torch.Tensor, g: torch.Tensor) -> torch.Tensor:
    _check_gpu(x, "Generator")
    plan = get_plan(gen, GeneratorPlan)
    out = plan.run(_f32(x), _f32(g))
    return out.to(x.dtype)


def flow_infer(block, x: torch.Tensor, g: torch.Tensor) -> torch.Tensor:
    _check_gpu(x, "ResidualCouplingBlock.infer")
    plan = get_plan(block, CouplingFlowPlan)
    z = _f32(x).clone()
    plan.run_(z, _f32(g))
    return z.to(x.dtype)


def flow_reverse_masked(block, x: torch.Tensor, lengths: torch.Tensor, g: torch.Tensor):
    _check_gpu(x, "ResidualCouplingBlock(reverse=True)")
    plan = get_plan(block, CouplingFlowPlan)
    z = _f32(x).clone()
    plan.run_(z, _f32(g), lengths=lengths.to(torch.int32).contiguous())
    return z.to(x.dtype)


def coupling_infer(layer, x, g):
    """Single ResidualCouplingLayer.infer through a one-layer plan."""
    _check_gpu(x, "ResidualCouplingLayer.infer")

    class _One:
        flows_reversed = [layer]

    plan = layer.__dict__.get("_vits_amd_single")
    sig = _param_signature(layer)
    if plan is None or plan.signature != sig:
        with torch.no_grad():
            plan = CouplingFlowPlan(_One)
        plan.signature = sig
        layer.__dict__["_vits_amd_single"] = plan
    z = _f32(x).clone()
    plan.run_(z, _f32(g) if g is not None else None)
    return z.to(x.dtype)


def wn_infer(wn, x, g=None):
    _check_gpu(x, "WN.infer")

    class _Holder:
        pass

    plan = wn.__dict__.get("_vits_amd_wn")
    sig = _param_signature(wn)
    if plan is None or plan.signature != sig:
        with torch.no_grad():
            conds = _CondStack()
            wp = WNPlan(wn, conds)
            plan = _Holder()
            plan.wn = wp
            plan.cond_w, plan.cond_b = conds.finish()
        plan.signature = sig
        wn.__dict__["_vits_amd_wn"] = plan
    h = _f32(x).clone()
    B, H, T = h.shape
    skip = torch.empty_like(h)
    abuf = torch.empty_like(h)
    cond = None if plan.cond_w is None else ops.linear_rows(_f32(g), plan.cond_w, plan.cond_b)
    ops.conv1d_launch_seq(plan.wn.descs(h, skip, abuf, cond, None), B, h.device)
    return skip.to(x.dtype)


def resblock_infer(rb, x, g):
    _check_gpu(x, "ResBlock2")

    class _Gen:
        pass

    plan = rb.__dict__.get("_vits_amd_rb")
    sig = _param_signature(rb)
    if plan is None or plan.signature != sig:
        with torch.no_grad():
            conds = _CondStack()
            pairs = []
            for c1, c2, cs in zip(rb.convs1, rb.convs2, rb.conds):
                w1, b1 = _conv_eff(c1)
                w2, b2 = _conv_eff(c2)
                wc, bc = _linear_eff(cs)
                pairs.append((pack_conv(w1, b1, dilation=c1.dilation[0], padding=c1.padding[0],
                                        gate=True),
                              pack_conv(w2, b2, dilation=c2.dilation[0], padding=c2.padding[0]),
                              conds.add(wc, bc)))
            plan = _Gen()
            plan.pairs = pairs
            plan.cond_w, plan.cond_b = conds.finish()
        plan.signature = sig
        rb.__dict__["_vits_amd_rb"] = plan
    xf = _f32(x)
    B, C, T = xf.shape
    cond = ops.linear_rows(_f32(g), plan.cond_w, plan.cond_b)
    gbuf = torch.empty(B, C // 2, T, device=x.device, dtype=torch.float32)
    cur = xf
    for c1, c2, coff in plan.pairs:
        ops.conv1d_launch(make_desc(c1, cur, make_out(gbuf), in_slope=0.1, cond=cond,
                                    cond_offset=coff), B, x.device)
        nxt = torch.empty(B, C, T, device=x.device, dtype=torch.float32)
        ops.conv1d_launch(make_desc(c2, gbuf, make_out(nxt, res=cur)), B, x.device)
        cur = nxt
    return cur.to(x.dtype)


def encoder_infer(encoder, x, g):
    raise NotImplementedError(
        "attentions.Encoder.infer standalone: call TextEncoder.infer / SynthesizerTrn.infer_p1, "
        "which lower the whole encoder (embedding + layers + projection) at once")


__all__ = [
    "GeneratorPlan", "CouplingFlowPlan", "TextEncoderPlan", "DurationPlan", "PosteriorPlan",
    "get_plan", "drop_plans", "generator_forward", "flow_infer", "flow_reverse_masked",
    "coupling_infer", "wn_infer", "resblock_infer", "math",
]
