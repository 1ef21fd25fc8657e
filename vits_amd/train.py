"""Data-parallel training step of ``train_stft.py`` on the vits_amd modules.

``TrainStep.step`` reproduces one iteration of the reference hot loop
(train_stft.py:162-236): fp16 autocast G forward (HIP monotonic alignment
search inside), logging mels, waveform slice, MR-STFT loss on the HIP STFT
kernels (forward + adjoint), D forward on real / detached fake, D loss ->
scaled backward -> unscale -> grad norm -> RAdam step; D forward on fake,
G losses (dur, stft, kl, kl_q, adversarial) -> scaled backward -> AdamW step
-> scaler update.  Under ``torch.distributed`` both networks are DDP-wrapped
(train_stft.py:108-110): the only collective is DDP's bucketed gradient
all-reduce over RCCL/xGMI (the ``nccl`` backend on ROCm).

Differences from the reference, all on the host side: per-discriminator
losses stay on the device (no ``.item()`` per loss, losses.py:28-29) and the
grad norm is reduced on the device once (commons.py:158-173 syncs per
parameter); the D optimizer is radam.py's RAdam as one fused HIP launch
(vits_amd.optim.FusedRAdam, GradScaler-aware without a host sync).

``capture()`` records the whole step into one hipGraph (single process):
the step is then GPU-bound instead of bound by ~14k host-side launches.
"""
from __future__ import annotations

import argparse
import contextlib
import os
import sys
import time

import torch
import torch.distributed as dist
from torch.nn.parallel import DistributedDataParallel as DDP

from . import commons, train_ops, utils
from .discriminators import MultiWaveSTFTDiscriminator
from .losses import discriminator_loss, feature_loss, generator_loss, kl_loss
from .mel_processing import mel_spectrogram_torch, spec_to_mel_torch
from .models import MultiPeriodDiscriminator, SynthesizerTrn
from .optim import FusedRAdam, RAdam
from .stft_loss import MultiResolutionSTFTLoss
from .wnorm import WeightNormCache


def build_models(hps, device, variant: str = "stft"):
    """(net_g, net_d): variant "stft" = train_stft.py (MWSD discriminator,
    train_stft.py:88-90), "mel" = train.py (MultiPeriodDiscriminator,
    train.py:74-83)."""
    net_g = SynthesizerTrn(hps.data.text_channels, hps.data.filter_length // 2 + 1,
                           hps.train.segment_size // hps.data.hop_length,
                           n_speakers=hps.data.n_speakers, align_noise=hps.train.align_noise,
                           align_noise_decay=hps.train.align_noise_decay, **hps.model).to(device)
    if variant == "mel":
        net_d = MultiPeriodDiscriminator(hps.model.get("use_spectral_norm", False)).to(device)
    else:
        net_d = MultiWaveSTFTDiscriminator().to(device)
    return net_g, net_d


def _layer_prefixes(stem: str, names, idx):
    return tuple(f"{stem}{n}.{i}." for n in names for i in idx)


# G's gradient buckets for the overlapped all-reduce: each is a tuple of
# parameter-name prefixes (a parameter joins the first bucket with a matching
# prefix; "" matches all).  Ordered as the backward finishes them, and each at
# most ~50 MB of fp32 gradients (base.json sizes in the comments): the
# decoder's late stages first (their weight-norm group's backward fires as
# soon as their last conv's weight gradient is in), then its first stage, the
# flow's couplings (reverse order of the forward), the posterior encoder's
# upper and lower WN layers, the text encoder's upper and lower blocks, and
# the rest (speaker embedding, duration predictor).  Every bucket is also one
# weight-norm group (wnorm.WeightNormCache), so its gradients are final
# together.
G_BUCKETS = (
    ("dec.ups.1.", "dec.ups.2.", "dec.ups.3.", "dec.conv_post.")
    + tuple(f"dec.resblocks.{i}." for i in range(3, 12)),                  # 18 MB
    ("dec.",),                                                               # 45 MB
    ("flow.flows.6.", "flow.flows.4."),                                      # 42 MB
    ("flow.",),                                                              # 42 MB
    _layer_prefixes("enc_q.enc.", ("in_layers", "res_skip_layers"), range(8, 16))
    + ("enc_q.proj.",),                                                      # 25 MB
    ("enc_q.",),                                                             # 26 MB
    _layer_prefixes("enc_p.encoder.", ("attn_layers", "norm_layers_1", "ffn_layers",
                                       "norm_layers_2"), range(3, 6)),       # 39 MB
    ("enc_p.",),                                                             # 41 MB
    ("",),                                                                   # 13 MB
)


def _bucket_of(name: str, buckets) -> int:
    return next(i for i, pres in enumerate(buckets) if any(name.startswith(p) for p in pres))


class _GradBuckets:
    """Bucketed, overlapped gradient all-reduce for one network (the
    graph-capturable counterpart of DDP's reducer, train_stft.py:108-110):
    each parameter's post-accumulate-grad hook counts its bucket down; a
    bucket whose gradients are all final is averaged over the ranks - on the
    GPU on a side stream (forked from the backward's stream by an event:
    copy into one flat buffer, one RCCL all-reduce over xGMI, scale, copy
    back) while the backward of the earlier layers continues; on CPU (gloo)
    synchronously.

    Collectives must pair up across ranks, so buckets are launched strictly
    by index (as DDP's reducer does): a bucket that completes early waits
    until every lower-indexed bucket has been launched.  finish() launches
    whatever is still waiting, in order, and joins the side stream.  Every
    bucket always holds ALL its parameters: one without a gradient this step
    (unused on this rank - an error under the reference's DDP) contributes
    zeros, so every rank's flat layout is the same."""

    def __init__(self, net, buckets, device):
        self.device = device
        named = [(n, p) for n, p in net.named_parameters() if p.requires_grad]
        self.buckets = [[] for _ in buckets]
        for n, p in named:
            self.buckets[_bucket_of(n, buckets)].append(p)
        self.buckets = [b for b in self.buckets if b]
        self.comm = torch.cuda.Stream(device) if device.type == "cuda" else None
        self._flat = [None] * len(self.buckets)
        self._left = None
        self._hooks = []
        for bi, ps in enumerate(self.buckets):
            for p in ps:
                self._hooks.append(p.register_post_accumulate_grad_hook(
                    lambda p, bi=bi: self._arrived(bi)))

    def begin(self):
        self._left = [len(b) for b in self.buckets]
        self._next = 0  # lowest bucket index not yet launched

    def _arrived(self, bi):
        if self._left is None:  # (a backward outside step(): no all-reduce)
            return
        self._left[bi] -= 1
        # launch, in index order, every bucket whose gradients are complete
        while self._next < len(self.buckets) and self._left[self._next] == 0:
            self._launch(self._next)
            self._next += 1

    def _launch(self, bi):
        ps = self.buckets[bi]
        for p in ps:
            if p.grad is None:
                p.grad = torch.zeros_like(p)
        if self._flat[bi] is None:
            flat = torch.empty(sum(p.numel() for p in ps), device=ps[0].device,
                               dtype=torch.float32)
            views, o = [], 0
            for p in ps:
                views.append(flat[o:o + p.numel()].view_as(p))
                o += p.numel()
            self._flat[bi] = (flat, views)
        flat, views = self._flat[bi]
        grads = [p.grad for p in ps]
        if self.comm is None:
            torch._foreach_copy_(views, grads)
            dist.all_reduce(flat)
            flat.div_(dist.get_world_size())
            torch._foreach_copy_(grads, views)
            return
        main = torch.cuda.current_stream(self.device)
        self.comm.wait_stream(main)  # this bucket's gradients are final on `main`
        with torch.cuda.stream(self.comm):
            torch._foreach_copy_(views, grads)
            dist.all_reduce(flat)
            flat.div_(dist.get_world_size())
            torch._foreach_copy_(grads, views)

    def finish(self):
        while self._next < len(self.buckets):
            self._launch(self._next)
            self._next += 1
        self._left = None
        if self.comm is not None:
            torch.cuda.current_stream(self.device).wait_stream(self.comm)


class TrainStep:
    def __init__(self, hps, net_g, net_d, device, ddp=False, log_mels=True, fused_adamw=True,
                 capturable=False, allreduce=False, variant: str = "stft"):
        """ddp: wrap both networks in DDP (eager steps).  allreduce: the
        graph-capturable alternative for multi-process runs - no DDP hooks;
        rank 0's parameters/buffers are broadcast once, G's gradients are
        averaged in buckets that overlap its backward (_GradBuckets,
        G_BUCKETS; allreduce="flat": one flat all-reduce after the
        backward) and D's with one flat RCCL all-reduce after its backward
        (the same averaged-gradient semantics as DDP)."""
        assert not (ddp and allreduce)
        assert variant in ("stft", "mel"), variant
        # "stft": train_stft.py (MWSD D + MR-STFT loss, D optimizer RAdam);
        # "mel": train.py (MultiPeriodDiscriminator + mel-L1 + feature
        # matching, D optimizer AdamW with weight_decay 0, train.py:93-99)
        self.variant = variant
        self.hps = hps
        self.device = device
        self.log_mels = log_mels
        # capturable: optimizer steps and the GradScaler skip rule stay on the
        # device (no host sync), so the whole step can be captured (capture())
        self.capturable = bool(capturable) and device.type == "cuda"
        self.graph = None
        self.mstft = MultiResolutionSTFTLoss().to(device)
        # under capture the learning rates are device tensors: the kernels read
        # them at replay time, so the ExponentialLR schedulers below (which
        # fill_ tensor lrs in place) keep working on a captured step
        lr_of = (lambda v: torch.tensor(float(v), device=device)) if self.capturable \
            else (lambda v: v)
        self.optim_g = torch.optim.AdamW(net_g.parameters(), lr_of(hps.train.learning_rate),
                                         betas=hps.train.betas, weight_decay=hps.train.weight_decay,
                                         eps=hps.train.eps,
                                         fused=fused_adamw and device.type == "cuda",
                                         capturable=self.capturable)
        # radam.py's RAdam (train_stft.py:97): one fused HIP launch on the GPU
        # (GradScaler-aware, sync-free); torch's RAdam (same update) on CPU
        if variant == "mel":
            self.optim_d = torch.optim.AdamW(net_d.parameters(), lr_of(hps.train.learning_rate),
                                             betas=hps.train.betas, weight_decay=0,
                                             eps=hps.train.eps,
                                             fused=fused_adamw and device.type == "cuda",
                                             capturable=self.capturable)
        elif device.type == "cuda":
            self.optim_d = FusedRAdam(
                net_d.parameters(),
                torch.tensor(1e-4, device=device, dtype=torch.float64) if self.capturable else 1e-4)
        else:
            self.optim_d = RAdam(net_d.parameters(), 1e-4)
        # train_stft.py:127-128 / train.py:135-136; stepped once per epoch by
        # the caller (end_epoch(), train_stft.py:138-139)
        if self.capturable:
            # a checkpoint load (utils.load_checkpoint -> load_state_dict)
            # writes into the lr / moment tensors the captured graph reads
            utils.pin_optimizer_state(self.optim_g)
            utils.pin_optimizer_state(self.optim_d)
        self.scheduler_g = torch.optim.lr_scheduler.ExponentialLR(
            self.optim_g, gamma=hps.train.lr_decay, last_epoch=-1)
        self.scheduler_d = torch.optim.lr_scheduler.ExponentialLR(
            self.optim_d, gamma=hps.train.lr_decay, last_epoch=-1)
        if ddp:
            ids = [device.index] if device.type == "cuda" else None
            net_g = DDP(net_g, device_ids=ids)
            net_d = DDP(net_d, device_ids=ids)
        self.allreduce = bool(allreduce) and dist.is_available() and dist.is_initialized()
        self._flat = {}
        self._gbuckets = (_GradBuckets(net_g, G_BUCKETS, device)
                          if self.allreduce and allreduce != "flat" else None)
        if self.allreduce:
            with torch.no_grad():
                for net in (net_g, net_d):
                    for t in list(net.parameters()) + list(net.buffers()):
                        dist.broadcast(t, src=0)
        self.net_g, self.net_d = net_g, net_d
        # every weight-normed generator layer in one launch each way (GPU)
        self._wn_g = (WeightNormCache(net_g.module if isinstance(net_g, DDP) else net_g,
                                      G_BUCKETS if self._gbuckets is not None else (("",),))
                      if device.type == "cuda" else None)
        fp16 = bool(hps.train.fp16_run) and device.type == "cuda"
        # the autocast weight-cast cache must be off under graph capture (cached
        # fp16 weight copies would outlive / escape the captured region)
        cache = not self.capturable
        self.autocast = lambda enabled=fp16: torch.autocast(device.type, dtype=torch.float16,
                                                            enabled=enabled, cache_enabled=cache)
        self.scaler = torch.amp.GradScaler(device.type, enabled=fp16)

    def _g_weights(self):
        return self._wn_g.active() if self._wn_g is not None else contextlib.nullcontext()

    def end_epoch(self):
        """The per-epoch lr decay of train_stft.py:138-139; reaches a captured
        step too (the lrs are device tensors there)."""
        self.scheduler_g.step()
        self.scheduler_d.step()

    def step(self, batch):
        if self.variant == "mel":
            return self._step_mel(batch)
        hps = self.hps
        rf = torch.profiler.record_function  # phase labels for torch.profiler tables
        x, x_lengths, spec, spec_lengths, y, y_lengths, emo, speakers = (
            t.to(self.device, non_blocking=True) for t in batch)
        with self.autocast():
            with rf("step:G.forward"), self._g_weights(), train_ops.prepacked(self.net_g):
                (y_hat, l_length, attn, ids_slice, x_mask, z_mask,
                 (z, z_p, m_p, logs_p, m_q, logs_q), z_q, (x_hidden, logw, logw_)) = self.net_g(
                    x, x_lengths, spec, spec_lengths, emo, speakers)
            if self.log_mels:  # train_stft.py:173-191 (logging mels, computed every step)
                with rf("step:log_mels"):
                    mel = spec_to_mel_torch(spec[:1].float(), hps.data.filter_length,
                                            hps.data.n_mel_channels, hps.data.sampling_rate,
                                            hps.data.mel_fmin, hps.data.mel_fmax)
                    _ = commons.slice_segments(mel, ids_slice[:1],
                                               hps.train.segment_size // hps.data.hop_length)
                    with torch.no_grad():
                        _ = mel_spectrogram_torch(y_hat[:1].squeeze(1).detach().float(),
                                                  hps.data.filter_length, hps.data.n_mel_channels,
                                                  hps.data.sampling_rate, hps.data.hop_length,
                                                  hps.data.win_length, hps.data.mel_fmin,
                                                  hps.data.mel_fmax)
            with rf("step:mrstft"):
                y = commons.slice_segments(y, ids_slice * hps.data.hop_length, hps.train.segment_size)
                sc_loss, mag_loss, y_mag, y_hat_mag = self.mstft(y.squeeze(1), y_hat.squeeze(1))
            with rf("step:D.forward(real,fake)"):
                if isinstance(self.net_d, MultiWaveSTFTDiscriminator):
                    # (one spectral-norm node for both passes; DDP keeps two calls)
                    y_d_hat_r, y_d_hat_g = self.net_d.forward_pair(
                        y, y_mag, y_hat.detach(), [m.detach() for m in y_hat_mag])
                else:
                    y_d_hat_r = self.net_d(y, y_mag)
                    y_d_hat_g = self.net_d(y_hat.detach(), [m.detach() for m in y_hat_mag])
                with self.autocast(False):
                    loss_disc, _, _ = discriminator_loss(y_d_hat_r, y_d_hat_g)
        with rf("step:D.backward"):
            self.optim_d.zero_grad()
            self.scaler.scale(loss_disc).backward()
            if self.allreduce:
                self._allreduce_grads("d", self.net_d)
        with rf("step:D.optimizer"):
            self.scaler.unscale_(self.optim_d)
            grad_norm_d = commons.clip_grad_value_(self.net_d.parameters(), None,
                                                   as_tensor=self.capturable)
            self.scaler.step(self.optim_d)

        # The generator loss backpropagates through D only for dL/dy_hat: D's
        # own weight gradients from this backward are discarded by the next
        # optim_d.zero_grad() (train_stft.py:202-232), so they are not computed
        # (identical updates, ~1/3 less D backward work).
        # Under DDP the D pass runs in no_sync() (no all-reduce of D grads that
        # nobody uses; the reference pays for it).
        d_params = [p for p in self.net_d.parameters() if p.requires_grad]
        for p in d_params:
            p.requires_grad_(False)
        d_ctx = self.net_d.no_sync() if isinstance(self.net_d, DDP) else contextlib.nullcontext()
        with self.autocast(), d_ctx:
            with rf("step:D.forward(gen)"):
                y_d_hat_g = self.net_d(y_hat, y_hat_mag)
            with rf("step:G.losses"), self.autocast(False):
                loss_dur = torch.sum(l_length.float()) * hps.train.c_dur
                loss_stft = (sc_loss.float() + mag_loss.float()) * hps.train.c_stft
                loss_kl = kl_loss(z_p, logs_q, m_p, logs_p, z_mask) * hps.train.c_kl
                loss_kl_q = kl_loss(z_q, logs_p, m_q, logs_q, z_mask) * hps.train.c_kl_q
                loss_gen, _ = generator_loss(y_d_hat_g)
                loss_gen_all = loss_gen + loss_stft + loss_dur + loss_kl + loss_kl_q
        with rf("step:G.backward"):
            self._backward_g(loss_gen_all)
        for p in d_params:
            p.requires_grad_(True)
        with rf("step:G.optimizer"):
            self.scaler.unscale_(self.optim_g)
            grad_norm_g = commons.clip_grad_value_(self.net_g.parameters(), None,
                                                   as_tensor=self.capturable)
            self.scaler.step(self.optim_g)
            self.scaler.update()
        return {"loss_disc": loss_disc.detach(), "loss_gen_all": loss_gen_all.detach(),
                "loss_gen": loss_gen.detach(), "loss_stft": loss_stft.detach(),
                "loss_dur": loss_dur.detach(), "loss_kl": loss_kl.detach(),
                "loss_kl_q": loss_kl_q.detach(), "sc_loss": sc_loss.detach(),
                "mag_loss": mag_loss.detach(), "grad_norm_g": grad_norm_g,
                "grad_norm_d": grad_norm_d}

    def _step_mel(self, batch):
        """One iteration of train.py's loop (train.py:171-233; the unused
        DurationDiscriminator branch, ``use_dur_dis``, is off in the
        reference and its class is not defined there)."""
        hps = self.hps
        rf = torch.profiler.record_function
        x, x_lengths, spec, spec_lengths, y, y_lengths, emo, speakers = (
            t.to(self.device, non_blocking=True) for t in batch)
        seg = hps.train.segment_size // hps.data.hop_length
        with self.autocast():
            with rf("step:G.forward"), self._g_weights(), train_ops.prepacked(self.net_g):
                (y_hat, l_length, attn, ids_slice, x_mask, z_mask,
                 (z, z_p, m_p, logs_p, m_q, logs_q), z_q, (x_hidden, logw, logw_)) = self.net_g(
                    x, x_lengths, spec, spec_lengths, emo, speakers)
            with rf("step:mel"):
                mel = spec_to_mel_torch(spec.float(), hps.data.filter_length,
                                        hps.data.n_mel_channels, hps.data.sampling_rate,
                                        hps.data.mel_fmin, hps.data.mel_fmax)
                y_mel = commons.slice_segments(mel, ids_slice, seg)
                y_hat_mel = mel_spectrogram_torch(y_hat.squeeze(1).float(), hps.data.filter_length,
                                                  hps.data.n_mel_channels, hps.data.sampling_rate,
                                                  hps.data.hop_length, hps.data.win_length,
                                                  hps.data.mel_fmin, hps.data.mel_fmax)
                y = commons.slice_segments(y, ids_slice * hps.data.hop_length, hps.train.segment_size)
            with rf("step:D.forward(real,fake)"):
                y_d_hat_r, y_d_hat_g, _, _ = self.net_d(y, y_hat.detach())
                with self.autocast(False):
                    loss_disc, _, _ = discriminator_loss(y_d_hat_r, y_d_hat_g)
        with rf("step:D.backward"):
            self.optim_d.zero_grad()
            self.scaler.scale(loss_disc).backward()
            if self.allreduce:
                self._allreduce_grads("d", self.net_d)
        with rf("step:D.optimizer"):
            self.scaler.unscale_(self.optim_d)
            grad_norm_d = commons.clip_grad_value_(self.net_d.parameters(), None,
                                                   as_tensor=self.capturable)
            self.scaler.step(self.optim_d)

        # as in step(): D's weight gradients of the generator pass are
        # discarded by the next optim_d.zero_grad(), so they are not computed;
        # the real branch then needs no autograd graph at all
        d_params = [p for p in self.net_d.parameters() if p.requires_grad]
        for p in d_params:
            p.requires_grad_(False)
        d_ctx = self.net_d.no_sync() if isinstance(self.net_d, DDP) else contextlib.nullcontext()
        with self.autocast(), d_ctx:
            with rf("step:D.forward(gen)"):
                y_d_hat_r, y_d_hat_g, fmap_r, fmap_g = self.net_d(y, y_hat)
            with rf("step:G.losses"), self.autocast(False):
                loss_dur = torch.sum(l_length.float()) * hps.train.c_dur
                loss_mel = torch.nn.functional.l1_loss(y_mel, y_hat_mel) * hps.train.c_mel
                loss_kl = kl_loss(z_p, logs_q, m_p, logs_p, z_mask) * hps.train.c_kl
                loss_kl_q = kl_loss(z_q, logs_p, m_q, logs_q, z_mask) * hps.train.c_kl_q
                loss_fm = feature_loss(fmap_r, fmap_g)
                loss_gen, _ = generator_loss(y_d_hat_g)
                loss_gen_all = loss_gen + loss_fm + loss_mel + loss_dur + loss_kl + loss_kl_q
        with rf("step:G.backward"):
            self._backward_g(loss_gen_all)
        for p in d_params:
            p.requires_grad_(True)
        with rf("step:G.optimizer"):
            self.scaler.unscale_(self.optim_g)
            grad_norm_g = commons.clip_grad_value_(self.net_g.parameters(), None,
                                                   as_tensor=self.capturable)
            self.scaler.step(self.optim_g)
            self.scaler.update()
        return {"loss_disc": loss_disc.detach(), "loss_gen_all": loss_gen_all.detach(),
                "loss_mel": loss_mel.detach(), "loss_fm": loss_fm.detach(),
                "loss_dur": loss_dur.detach(), "loss_kl": loss_kl.detach(),
                "grad_norm_g": grad_norm_g, "grad_norm_d": grad_norm_d}

    def _backward_g(self, loss_gen_all):
        """G's scaled backward; under allreduce its gradients are averaged
        over the ranks - bucket by bucket while the backward runs, or (flat
        mode) in one all-reduce afterwards."""
        self.optim_g.zero_grad()
        if self._gbuckets is not None:
            self._gbuckets.begin()
        self.scaler.scale(loss_gen_all).backward()
        if self._gbuckets is not None:
            self._gbuckets.finish()
        elif self.allreduce:
            self._allreduce_grads("g", self.net_g)

    def _allreduce_grads(self, key, net):
        """Average this network's gradients over the ranks: one flat buffer,
        one all-reduce (RCCL over xGMI on ROCm; capturable), copies in and
        out as multi-tensor launches.  Every rank has the same set of
        parameters with gradients (identical graphs), so the layout agrees."""
        ps = [p for p in net.parameters() if p.grad is not None]
        if not ps:
            return
        ent = self._flat.get(key)
        if ent is None or ent[0] != [id(p) for p in ps]:
            n = sum(p.numel() for p in ps)
            flat = torch.empty(n, device=ps[0].device, dtype=torch.float32)
            views, o = [], 0
            for p in ps:
                views.append(flat[o:o + p.numel()].view_as(p))
                o += p.numel()
            ent = ([id(p) for p in ps], flat, views)
            self._flat[key] = ent
        _, flat, views = ent
        grads = [p.grad for p in ps]
        torch._foreach_copy_(views, grads)
        dist.all_reduce(flat)
        flat.div_(dist.get_world_size())
        torch._foreach_copy_(grads, views)

    def capture(self, batch, warmup: int = 3):
        """Capture one whole step (both forwards, both backwards, both
        optimizer steps, the scaler update) into a hipGraph.  The batch is
        copied into static device buffers; replay(batch) refreshes them and
        replays.  Host-side randomness becomes device-side (rand_slice draw)
        and the alignment-noise decay runs inside the graph.  Multi-process
        runs capture with allreduce=True (the gradient all-reduce becomes a
        captured RCCL node); DDP's hooks are not capturable."""
        self._capture_warmup(batch, warmup)
        return self._capture_graph()

    def capture_agreed(self, batch, warmup: int = 3):
        """capture() for multi-process runs, with every rank agreeing on the
        outcome: the eager warm-up steps (they run real all-reduces) let an
        error propagate - torch.distributed.run then ends every rank - while
        a failure of the graph capture itself (no real collective runs while
        capturing) is caught, and one MIN all-reduce of a success flag makes
        every rank fall back to eager steps together.  A rank that replayed
        its graph while another stepped eagerly would pair their collectives
        wrongly and hang.  Returns None on success, else the error text
        (this rank's, or that another rank failed)."""
        self._capture_warmup(batch, warmup)
        err = None
        try:
            self._capture_graph()
        except Exception as e:  # noqa: BLE001 - reported, and agreed below
            err = f"{type(e).__name__}: {e}"[:300]
            self.graph = None
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
        if self.allreduce or (dist.is_available() and dist.is_initialized()):
            ok = torch.tensor([0 if err else 1], device=self.device, dtype=torch.int32)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            if int(ok.item()) == 0 and err is None:
                err = "graph capture failed on another rank"
                self.graph = None
        if err is not None:
            self._uncapture()
        return err

    def _uncapture(self):
        """Back to eager steps after a failed / abandoned capture: the host
        slice RNG and host-side alignment-noise decay of step()."""
        g_mod = self.net_g
        g_mod.__dict__.pop("_device_slice_rng", None)
        g_mod.__dict__.pop("_align_noise_t", None)
        self.graph = None

    def _capture_warmup(self, batch, warmup):
        assert self.capturable, "TrainStep(capturable=True) is required"
        assert not isinstance(self.net_g, DDP), \
            "DDP's hooks are not capturable: use TrainStep(allreduce=True) for multi-process capture"
        g_mod = self.net_g
        # this model's rand_slice_segments draws on the device from now on
        # (every replay re-draws); other models keep the host generator
        g_mod.__dict__["_device_slice_rng"] = True
        g_mod.__dict__["_align_noise_t"] = torch.tensor(float(g_mod.align_noise),
                                                        device=self.device)
        self.static = [t.to(self.device).clone() for t in batch]
        self._release_autograd_refs()
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            for _ in range(warmup):
                self.step(self.static)
        torch.cuda.current_stream(self.device).wait_stream(side)
        torch.cuda.synchronize(self.device)

    def _capture_graph(self):
        self._release_autograd_refs()
        self.graph = torch.cuda.CUDAGraph()
        self.optim_g.zero_grad(set_to_none=True)
        self.optim_d.zero_grad(set_to_none=True)
        # thread_local: the process-group watchdog thread keeps querying its
        # (pre-capture) events while this thread captures
        with torch.cuda.graph(self.graph, capture_error_mode="thread_local"):
            self.static_out = self.step(self.static)
        self._captured_lrs = self._lr_objects()
        return self.static_out

    def _lr_objects(self):
        return [g["lr"] for o in (self.optim_g, self.optim_d) for g in o.param_groups]

    def _check_lrs(self):
        """A captured step reads each group's lr tensor at replay time; a
        group whose lr was replaced by another object (e.g. a float assigned
        by hand) would silently keep the captured value - refuse that."""
        for old, new in zip(self._captured_lrs, self._lr_objects()):
            if new is not old:
                raise RuntimeError(
                    "TrainStep.replay: an optimizer's lr was replaced after capture(); update "
                    "the captured lr tensor in place (lr schedulers do) or capture again")

    def _release_autograd_refs(self):
        """Weight-norm / spectral-norm modules keep the last forward's
        computed ``weight`` (with its autograd graph) as an attribute, which
        keeps the parameters' AccumulateGrad nodes - and the stream they were
        created on - alive.  Eager steps on another stream before a capture
        would then make the captured backward accumulate on that stream.
        Drop those graphs (the hooks recompute ``weight`` every forward)."""
        for net in (self.net_g, self.net_d):
            for m in net.modules():
                for name in ("weight",):
                    if hasattr(m, name + "_g") or hasattr(m, name + "_orig"):
                        t = m.__dict__.get(name)
                        if isinstance(t, torch.Tensor) and t.grad_fn is not None:
                            m.__dict__[name] = t.detach()

    def replay(self, batch=None):
        if batch is not None:
            for dst, src in zip(self.static, batch):
                dst.copy_(src, non_blocking=True)
        self._check_lrs()
        self.graph.replay()
        g_mod = self.net_g
        g_mod.align_noise = max(g_mod.align_noise - g_mod.align_noise_decay, g_mod.align_noise_min)
        return self.static_out


def default_hps():
    """configs/base.json (the reference's shape source)."""
    return utils.get_hparams_from_dict({
        "train": {"log_interval": 1000, "eval_interval": 1000, "seed": 1234, "epochs": 500,
                  "steps": 3000, "learning_rate": 2e-4, "betas": [0.8, 0.99], "eps": 1e-9,
                  "batch_size": 32, "fp16_run": True, "lr_decay": 0.999875, "segment_size": 9216,
                  "weight_decay": 0.01, "c_mel": 45, "c_stft": 25, "c_dur": 2, "c_kl": 1.0,
                  "c_kl_q": 0.01, "align_noise": 1e-2, "align_noise_decay": 1e-6,
                  "align_noise_min": 1e-4},
        "data": {"max_text_len": 384, "max_wav_len": 192000, "text_channels": 256,
                 "sampling_rate": 16000, "filter_length": 1024, "hop_length": 192,
                 "win_length": 768, "n_mel_channels": 80, "mel_fmin": 0.0, "mel_fmax": None,
                 "n_speakers": 2048, "noise_scale": 0.707},
        "model": {"inter_channels": 192, "hidden_channels": 256, "filter_channels": 512,
                  "n_heads": 2, "n_layers": 6, "kernel_size": 5, "p_dropout": 0.1, "ffn": "FFN2",
                  "resblock": "2", "resblock_kernel_sizes": [3, 7, 11],
                  "resblock_dilation_sizes": [[1, 3, 5], [1, 3, 5], [1, 3, 5]],
                  "upsample_rates": [8, 6, 2, 2], "upsample_initial_channel": 512,
                  "upsample_kernel_sizes": [16, 12, 4, 4], "kernel_size_q": 5, "n_layers_q": 16,
                  "hidden_size_d": 256, "kernel_size_d": 5, "p_dropout_d": 0.5,
                  "act_func_d": "ReLU", "act_func_params_d": {}, "use_spectral_norm": False,
                  "dilation_rate": [1, 1, 1, 1], "n_flows": 4, "gin_channels": 1024}})


def synthetic_batch(hps, batch, tx=100, ty=500, seed=0, ragged=False):
    """One collated batch of SURVEY.md §8(d) C3 synthetic inputs."""
    from .data_utils import SyntheticTextAudioSpeaker, TextAudioSpeakerCollate

    ds = SyntheticTextAudioSpeaker(batch, tx=tx, ty=ty, text_channels=hps.data.text_channels,
                                   spec_channels=hps.data.filter_length // 2 + 1,
                                   hop=hps.data.hop_length, n_speakers=hps.data.n_speakers,
                                   seed=seed, ty_min=300 if ragged else None)
    return TextAudioSpeakerCollate()([ds[i] for i in range(batch)])


def main(argv=None):
    """Synthetic-data DDP training driver (torchrun: RANK/WORLD_SIZE/LOCAL_RANK)."""
    ap = argparse.ArgumentParser()
    ap.add_argument("-c", "--config", default=None)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--variant", choices=["stft", "mel"], default="stft",
                    help="stft: train_stft.py (MWSD + MR-STFT); mel: train.py (MPD + mel-L1)")
    args = ap.parse_args(argv)
    hps = utils.get_hparams_from_file(args.config) if args.config else default_hps()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    if world > 1:
        dist.init_process_group("nccl", init_method="env://", world_size=world, rank=rank)
    torch.manual_seed(hps.train.seed)
    net_g, net_d = build_models(hps, device, args.variant)
    stepper = TrainStep(hps, net_g, net_d, device, ddp=world > 1, variant=args.variant)
    bs = args.batch or hps.train.batch_size
    batch = synthetic_batch(hps, bs, seed=rank)
    for i in range(args.steps):
        t0 = time.perf_counter()
        out = stepper.step(batch)
        torch.cuda.synchronize()
        if rank == 0:
            print(f"step {i}: {time.perf_counter() - t0:.3f}s loss_g={float(out['loss_gen_all']):.4f} "
                  f"loss_d={float(out['loss_disc']):.4f}", flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
