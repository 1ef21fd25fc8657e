#!/usr/bin/env python3
"""Benchmark of the MI355X VITS hot path (BASELINE.json metric).

Workload (BASELINE.json configs[1]): ``SynthesizerTrn.infer_p2`` — prior
expansion + reverse flow + HiFi-GAN decoder — at batch 16, Tx=100 tokens,
5 frames/token -> Ty=500 frames -> 96,000 output samples per utterance
(configs/base.json: 16 kHz, hop 192), fp32, random-init weights
(deterministic key-hash fill), synthetic inputs.  One step = one infer_p2
call on one batch with every input already resident in HBM.

Multi-GPU: inference does not shard: N ranks run N
independent replicas of the same step; value = all output samples / the
slowest rank's time ("scaling": "weak").

Extra fields:
  roofline      the dominant kernel (conv1d_mfma_kernel + the fused ResBlock2
                pair kernel, every conv launch of the step): algorithmic FLOPs /
                HIP-event-timed kernel time,
                against the fp32 MFMA peak (157.3 TFLOP/s, MI355X_MICROARCH.md).
  cpu_baseline  the CPU oracle (oracle/vits_oracle.py, torch fp32 CPU: the
                reference algorithm restated) on a bounded sample.
  longform      BASELINE C5 (30 s utterances, B=4, bf16 model on the bf16-MFMA
                conv variant, hipGraph replay), with the fp32 time and the
                bf16-vs-fp32 waveform SNR beside it.
  kernels       the training-side HIP kernels at C3 shapes against their
                rooflines (MAS, neg_cent, MR-STFT magnitudes).
  train         the metric's second half (BASELINE configs 3/4): train utt/s of
                the train_stft step (vits_amd/train.py: G fwd/bwd, MWSD D,
                HIP MAS + MR-STFT, fp16 autocast, AdamW/RAdam) at
                --train-batch per GPU, Tx=100, Ty=500; under torchrun both
                networks are DDP-wrapped (RCCL gradient all-reduce), weak
                scaling, value = all ranks' utterances / slowest rank's time.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
       [--tx 100] [--ty 500] [--graph] [--no-cpu-baseline]
       [--train-batch 32] [--train-steps 5] [--train-warmup 2] [--no-train]
       [--no-longform]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "22.05 kHz audio samples/sec/GPU (infer RTF) + train utt/sec at 1/2/4/8 MI355X"
FP32_MFMA_PEAK_TFLOPS = 157.3
HOP = 192
SR = 16000

BASE_MODEL = dict(inter_channels=192, hidden_channels=256, filter_channels=512, n_heads=2,
                  n_layers=6, kernel_size=5, p_dropout=0.1, ffn="FFN2", resblock="2",
                  resblock_kernel_sizes=[3, 7, 11],
                  resblock_dilation_sizes=[[1, 3, 5], [1, 3, 5], [1, 3, 5]],
                  upsample_rates=[8, 6, 2, 2], upsample_initial_channel=512,
                  upsample_kernel_sizes=[16, 12, 4, 4], kernel_size_q=5, n_layers_q=16,
                  hidden_size_d=256, kernel_size_d=5, p_dropout_d=0.5, act_func_d="ReLU",
                  act_func_params_d={}, use_spectral_norm=False, dilation_rate=[1, 1, 1, 1],
                  n_flows=4, gin_channels=1024)


def build_model(device):
    from vits_amd.models import SynthesizerTrn
    from vits_amd.utils import deterministic_fill_

    m = SynthesizerTrn(256, 513, 48, n_speakers=2048, **BASE_MODEL).eval()
    deterministic_fill_(m)
    return m.to(device)


def make_inputs(B, Tx, Ty, device, seed=1234):
    from vits_amd.commons import infer_path

    g = torch.Generator().manual_seed(seed)
    per = Ty // Tx
    dur = torch.full((1, 1, Tx), float(per))
    dur[0, 0, -1] += Ty - per * Tx
    attn = infer_path(dur, Tx, Ty).expand(B, Ty, Tx).contiguous()
    m_p = torch.randn(B, 192, Tx, generator=g)
    s_p = torch.rand(B, 192, Tx, generator=g) + 0.3
    gg = torch.randn(B, 1024, generator=g) * 0.5
    noise = torch.randn(B, 192, Ty, generator=g) * 0.707
    return [t.to(device) for t in (attn, m_p, s_p, gg, noise)]


def cpu_baseline(model, Tx, Ty, budget_s=12.0):
    """Oracle (torch CPU fp32) infer_p2 on B=1 utterances until ~budget_s."""
    from oracle import vits_oracle as V

    sd = V.SD({k: v.detach().cpu() for k, v in model.state_dict().items()})
    attn, m_p, s_p, g, noise = make_inputs(1, Tx, Ty, "cpu")
    cores = torch.get_num_threads()
    with torch.no_grad():
        V.infer_p2(sd, attn, m_p, s_p, g, noise, BASE_MODEL)  # warm-up
        n, t0 = 0, time.perf_counter()
        while True:
            V.infer_p2(sd, attn, m_p, s_p, g, noise, BASE_MODEL)
            n += 1
            el = time.perf_counter() - t0
            if el >= budget_s or n >= 400:
                break
    samples = n * Ty * HOP
    out = {"value": samples / el, "unit": "output samples/s", "cores": cores, "kind": "port",
           "sample": f"{n} x infer_p2 B=1 Tx={Tx} Ty={Ty} ({Ty * HOP} samples each) in {el:.1f} s, "
                     f"oracle/vits_oracle.py torch-CPU fp32, torch.set_num_threads({cores})"}
    # the same at 8 threads (BASELINE.md's reference measurement: 8 vCPU);
    # one socket's cores exceed the box's CPU share (16 per GPU), so the
    # default thread count above is the largest figure measured
    if cores != 8:
        prev = torch.get_num_threads()
        torch.set_num_threads(8)
        try:
            with torch.no_grad():
                n8, t8 = 0, time.perf_counter()
                while True:
                    V.infer_p2(sd, attn, m_p, s_p, g, noise, BASE_MODEL)
                    n8 += 1
                    e8 = time.perf_counter() - t8
                    if e8 >= budget_s / 2 or n8 >= 200:
                        break
        finally:
            torch.set_num_threads(prev)
        out["by_threads"] = {str(cores): round(samples / el, 1), "8": round(n8 * Ty * HOP / e8, 1)}
    return out


def pmc_traffic():
    """HBM bytes per conv launch from the newest committed PMC summary
    (profiles/<tag>_summary.json, written by tools/summarize_profiles.py from
    separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes); None if absent."""
    import glob

    files = sorted(f for f in glob.glob(os.path.join(ROOT, "profiles", "*_summary.json"))
                   if not f.endswith(("_train_summary.json", "_longform_summary.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        d = json.load(f)
    c = d.get("conv_kernels", d.get("conv1d_mfma_kernel", {}))
    return c.get("hbm_bytes_per_launch"), os.path.relpath(files[-1], ROOT)


def _graph_rate(model, inputs, B, Ty, steps, warmup):
    with torch.no_grad():
        run = model.capture_infer_p2(B, inputs[0].shape[2], Ty)
        for _ in range(warmup):
            run(*inputs)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            out = run(*inputs)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
    return el, out.float().clone()


def longform_leg(model, device, rank, steps=5, warmup=2, B=4, Tx=500, Ty=2500):
    """BASELINE C5: 30 s utterances (B=4, Tx=500, Ty=2500 -> 480,000 samples
    each), bf16 model (bf16-MFMA convs, fp32 accumulation and activations),
    the whole infer_p2 replayed from one captured hipGraph.  The fp32 model
    is timed on the same inputs and its output is the SNR reference."""
    inputs = make_inputs(B, Tx, Ty, device, seed=4321 + rank)
    el32, ref = _graph_rate(model, inputs, B, Ty, steps, warmup)
    m16 = build_model(device).to(torch.bfloat16)  # same deterministic weights, bf16
    el16, out = _graph_rate(m16, inputs, B, Ty, steps, warmup)
    noise = float(((out - ref) ** 2).sum())
    snr = 10.0 * math.log10(float((ref ** 2).sum()) / max(noise, 1e-30))
    samples = steps * B * Ty * HOP
    # roofline: every conv launch of one eager bf16 step (HIP events per
    # launch) against the dense bf16 MFMA peak; traffic: PMC HBM bytes per
    # output frame of the replayed step (profiles/<tag>_longform_summary.json)
    from vits_amd.ops import ConvTimer

    with torch.no_grad(), ConvTimer() as timer:
        m16.infer_p2(*inputs)
    cs = timer.summary()
    conv_tf = (cs["total_flops"] / 1e12) / (cs["total_ms"] / 1e3)
    roof = {"bound": "mfma", "kernel": "every conv launch of the bf16 step",
            "achieved": round(conv_tf, 1), "peak": FP16_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(conv_tf / FP16_MFMA_PEAK_TFLOPS, 4),
            "conv_ms_per_step": round(cs["total_ms"], 3)}
    lf = _latest_summary("*_longform_summary.json")
    if lf:
        roof["traffic_bytes_per_frame"] = lf[0].get("hbm_bytes_per_frame")
        roof["traffic"] = lf[0].get("hbm_bytes_per_step")
        roof["traffic_source"] = lf[1]
        roof["fused_minimum_bytes_per_frame"] = 160_000  # fp32 stage in/out once
    del m16
    torch.cuda.empty_cache()
    return {"value": round(samples / el16, 1), "unit": "output samples/s", "roofline": roof,
            "ms_per_step": round(el16 / steps * 1e3, 3), "steps": steps, "warmup": warmup,
            "x_realtime_22k": round(samples / el16 / 22050.0, 1), "dtype": "bf16",
            "snr_db_vs_fp32": round(snr, 1),
            "fp32_ms_per_step": round(el32 / steps * 1e3, 3),
            "workload": f"infer_p2 batch={B} Tx={Tx} Ty={Ty} ({Ty * HOP / SR:.0f} s @16 kHz), "
                        "bf16 model, whole step replayed from one hipGraph"}


def _event_ms(fn, reps=20, warmup=3):
    for _ in range(warmup):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def _graph_ms(fn, reps=20, warmup=3):
    """Device time per call of ``fn``: ``reps`` calls captured into one
    hipGraph and replayed, timed with events on the replay stream, so host
    launch overhead (the Python wrapper: ~20-60 us per call) is excluded --
    these small kernels are shorter than their host-side call."""
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(warmup):
            fn()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for _ in range(reps):
            fn()
    graph.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    graph.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def latency_leg(model, device, reps=10):
    """Serving latency (EmoVITS / VITSWrap call pattern, one utterance):
    infer_p1 (text encoder + duration predictor) + infer_p2 (flow + decoder)
    at Tx=100, Ty=500 (96,000 samples = 6 s at 16 kHz), B=1, fp32."""
    g = torch.Generator().manual_seed(11)
    x = torch.randn(1, 100, 256, generator=g).to(device)
    emo = torch.randn(1, 1024, generator=g).to(device)
    sid = torch.tensor([1], device=device)
    attn, _, _, _, noise = make_inputs(1, 100, 500, device)

    def once():
        m_p, s_p, logw, gg = model.infer_p1(x, emo, sid)
        return model.infer_p2(attn, m_p, s_p, gg, noise)

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps * 1e3

    with torch.no_grad():
        ms = timed(once)
        p1 = model.capture_infer_p1(100)  # per-length graph (EmoVITS graph_cache > 0)

        def once_graph():
            m_p, s_p, logw, gg = p1(x, emo, sid)
            return model.infer_p2(attn, m_p, s_p, gg, noise)

        ms_g = timed(once_graph)
        # the whole utterance as ONE hipGraph (SynthesizerTrn.infer_bucketed:
        # durations / y_len / path on the device, flow + decoder masked at
        # y_len in a 512-frame bucket), incl. the y_len readback and the
        # waveform copy to the host that EmoVITS.infer returns
        whole = model.capture_infer_bucketed(100, 512)
        nz = torch.randn(1, 192, 512, device=device) * 0.707

        def once_whole():
            wav, yl = whole(x, emo, sid, nz)
            return wav[0, 0, :int(yl[0]) * HOP].cpu()

        ms_w = timed(once_whole)
    return {"ms": round(ms, 3), "ms_p1_graph": round(ms_g, 3), "ms_whole_graph": round(ms_w, 3),
            "audio_s": 6.0,
            "rtf_16k": round(ms / 6000.0, 6),
            "workload": "infer_p1 + infer_p2 (EmoVITS call pattern), B=1, Tx=100, Ty=500, fp32; "
                        "ms_whole_graph: the utterance with predicted durations as one replay"}


def kernels_leg(device):
    """The training-side HIP kernels at BASELINE C3 shapes (B=64, t_t=500
    frames, t_s=100 tokens, 9216-sample segments), each against its roofline
    (SURVEY §8(d)): MAS (latency-bound DP; HBM fraction reported), MR-STFT
    magnitudes (HBM), neg_cent (fp32 MFMA).  Device time per call from
    hipGraph replays (_graph_ms); the loss fwd+bwd is the eager host-side
    call."""
    from vits_amd import ops
    from vits_amd.stft_loss import MultiResolutionSTFTLoss

    g = torch.Generator(device="cpu").manual_seed(7)
    B, Tt, Ts, C, L = 64, 500, 100, 192, 9216
    nc = torch.randn(B, Tt, Ts, generator=g).to(device)
    tt = torch.full((B,), Tt, dtype=torch.int32, device=device)
    ts = torch.full((B,), Ts, dtype=torch.int32, device=device)
    mas_ms = _graph_ms(lambda: ops.maximum_path_lengths(nc, tt, ts))
    mas_bytes = B * Tt * Ts * 8
    mas_cpu = cpu_baseline_mas(nc, tt, ts)
    z = torch.randn(B, C, Tt, generator=g).to(device)
    m = torch.randn(B, C, Ts, generator=g).to(device)
    lg = (torch.randn(B, C, Ts, generator=g) * 0.5).to(device)
    nc_ms = _graph_ms(lambda: ops.neg_cent(z, m, lg))
    nc_flops = 2 * 2 * C * Tt * Ts * B
    loss = MultiResolutionSTFTLoss().to(device)
    y = (torch.randn(B, L, generator=g) * 0.1).to(device)
    yh = (torch.randn(B, L, generator=g) * 0.1).to(device).requires_grad_(True)
    specs = [(f.window, f.fft_size, f.hop_size, f.win_size, None, 1e-7) for f in loss.stft_losses]
    yd = yh.detach()
    # the loss's forward: both signals x 5 resolutions in one launch
    fwd_ms = _graph_ms(lambda: ops.stft_mag_multi([y] * 5 + [yd] * 5, specs + specs))
    mags = sum((f.fft_size // 2 + 1) * (L // f.hop_size + 1) for f in loss.stft_losses)
    fwd_bytes = 2 * B * (len(loss.stft_losses) * L * 4 + mags * 4)

    def fb():
        sc, mg, _, _ = loss(yh, y)
        (sc + mg).backward()

    fb_ms = _event_ms(fb, reps=10)
    peak = 8000.0
    return {
        "mas": {"ms": round(mas_ms, 4), "us_per_utt": round(mas_ms * 1e3 / B, 2),
                "shape": f"B={B} t_t={Tt} t_s={Ts}", "GBps": round(mas_bytes / mas_ms / 1e6, 1),
                "frac_hbm": round(mas_bytes / mas_ms / 1e6 / peak, 4),
                "bound": "latency (t_t sequential DP rows per utterance)",
                "cpu_baseline": mas_cpu,
                "vs_cpu": round(mas_cpu["ms"] / mas_ms, 1)},
        "neg_cent": {"ms": round(nc_ms, 4), "TFLOPs": round(nc_flops / nc_ms / 1e9, 2),
                     "arith": "split-f32 (three exact bf16 terms, six bf16 MFMAs per product)",
                     "frac": round(nc_flops / nc_ms / 1e9 / (FP16_MFMA_PEAK_TFLOPS / 6), 4),
                     "peak": round(FP16_MFMA_PEAK_TFLOPS / 6, 1),
                     "frac_fp32_mfma": round(nc_flops / nc_ms / 1e9 / FP32_MFMA_PEAK_TFLOPS, 4),
                     "shape": f"B={B} C={C} t_t={Tt} t_s={Ts}"},
        "mrstft_mag_fwd": {"ms": round(fwd_ms, 4), "GBps": round(fwd_bytes / fwd_ms / 1e6, 1),
                           "frac_hbm": round(fwd_bytes / fwd_ms / 1e6 / peak, 4),
                           "shape": f"B={B} L={L} x 5 resolutions x 2 signals, one launch"},
        "mrstft_loss_fwd_bwd_ms": round(fb_ms, 4),
    }


def cpu_baseline_mas(nc, tt, ts, reps=5):
    """CPU baseline of the MAS kernel (the C restatement
    with OpenMP over the batch): oracle/mas_oracle.c's
    mas_oracle_maximum_path_mt on the same [B, t_t, t_s] scores, the batch
    spread over min(16, cpu_count) host threads (the box's CPU share), median
    of `reps` calls including the float32 copy the DP works on."""
    from oracle import mas as mas_oracle

    a, b, c = nc.cpu().numpy(), tt.cpu().numpy(), ts.cpu().numpy()
    threads = min(16, os.cpu_count() or 1)
    mas_oracle.maximum_path_lengths_mt(a, b, c, threads)  # thread pool start-up
    times = []
    for _ in range(reps):
        t0 = time.perf_counter()
        mas_oracle.maximum_path_lengths_mt(a, b, c, threads)
        times.append(time.perf_counter() - t0)
    ms = sorted(times)[len(times) // 2] * 1e3
    return {"ms": round(ms, 3), "cores": threads, "kind": "port",
            "sample": f"the kernel's B={a.shape[0]} t_t={a.shape[1]} t_s={a.shape[2]} scores, "
                      f"median of {reps} calls"}


def train_cpu_baseline(budget_s=10.0, B=4, max_steps=50):
    """The same train_stft step on the host cores (BASELINE.md measured the
    reference at B=4 on 8 vCPU): vits_amd.train.TrainStep on CPU with the
    three HIP-only ops swapped for CPU restatements -- MAS from
    oracle/mas_oracle.c, neg_cent from oracle/vits_oracle.py, STFT magnitude
    from torch.stft -- i.e. the reference algorithm in PyTorch-CPU fp32."""
    import vits_amd.models as vm
    from vits_amd import ops
    from vits_amd.train import TrainStep, build_models, default_hps, synthetic_batch
    from oracle import mas as mas_oracle
    from oracle.vits_oracle import neg_cent as nc_oracle

    def cpu_mas(neg_cent, mask):
        p = mas_oracle.maximum_path(neg_cent.detach().float().numpy(), mask.detach().float().numpy())
        return torch.from_numpy(p).to(dtype=neg_cent.dtype)

    def cpu_nc(z, m, lg):
        return nc_oracle(z.detach().float(), m.detach().float(), lg.detach().float())

    def cpu_stft(x, window, n_fft, hop, win, pad=None, eps=1e-7):
        spec = torch.stft(x.float(), n_fft, hop, win, window, center=True, pad_mode="reflect",
                          return_complex=True)
        return torch.sqrt(spec.real ** 2 + spec.imag ** 2 + eps)

    saved = (vm.maximum_path, vm.neg_cent_scores, ops.stft_mag)
    vm.maximum_path, vm.neg_cent_scores, ops.stft_mag = cpu_mas, cpu_nc, cpu_stft
    try:
        hps = default_hps()
        torch.manual_seed(hps.train.seed)
        dev = torch.device("cpu")
        g, d = build_models(hps, dev)
        st = TrainStep(hps, g, d, dev, log_mels=False)
        batch = synthetic_batch(hps, B, seed=0)
        st.step(batch)  # warm-up
        t0 = time.perf_counter()
        steps = 0
        while steps < max_steps and (steps < 2 or time.perf_counter() - t0 < budget_s):
            st.step(batch)
            steps += 1
        el = time.perf_counter() - t0
    finally:
        vm.maximum_path, vm.neg_cent_scores, ops.stft_mag = saved
    return {"value": round(B * steps / el, 3), "unit": "utt/s", "cores": torch.get_num_threads(),
            "kind": "port",
            "sample": f"{steps} x train_stft step B={B} Tx=100 Ty=500 fp32 on CPU in {el:.1f} s "
                      "(vits_amd.train.TrainStep, MAS/neg_cent from oracle/, torch.stft)"}


TRAIN_GFLOP_PER_UTT = 365.4  # FlopCounterMode, train_stft step, Tx=100 Ty=500
FP16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X dense fp16 / bf16 MFMA (MI355X_MICROARCH.md)


def _latest_summary(pattern):
    """(dict, relpath) of the newest committed profiles/<pattern>, or None."""
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", pattern)))
    if not files:
        return None
    with open(files[-1]) as f:
        return json.load(f), os.path.relpath(files[-1], ROOT)


def train_traffic(batch=None):
    """HBM bytes per train step from the committed train PMC summaries
    (profiles/<tag>_train_summary.json, tools/summarize_train_profiles.py):
    the newest one measured at this batch, else the newest (scaled)."""
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_train_summary.json")))
    if not files:
        return None, None, None
    ds = []
    for fn in files:
        with open(fn) as f:
            ds.append((json.load(f), fn))
    same = [x for x in ds if x[0].get("batch") == batch]
    d, fn = (same or ds)[-1]
    return (d.get("hbm_bytes_per_step"), d.get("batch"), os.path.relpath(fn, ROOT))


def train_leg(args, device, rank, world, dist, B=None, cpu_base=True):
    """Timed train_stft steps (BASELINE C3/C4) on synthetic base.json batches."""
    from vits_amd.train import TrainStep, build_models, default_hps, synthetic_batch

    hps = default_hps()
    torch.manual_seed(hps.train.seed)
    # train_stft.py:26 sets cudnn.benchmark: MIOpen's exhaustive find for the
    # STFT discriminators' Conv2d layers (the step's only MIOpen convs) picks
    # faster solvers than its default find (69.2 -> 67.0 ms per B=32 step,
    # profiles/r06_cudnn_benchmark_ab.txt); the search runs in the warm-up
    torch.backends.cudnn.benchmark = True
    net_g, net_d = build_models(hps, device)
    # the whole step replayed from one hipGraph (TrainStep.capture); with
    # several ranks G's gradients are averaged in nine ordered RCCL buckets
    # on a side stream as each bucket completes, D's in one flat all-reduce,
    # all captured in the graph (allreduce=True; DDP's hooks are not
    # capturable, so the eager path keeps DDP)
    use_graph = not args.train_eager
    st = TrainStep(hps, net_g, net_d, device, ddp=world > 1 and not use_graph,
                   capturable=use_graph, allreduce=world > 1 and use_graph)
    B = B or args.train_batch
    batch = [t.to(device) for t in synthetic_batch(hps, B, tx=args.tx, ty=args.ty, seed=rank)]
    graph_err = None
    if use_graph:
        # a failed capture falls back to eager steps on EVERY rank together
        # (capture_agreed all-reduces the outcome; warm-up errors propagate)
        graph_err = st.capture_agreed(batch, warmup=max(1, args.train_warmup))
        use_graph = graph_err is None
    run = (lambda: st.replay()) if use_graph else (lambda: st.step(batch))
    for _ in range(args.train_warmup):
        run()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.train_steps):
        out = run()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    el = torch.tensor([time.perf_counter() - t0], device=device, dtype=torch.float64)
    if dist:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    el = float(el.item())
    utt = B * world * args.train_steps
    res = {"value": round(utt / el, 2), "unit": "utt/s", "per_gpu": round(utt / el / world, 2),
           "ms_per_step": round(el / args.train_steps * 1e3, 2), "steps": args.train_steps,
           "warmup": args.train_warmup, "global_batch": B * world, "dtype": "fp16 autocast",
           "scaling": "weak",
           "workload": f"train_stft step (G fwd/bwd + MWSD D x3 + MR-STFT + MAS) batch={B}/GPU "
                       f"Tx={args.tx} Ty={args.ty} segment 48 frames",
           "parallelism": (f"dp{world} (G: 9 overlapped RCCL buckets, D: one flat all-reduce)"
                            if st.allreduce else
                           f"ddp{world} (RCCL all-reduce)") if world > 1 else "single GPU",
           "graph": use_graph,
           "tflops_alg": round(TRAIN_GFLOP_PER_UTT * 1e9 * utt / el / 1e12, 2),
           "loss_gen_all": round(float(out["loss_gen_all"]), 4),
           "reference_cpu": "0.945 utt/s at B=4 on 8 vCPU (BASELINE.md, measured in the survey)"}
    # roofline of the whole step: algorithmic FLOPs (365.4 GFLOP per
    # utterance) per GPU-second against the dense fp16 MFMA peak; traffic =
    # PMC HBM bytes per step (FETCH x2 + WRITE over every kernel of one
    # replayed step, scaled to this batch) from the committed summary
    achieved = TRAIN_GFLOP_PER_UTT * 1e9 * B * args.train_steps / el / 1e12
    tb, tbatch, tsrc = train_traffic(B)
    res["roofline"] = {
        "bound": "mfma", "kernel": "whole train_stft step (every kernel of the replayed graph)",
        "achieved": round(achieved, 2), "peak": FP16_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
        "frac": round(achieved / FP16_MFMA_PEAK_TFLOPS, 4),
        "traffic": None if tb is None else int(tb * B / tbatch),
        "traffic_unit": ("HBM bytes per step (PMC at this batch)" if tbatch == B else
                         "HBM bytes per step (PMC, scaled from batch %s)" % tbatch),
        "traffic_source": tsrc}
    if graph_err:
        res["graph_error"] = graph_err
    if rank == 0 and world == 1 and not args.no_cpu_baseline and cpu_base:
        res["cpu_baseline"] = train_cpu_baseline()
    del st, net_g, net_d
    torch.cuda.empty_cache()
    return res


def conv_kernel_table(timer, steps):
    """Per-shape rows of the headline step's conv launches (the "kernel,
    TF/s, fraction of ceiling" table): launches grouped by descriptor label
    (rows m, input channels c, taps k, dilation d, output length T, epilogue
    e, tile t), each against the MFMA peak of its arithmetic (exact f32
    157.3, split f32 416.7, bf16 2500 TF/s).  Sorted by time per step."""
    from vits_amd.ops import MFMA_PEAK_TFLOPS, WDT_F32S

    rows = {}
    torch.cuda.synchronize()
    for lab, (s, e, fl), pk in zip(timer.shapes, timer.records, timer.peaks):
        r = rows.setdefault(lab, [0, 0.0, 0, pk])
        r[0] += 1
        r[1] += s.elapsed_time(e)
        r[2] += fl
    out = []
    for lab, (n, ms, fl, pk) in sorted(rows.items(), key=lambda kv: -kv[1][1]):
        tf = fl / (ms * 1e9)
        kind = ("split-f32" if pk == MFMA_PEAK_TFLOPS[WDT_F32S] else
                "exact-f32" if pk < 200 else "16-bit")
        out.append({"kernel": lab, "arith": kind, "launches_per_step": round(n / steps, 2),
                    "ms_per_step": round(ms / steps, 4), "achieved": round(tf, 1),
                    "unit": "TFLOP/s", "peak": round(pk, 1), "frac": round(tf / pk, 3)})
    return out


def fp32_arith() -> str:
    from vits_amd import engine

    if engine.FP32_MODE == "exact":
        return "exact: v_mfma_f32_32x32x2_f32 (bitwise an fp32 fma chain)"
    from vits_amd import ops

    return (f"split: convs with >= {ops._f32s_min_rows()} GEMM rows, and every fused ResBlock2 "
            "pair (the 32-channel stage included), split each fp32 operand exactly into three "
            "bf16 terms (weights pre-split into planes), six bf16 MFMAs per product, fp32 "
            "accumulation (error vs fp64 at or below the exact-f32 kernel's, "
            "tests/test_kernels_gpu.py): every conv / pair launch of the headline step; conv_post "
            "+ tanh (1 output row) is its own fp32 FMA kernel")


def _launch_ranks(args) -> int:
    """``--gpus N`` (N > 1) without a torchrun environment: start N ranks as
    ``python -m torch.distributed.run`` in a CHILD process - this process
    never touches the GPU - and exit with its status.  Rank 0 prints the
    JSON line (its stdout is passed through)."""
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=env)


def dry_run_line(args, world, rank, dist):
    """--dry-run: the launcher / rank / aggregation logic without a GPU
    (gloo, a small CPU matmul as the "step"); same fields as the real line."""
    x = torch.randn(256, 256)
    for _ in range(args.warmup):
        x @ x
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        x @ x
    if dist:
        dist.barrier()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())
    B, Ty = args.batch, args.ty
    return {"metric": METRIC, "value": round(args.steps * B * Ty * HOP * world / el, 1),
            "unit": "output samples/s", "n_gpus": world, "rank_seen": rank, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
            "data": "dry run (CPU, no GPU work)",
            "config": {"workload": "dry run", "global_batch": B * world, "seq_len": Ty,
                       "parallelism": f"replicas x{world}" if world > 1 else "single GPU"}}


def _guarded(name, fn, *a, **k):
    """fn(*a, **k), or {"error": ...} when it raises (reported in the line)."""
    try:
        return fn(*a, **k)
    except Exception as e:  # noqa: BLE001
        import traceback

        traceback.print_exc()
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        return {"error": f"{name}: {type(e).__name__}: {e}"[:400]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--tx", type=int, default=100)
    ap.add_argument("--ty", type=int, default=500)
    ap.add_argument("--graph", action="store_true", help="replay a captured hipGraph per step")
    ap.add_argument("--fp32-mode", choices=("split", "exact"), default=None,
                    help="fp32 conv arithmetic (vits_amd.engine.FP32_MODE; default split)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--train-batch", type=int, default=32, help="C4: utterances per GPU")
    ap.add_argument("--train-batch-c3", type=int, default=64,
                    help="C3: the one-GPU train_stft batch (0: skip)")
    ap.add_argument("--train-steps", type=int, default=5)
    ap.add_argument("--train-warmup", type=int, default=2)
    ap.add_argument("--no-train", action="store_true")
    ap.add_argument("--train-eager", action="store_true",
                    help="time the eager train step instead of the captured hipGraph")
    ap.add_argument("--no-longform", action="store_true")
    ap.add_argument("--no-kernels", action="store_true")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU-only check of the rank launcher / aggregation (gloo, no GPU work)")
    args = ap.parse_args()
    if args.fp32_mode:  # read by vits_amd.engine at import
        os.environ["VITS_FP32_MODE"] = args.fp32_mode
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # not under torchrun: start the N ranks ourselves (before any GPU use)
        sys.exit(_launch_ranks(args))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; measuring {world} ranks",
              file=sys.stderr)
    dist = None
    if world > 1:
        import torch.distributed as dist

        if not args.dry_run:
            torch.cuda.set_device(local_rank)
        dist.init_process_group("gloo" if args.dry_run else "nccl", init_method="env://",
                                world_size=world, rank=rank)
    if args.dry_run:
        line = dry_run_line(args, world, rank, dist)
        if rank == 0:
            print(json.dumps(line), flush=True)
        if dist:
            dist.destroy_process_group()
        return
    device = torch.device("cuda", local_rank)

    # the train legs run first, on a clean allocator (its MIOpen algorithm
    # choice depends on free workspace), and release their memory afterwards:
    # C4 = --train-batch per GPU (32, weak scaling over the ranks), and at
    # one rank also C3 = the train_stft step at batch 64 on one GPU
    train = train_c3 = None
    if not args.no_train:
        # a leg that raises (a VitsAmdError shape / support check, deterministic
        # on every rank) is reported in the line instead of losing the whole
        # line; a GPU fault still ends the process
        train = _guarded("train", train_leg, args, device, rank, world, dist, args.train_batch)
        if world == 1 and args.train_batch_c3 and args.train_batch_c3 != args.train_batch:
            train_c3 = _guarded("train_c3", train_leg, args, device, rank, world, dist,
                                args.train_batch_c3, cpu_base=False)

    model = build_model(device)
    B, Tx, Ty = args.batch, args.tx, args.ty
    inputs = make_inputs(B, Tx, Ty, device, seed=1234 + rank)

    step = None
    if args.graph:
        run = model.capture_infer_p2(B, Tx, Ty)
        step = lambda: run(*inputs)  # noqa: E731
    else:
        step = lambda: model.infer_p2(*inputs)  # noqa: E731

    with torch.no_grad():
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            out = step()
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0

        roof = None
        kernel_table = []
        if not args.no_roofline and not args.graph:
            from vits_amd.ops import ConvTimer

            with ConvTimer() as timer:
                for _ in range(args.steps):
                    model.infer_p2(*inputs)
            s = timer.summary()
            per_launch_flops = s["total_flops"] / max(1, s["launches"])
            achieved = (s["total_flops"] / 1e12) / (s["total_ms"] / 1e3)
            # launches run exact fp32 (f32 MFMA, 157.3 TF/s) or split fp32
            # (six bf16 MFMAs per product, 2.5 PF/s / 6): the peak is the
            # rate of the MFMA-bound minimum time of the same launches
            peak = (s["total_flops"] / 1e12) / (s["mfma_bound_ms"] / 1e3)
            traffic, tsrc = pmc_traffic()
            kernel_table = conv_kernel_table(timer, args.steps)
            roof = {"bound": "mfma",
                    "kernel": "conv1d_mfma_kernel + resblock_f32p_kernel (every conv / fused "
                              "ResBlock2-pair launch of a step)",
                    "achieved": round(achieved, 2), "peak": round(peak, 1),
                    "unit": "TFLOP/s", "frac": round(achieved / peak, 4),
                    "peak_basis": "time-weighted: exact-fp32 launches at the f32 MFMA peak "
                                  f"{FP32_MFMA_PEAK_TFLOPS}, split-fp32 launches "
                                  f"({100 * s['f32s_flops'] / s['total_flops']:.0f} % of the "
                                  "FLOPs) at the bf16 dense peak / 6 = 416.7",
                    "frac_vs_f32_mfma_peak": round(achieved / FP32_MFMA_PEAK_TFLOPS, 4),
                    "traffic": traffic, "traffic_unit": "HBM bytes per launch (PMC)",
                    "traffic_source": tsrc, "launches_per_step": s["launches"] // args.steps,
                    "avg_launch_ms": round(s["avg_ms"], 4),
                    "flops_per_launch": int(per_launch_flops),
                    "conv_ms_per_step": round(s["total_ms"] / args.steps, 3)}

    longform = None if args.no_longform else _guarded("longform", longform_leg, model, device,
                                                      rank)
    kern = None if args.no_kernels else _guarded("kernels", kernels_leg, device)
    if kern:
        for name, k in kern.items():
            if not isinstance(k, dict):
                continue
            if "TFLOPs" in k:
                kernel_table.append({"kernel": name, "shape": k["shape"], "ms": k["ms"],
                                     "achieved": k["TFLOPs"], "unit": "TFLOP/s",
                                     "peak": FP32_MFMA_PEAK_TFLOPS, "frac": k["frac_fp32_mfma"]})
            elif "GBps" in k:
                kernel_table.append({"kernel": name, "shape": k["shape"], "ms": k["ms"],
                                     "achieved": k["GBps"], "unit": "GB/s", "peak": 8000.0,
                                     "frac": k["frac_hbm"], "bound": k.get("bound", "hbm")})
    latency = None if args.no_kernels else latency_leg(model, device)

    t = torch.tensor([elapsed], device=device, dtype=torch.float64)
    if dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    samples_per_rank = args.steps * B * Ty * HOP
    total_samples = samples_per_rank * world
    value = total_samples / elapsed
    ms_per_step = elapsed / args.steps * 1e3

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "output samples/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "fp32",
            "fp32_arith": fp32_arith(),
            "data": "synthetic: random-init weights (deterministic key-hash fill), random priors, "
                    "5 frames/token durations",
            "config": {"workload": f"SynthesizerTrn.infer_p2 batch={B} Tx={Tx} Ty={Ty} "
                                   f"(configs/base.json, 16 kHz, hop 192) per GPU",
                       "global_batch": B * world, "seq_len": Ty,
                       "parallelism": f"replicas x{world}" if world > 1 else "single GPU",
                       "graph": bool(args.graph)},
            "rtf_16k": round((ms_per_step / 1e3) / (B * Ty * HOP / SR), 6),
            "x_realtime_22k": round(value / world / 22050.0, 1),
            "roofline": roof,
        }
        if not args.no_cpu_baseline and world == 1:
            line["cpu_baseline"] = cpu_baseline(model, Tx, Ty)
        else:
            line["cpu_baseline"] = None
        # the per-shape kernel table (long) goes on a line of its own before
        # the result line; the result line ends with the legs of the metric's
        # second half so a tail of stdout shows them
        print("kernel_table " + json.dumps(kernel_table), flush=True)
        line.update({"kernels": kern, "latency_b1": latency, "longform": longform,
                     "train_c3": train_c3, "train": train})
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
