"""Training side (train_stft.py step, DDP, sampler, collate, discriminators).

CPU tests run the full TrainStep on the tiny config with the two HIP-only
ops swapped for CPU checkers (MAS -> oracle/mas, STFT magnitude -> torch.stft),
including a world_size-2 ``gloo`` DDP run that checks gradient averaging
keeps the replicas identical.  The GPU test runs the same step on the HIP
path (fp16 autocast + GradScaler, as configs/base.json fp16_run=true).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from common import tiny_cfg

SEG_FRAMES = 16  # 3072 samples: long enough for the 2048-point MR-STFT resolution


def tiny_hps():
    from vits_amd.utils import get_hparams_from_dict

    c = tiny_cfg()
    return get_hparams_from_dict({
        "train": {"seed": 1234, "learning_rate": 2e-4, "betas": [0.8, 0.99], "eps": 1e-9,
                  "fp16_run": True, "segment_size": SEG_FRAMES * 192, "weight_decay": 0.01,
                  "c_stft": 25, "c_dur": 2, "c_kl": 1.0, "c_kl_q": 0.01, "align_noise": 1e-2,
                  "align_noise_decay": 1e-6, "align_noise_min": 1e-4, "lr_decay": 0.999875},
        "data": {"text_channels": c["data"]["text_channels"], "sampling_rate": 16000,
                 "filter_length": (c["data"]["spec_channels"] - 1) * 2, "hop_length": 192,
                 "win_length": 64, "n_mel_channels": 16, "mel_fmin": 0.0, "mel_fmax": None,
                 "n_speakers": c["data"]["n_speakers"]},
        "model": c["model"]})


def _cpu_stft_mag(x, window, n_fft, hop, win, pad=None, eps=1e-7):
    spec = torch.stft(x.float(), n_fft, hop, win, window.to(x.device), center=True,
                      pad_mode="reflect", return_complex=True)
    return torch.sqrt(spec.real ** 2 + spec.imag ** 2 + eps)


def _cpu_mas(neg_cent, mask):
    from oracle import mas as mas_oracle

    p = mas_oracle.maximum_path(neg_cent.detach().cpu().float().numpy(),
                                mask.detach().cpu().float().numpy())
    return torch.from_numpy(p).to(device=neg_cent.device, dtype=neg_cent.dtype)


def _cpu_neg_cent(z_p, m_p, logs_p):
    from oracle.vits_oracle import neg_cent

    return neg_cent(z_p.detach().float(), m_p.detach().float(), logs_p.detach().float())


def _patch_cpu():
    import vits_amd.models as vm
    import vits_amd.ops as ops

    vm.maximum_path = _cpu_mas
    vm.neg_cent_scores = _cpu_neg_cent
    ops.stft_mag = _cpu_stft_mag


def tiny_mel_hps():
    """tiny_hps for train.py's variant: the mel-L1 loss needs hop <= n_fft,
    so the spectrogram is 512-point (257 channels) with the reference's
    hop 192; c_mel 45 as configs/base.json."""
    hps = tiny_hps()
    hps.data.filter_length = 512
    hps.data.win_length = 512
    hps.train.c_mel = 45
    return hps


def _make(hps, device, ddp=False, seed=0, capturable=False, allreduce=False, variant="stft"):
    from vits_amd.train import TrainStep, build_models

    torch.manual_seed(seed)
    net_g, net_d = build_models(hps, device, variant)
    # the logging mels need hop <= n_fft; the tiny config (n_fft 64, hop 192)
    # skips them, the base-config train bench (tools/train_bench.py) runs them
    return TrainStep(hps, net_g, net_d, device, ddp=ddp, log_mels=False, capturable=capturable,
                     allreduce=allreduce, variant=variant)


def _batch(hps, n, seed):
    from vits_amd.train import synthetic_batch

    return synthetic_batch(hps, n, tx=10, ty=40, seed=seed, ragged=False)


def test_discriminator_shapes():
    from vits_amd.discriminators import MultiWaveSTFTDiscriminator

    d = MultiWaveSTFTDiscriminator()
    sd = d.state_dict()
    assert any(k.endswith("weight_orig") for k in sd)  # spectral norm keys (mrd.py)
    y = torch.randn(2, 1, 3072)
    mags = [_cpu_stft_mag(y.squeeze(1), torch.hann_window(f), f, f // 4, f)
            for f in (128, 256, 512, 1024, 2048)]
    outs = d(y, mags)
    assert len(outs) == 10
    for o in outs[:5]:  # wave branch: [B, T']
        assert o.dim() == 2 and o.size(0) == 2 and torch.isfinite(o).all()
    for o in outs[5:]:  # STFT branch keeps the reference's [B, 1, T'] (mrd.py:156)
        assert o.shape[:2] == (2, 1) and torch.isfinite(o).all()


def test_bucket_sampler_shards_disjoint_and_padded():
    from vits_amd.data_utils import DistributedBucketSampler

    class DS:
        lengths = [100 + 37 * i % 900 for i in range(50)]

        def __len__(self):
            return len(self.lengths)

    ds = DS()
    bounds = [32, 300, 400, 500, 600, 700, 800, 900, 1000]
    per_rank = []
    for r in range(2):
        s = DistributedBucketSampler(ds, 4, bounds, num_replicas=2, rank=r, shuffle=True)
        s.set_epoch(3)
        batches = list(iter(s))
        assert len(batches) == len(s)
        for b in batches:
            assert len(b) == 4
            # a batch never straddles a bucket boundary
            bk = {next(i for i in range(len(s.boundaries) - 1)
                       if s.boundaries[i] < ds.lengths[j] <= s.boundaries[i + 1]) for j in b}
            assert len(bk) == 1
        per_rank.append(sorted(j for b in batches for j in b))
    allids = per_rank[0] + per_rank[1]
    assert set(allids) == set(range(50))  # every utterance is seen (padding repeats some)
    # determinism per epoch
    s = DistributedBucketSampler(ds, 4, bounds, num_replicas=2, rank=0)
    s.set_epoch(3)
    assert sorted(j for b in s for j in b) == per_rank[0]


def test_collate_sorts_by_spec_length():
    from vits_amd.data_utils import SyntheticTextAudioSpeaker, TextAudioSpeakerCollate

    ds = SyntheticTextAudioSpeaker(5, tx=8, ty=30, text_channels=16, spec_channels=33, seed=1,
                                   ty_min=10)
    text, tl, spec, sl, wav, wl, emo, sid, order = TextAudioSpeakerCollate(True)([ds[i] for i in range(5)])
    assert (sl[:-1] >= sl[1:]).all()
    assert torch.equal(wl, sl * 192)
    for i, k in enumerate(order.tolist()):
        t, s, w, e, spk = ds[k]
        assert torch.equal(spec[i, :, :s.size(1)], s) and spec[i, :, s.size(1):].abs().sum() == 0
        assert torch.equal(text[i, :t.size(0)], t) and int(sid[i]) == spk


def test_train_step_cpu_reduces_loss_and_updates(monkeypatch):
    import vits_amd.models as vm
    import vits_amd.ops as ops

    monkeypatch.setattr(vm, "maximum_path", _cpu_mas)
    monkeypatch.setattr(vm, "neg_cent_scores", _cpu_neg_cent)
    monkeypatch.setattr(ops, "stft_mag", _cpu_stft_mag)
    hps = tiny_hps()
    st = _make(hps, torch.device("cpu"))
    batch = _batch(hps, 2, seed=0)
    before = {n: p.detach().clone() for n, p in st.net_g.named_parameters()}
    out = st.step(batch)
    for k in ("loss_disc", "loss_gen_all", "loss_stft", "loss_dur", "loss_kl"):
        assert torch.isfinite(out[k]), k
    assert out["grad_norm_g"] > 0 and out["grad_norm_d"] > 0
    changed = sum(not torch.equal(before[n], p) for n, p in st.net_g.named_parameters())
    assert changed > 50


def test_train_step_mel_variant_cpu(monkeypatch):
    """train.py's loop (MultiPeriodDiscriminator, mel-L1, feature matching,
    AdamW for D) on CPU: finite losses, both networks updated."""
    import vits_amd.models as vm
    import vits_amd.ops as ops
    from vits_amd.models import MultiPeriodDiscriminator

    monkeypatch.setattr(vm, "maximum_path", _cpu_mas)
    monkeypatch.setattr(vm, "neg_cent_scores", _cpu_neg_cent)
    monkeypatch.setattr(ops, "stft_mag", _cpu_mel_stft_mag)
    hps = tiny_mel_hps()
    st = _make(hps, torch.device("cpu"), variant="mel")
    assert isinstance(st.net_d, MultiPeriodDiscriminator)
    assert isinstance(st.optim_d, torch.optim.AdamW)
    batch = _batch(hps, 2, seed=0)
    g0 = {n: p.detach().clone() for n, p in st.net_g.named_parameters()}
    d0 = {n: p.detach().clone() for n, p in st.net_d.named_parameters()}
    out = st.step(batch)
    for k in ("loss_disc", "loss_gen_all", "loss_mel", "loss_fm", "loss_dur", "loss_kl"):
        assert torch.isfinite(out[k]), k
    assert out["loss_mel"] > 0 and out["loss_fm"] > 0
    assert sum(not torch.equal(g0[n], p) for n, p in st.net_g.named_parameters()) > 50
    assert sum(not torch.equal(d0[n], p) for n, p in st.net_d.named_parameters()) > 20


def _cpu_mel_stft_mag(x, window, n_fft, hop, win, pad=None, eps=1e-7):
    """stft_mag with the explicit reflect pad + center=False of
    mel_processing.spectrogram_torch (torch.stft on CPU)."""
    if pad is None:
        return _cpu_stft_mag(x, window, n_fft, hop, win, eps=eps)
    xp = torch.nn.functional.pad(x.float().unsqueeze(1), (pad, pad), mode="reflect").squeeze(1)
    spec = torch.stft(xp, n_fft, hop, win, window.to(x.device), center=False,
                      return_complex=True)
    return torch.sqrt(spec.real ** 2 + spec.imag ** 2 + eps)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _ddp_worker(rank, world, port, out_dir, mode="ddp"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    _patch_cpu()
    hps = tiny_hps()
    # different init per rank: the allreduce mode must broadcast rank 0's
    st = _make(hps, torch.device("cpu"), ddp=mode == "ddp", seed=0 if mode == "ddp" else rank,
               allreduce={"allreduce": True, "flat": "flat"}.get(mode, False))
    if mode == "allreduce":  # G's gradients go through the overlapped buckets
        assert st._gbuckets is not None and len(st._gbuckets.buckets) >= 3
    for i in range(2):
        out = st.step(_batch(hps, 2, seed=10 * i + rank))  # different data per rank
    flat = torch.cat([p.detach().flatten() for p in st.net_g.parameters()] +
                     [p.detach().flatten() for p in st.net_d.parameters()])
    np.save(os.path.join(out_dir, f"rank{rank}.npy"), flat.numpy())
    np.save(os.path.join(out_dir, f"loss{rank}.npy"), np.array([float(out["loss_gen_all"])]))
    dist.destroy_process_group()


def _capture_fail_worker(rank, world, port, out_dir):
    """TrainStep.capture_agreed with the graph capture failing on rank 1
    only: both ranks must report the failure and fall back to eager steps
    together (the collectives of the eager steps then pair up: no hang)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    _patch_cpu()
    hps = tiny_hps()
    st = _make(hps, torch.device("cpu"), seed=rank, allreduce=True)
    batch = _batch(hps, 2, seed=rank)

    def warmup(b, n):  # the eager warm-up steps of _capture_warmup
        for _ in range(n):
            st.step(b)

    def graph():
        if rank == 1:
            raise RuntimeError("forced capture failure")
        st.graph = "captured"

    st._capture_warmup, st._capture_graph = warmup, graph
    err = st.capture_agreed(batch, warmup=1)
    out = st.step(batch)  # eager on both ranks
    flat = torch.cat([p.detach().flatten() for p in st.net_g.parameters()])
    np.save(os.path.join(out_dir, f"rank{rank}.npy"), flat.numpy())
    with open(os.path.join(out_dir, f"err{rank}.txt"), "w") as f:
        f.write(f"{err}|{st.graph}|{float(out['loss_gen_all'])}")
    dist.destroy_process_group()


def test_capture_failure_on_one_rank_falls_back_on_all_ranks(tmp_path):
    port = _free_port()
    mp.spawn(_capture_fail_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    e0 = (tmp_path / "err0.txt").read_text().split("|")
    e1 = (tmp_path / "err1.txt").read_text().split("|")
    assert e0[0] == "graph capture failed on another rank" and e0[1] == "None"
    assert e1[0].startswith("RuntimeError: forced capture failure") and e1[1] == "None"
    assert np.array_equal(np.load(tmp_path / "rank0.npy"), np.load(tmp_path / "rank1.npy"))


@pytest.mark.parametrize("mode", ["ddp", "allreduce", "flat"])
def test_ddp_gloo_world2_replicas_stay_identical(tmp_path, mode):
    """Every multi-process mode (DDP; the graph-capturable all-reduce with
    G's gradients in overlapped buckets; the same with one flat all-reduce)
    keeps the replicas bit-identical while each rank sees different data."""
    port = _free_port()
    mp.spawn(_ddp_worker, args=(2, port, str(tmp_path), mode), nprocs=2, join=True)
    a = np.load(tmp_path / "rank0.npy")
    b = np.load(tmp_path / "rank1.npy")
    assert np.array_equal(a, b)  # gradient all-reduce -> identical updates
    la, lb = np.load(tmp_path / "loss0.npy"), np.load(tmp_path / "loss1.npy")
    assert np.isfinite(la).all() and np.isfinite(lb).all() and la[0] != lb[0]


def test_bucketed_allreduce_equals_flat_allreduce(tmp_path):
    """The overlapped bucketed G all-reduce averages exactly what the flat
    one does: two steps of each mode from the same seeds and data end in
    bit-identical parameters."""
    res = {}
    for mode in ("allreduce", "flat"):
        d = tmp_path / mode
        d.mkdir()
        mp.spawn(_ddp_worker, args=(2, _free_port(), str(d), mode), nprocs=2, join=True)
        res[mode] = np.load(d / "rank0.npy")
    assert np.array_equal(res["allreduce"], res["flat"])


class _RecordingDist:
    """Stand-in for torch.distributed in _GradBuckets' CPU path: records the
    size of every all-reduced flat buffer (world size 1)."""

    def __init__(self):
        self.calls = []

    def all_reduce(self, t):
        self.calls.append(t.numel())

    def get_world_size(self):
        return 1


def test_grad_buckets_launch_in_index_order(monkeypatch):
    """Buckets whose gradients complete out of order are all-reduced in
    bucket-index order (collectives pair up across ranks), and a parameter
    without a gradient is zero-filled so every rank's bucket layout agrees."""
    from vits_amd import train as T

    rec = _RecordingDist()
    monkeypatch.setattr(T, "dist", rec)
    net = torch.nn.Module()
    net.a = torch.nn.Linear(3, 2)        # bucket 0: 8 elements
    net.b = torch.nn.Linear(4, 4)        # bucket 1: 20 elements
    net.c = torch.nn.Linear(1, 1, bias=False)  # bucket 2: 1 element, never gets a gradient
    gb = T._GradBuckets(net, (("a.",), ("b.",), ("",)), torch.device("cpu"))
    assert [sum(p.numel() for p in b) for b in gb.buckets] == [8, 20, 1]
    gb.begin()
    net.b(torch.randn(2, 4)).sum().backward()  # bucket 1 completes first
    assert rec.calls == []                     # ... but waits for bucket 0
    net.a(torch.randn(2, 3)).sum().backward()
    assert rec.calls == [8, 20]
    gb.finish()                                # bucket 2: no gradient -> zeros
    assert rec.calls == [8, 20, 1]
    assert torch.equal(net.c.weight.grad, torch.zeros_like(net.c.weight))


def test_g_buckets_cover_every_parameter_within_50mb():
    """G_BUCKETS at configs/base.json: every G parameter in exactly one
    bucket (the first matching), each bucket <= 50 MB of fp32 gradients."""
    from vits_amd.train import G_BUCKETS, _bucket_of, build_models, default_hps

    net_g, _ = build_models(default_hps(), torch.device("cpu"))
    sizes = [0] * len(G_BUCKETS)
    for n, p in net_g.named_parameters():
        sizes[_bucket_of(n, G_BUCKETS)] += 4 * p.numel()
    assert all(0 < s <= 50e6 for s in sizes), sizes
    assert sum(sizes) == 4 * sum(p.numel() for p in net_g.parameters())


@pytest.mark.gpu
def test_train_step_gpu_fp16(device):
    hps = tiny_hps()
    st = _make(hps, device)
    batch = _batch(hps, 4, seed=0)
    outs = [st.step(batch) for _ in range(3)]
    torch.cuda.synchronize()
    for out in outs:
        assert torch.isfinite(out["loss_gen_all"]) and torch.isfinite(out["loss_disc"])
    assert st.scaler.is_enabled()


@pytest.mark.gpu
def test_train_step_mel_variant_gpu_eager_and_graph(device):
    """train.py's variant on the HIP path: eager steps, then the whole step
    captured into one hipGraph and replayed (finite losses, D and G move)."""
    hps = tiny_mel_hps()
    st = _make(hps, device, variant="mel")
    batch = [t.to(device) for t in _batch(hps, 4, seed=0)]
    outs = [st.step(batch) for _ in range(2)]
    torch.cuda.synchronize()
    for out in outs:
        assert torch.isfinite(out["loss_gen_all"]) and torch.isfinite(out["loss_mel"])
    st = _make(hps, device, variant="mel", capturable=True)
    st.scaler = torch.amp.GradScaler("cuda", init_scale=64.0)
    st.capture(batch, warmup=2)
    d_p = [p.detach().clone() for p in st.net_d.parameters()]
    g_p = [p.detach().clone() for p in st.net_g.parameters()]
    outs = [{k: v.clone() for k, v in st.replay().items()} for _ in range(3)]
    torch.cuda.synchronize()
    for out in outs:
        assert torch.isfinite(out["loss_gen_all"]) and torch.isfinite(out["loss_disc"])
    assert any(not torch.equal(a, b) for a, b in zip(g_p, st.net_g.parameters()))
    assert any(not torch.equal(a, b) for a, b in zip(d_p, st.net_d.parameters()))


def test_grouped_spectral_norm_matches_torch_hooks():
    """GroupedSpectralNorm (one batched power iteration per weight shape) is
    the same math as torch.nn.utils.spectral_norm's per-layer hooks: in
    float64, outputs, gradients and the updated u/v buffers agree to 1e-12
    over two training forwards."""
    import copy

    import vits_amd.discriminators as D

    torch.manual_seed(0)
    d = D.MultiWaveSTFTDiscriminator().double()
    assert len(d._sn.groups) > 0
    sd = copy.deepcopy(d.state_dict())
    orig = D.GroupedSpectralNorm.__init__

    class Ref(D.MultiWaveSTFTDiscriminator):
        def forward(self, x, m):  # torch's hooks, no grouped pass
            return self.mwd(x) + self.mfd(m)

    D.GroupedSpectralNorm.__init__ = lambda self, root: setattr(self, "groups", {})
    try:
        r = Ref().double()
    finally:
        D.GroupedSpectralNorm.__init__ = orig
    r.load_state_dict(sd)
    d.load_state_dict(sd)
    y = torch.randn(2, 1, 3072, dtype=torch.float64)
    mags = [torch.rand(2, f // 2 + 1, 3072 // (f // 4) + 1, dtype=torch.float64)
            for f in (128, 256, 512, 1024, 2048)]
    for _ in range(2):
        la = sum(o.pow(2).mean() for o in d(y, mags))
        lb = sum(o.pow(2).mean() for o in r(y, mags))
        assert abs(la.item() - lb.item()) <= 1e-12 * abs(lb.item())
    la.backward()
    lb.backward()
    gr = dict(r.named_parameters())
    for k, p in d.named_parameters():
        assert torch.allclose(p.grad, gr[k].grad, rtol=1e-10, atol=1e-14), k
    for k, v in d.state_dict().items():
        assert torch.allclose(v, r.state_dict()[k], rtol=1e-12, atol=1e-15), k


@pytest.mark.gpu
def test_train_step_graph_capture_and_skip_rule(device):
    """The whole step captured into one hipGraph (TrainStep.capture): replays
    train (finite losses, parameters move, the device-side alignment noise
    decays) and GradScaler's skip rule holds without a host sync - with an
    overflowing loss scale every gradient is inf, so neither optimizer may
    touch its parameters or moments and the scale must back off."""
    hps = tiny_hps()
    st = _make(hps, device, capturable=True)
    # a small initial scale so the first replays are not skipped for fp16
    # overflow (GradScaler starts at 2**16 and halves per overflowing step)
    st.scaler = torch.amp.GradScaler("cuda", init_scale=64.0)
    batch = [t.to(device) for t in _batch(hps, 4, seed=0)]
    st.capture(batch, warmup=2)
    g_p = [p.detach().clone() for p in st.net_g.parameters()]
    d_p = [p.detach().clone() for p in st.net_d.parameters()]
    an0 = float(st.net_g.__dict__["_align_noise_t"])
    outs = [{k: v.clone() for k, v in st.replay().items()} for _ in range(3)]
    torch.cuda.synchronize()
    for out in outs:
        assert torch.isfinite(out["loss_gen_all"]) and torch.isfinite(out["loss_disc"])
    assert any(not torch.equal(a, b) for a, b in zip(g_p, st.net_g.parameters()))
    assert any(not torch.equal(a, b) for a, b in zip(d_p, st.net_d.parameters()))
    assert float(st.net_g.__dict__["_align_noise_t"]) < an0
    # force overflow: every step must be skipped
    st.scaler._scale.fill_(3.0e38)
    g_p = [p.detach().clone() for p in st.net_g.parameters()]
    d_p = [p.detach().clone() for p in st.net_d.parameters()]
    d_m = [st.optim_d.state[p]["exp_avg"].clone() for p in st.net_d.parameters()]
    st.replay()
    torch.cuda.synchronize()
    assert all(torch.equal(a, b) for a, b in zip(g_p, st.net_g.parameters()))
    assert all(torch.equal(a, b) for a, b in zip(d_p, st.net_d.parameters()))
    assert all(torch.equal(a, st.optim_d.state[p]["exp_avg"])
               for a, p in zip(d_m, st.net_d.parameters()))
    assert float(st.scaler._scale) < 3.0e38


@pytest.mark.gpu
def test_train_step_captured_lr_schedule(device):
    """Under capture both learning rates are device tensors read at replay:
    end_epoch() (the ExponentialLR decay of train_stft.py:138-139) changes
    what the replays use; replacing an lr object after capture raises
    instead of silently keeping the captured value."""
    hps = tiny_hps()
    st = _make(hps, device, capturable=True)
    st.scaler = torch.amp.GradScaler("cuda", init_scale=64.0)
    batch = [t.to(device) for t in _batch(hps, 4, seed=0)]
    st.capture(batch, warmup=2)
    lr_g = st.optim_g.param_groups[0]["lr"]
    lr_d = st.optim_d.param_groups[0]["lr"]
    assert isinstance(lr_g, torch.Tensor) and isinstance(lr_d, torch.Tensor)
    st.replay()
    st.end_epoch()
    st.end_epoch()
    assert st.optim_g.param_groups[0]["lr"] is lr_g  # updated in place
    assert abs(float(lr_g) - 2e-4 * hps.train.lr_decay ** 2) < 1e-10
    assert abs(float(lr_d) - 1e-4 * hps.train.lr_decay ** 2) < 1e-14
    st.replay()
    torch.cuda.synchronize()
    st.optim_d.param_groups[0]["lr"] = 5e-5
    with pytest.raises(RuntimeError):
        st.replay()


def test_rand_slice_device_rng_is_per_model():
    """capture() switches only its own model's slice draws to the device
    generator (it used to flip a module global for the whole
    process); another model's forward keeps the reference's host draw."""
    from vits_amd import commons

    x = torch.arange(2 * 3 * 40, dtype=torch.float32).view(2, 3, 40)
    torch.manual_seed(11)
    a, ids_a = commons.rand_slice_segments(x, torch.tensor([40, 30]), 8)
    torch.manual_seed(11)
    r = torch.rand([2])
    assert torch.equal(ids_a, (r * torch.tensor([33, 23])).long())
    assert torch.equal(a[1, 0], x[1, 0, ids_a[1]:ids_a[1] + 8])


@pytest.mark.gpu
def test_train_step_mel_variant_base_config_eager(device):
    """train.py's variant at configs/base.json shapes, B=32, eager (no graph):
    the configuration that hit a GPU memory fault in r01 while the MPD's
    strided / grouped convs ran on MIOpen.  Three eager steps
    on the current path (those convs as im2col + GEMM, stride-1 layers on
    the HIP conv): finite losses, both networks move."""
    from vits_amd.train import TrainStep, build_models, default_hps, synthetic_batch

    hps = default_hps()
    torch.manual_seed(1234)
    net_g, net_d = build_models(hps, device, "mel")
    st = TrainStep(hps, net_g, net_d, device, variant="mel")
    # GradScaler's default 2**16 would skip the first steps for fp16 overflow
    st.scaler = torch.amp.GradScaler("cuda", init_scale=64.0)
    batch = [t.to(device) for t in synthetic_batch(hps, 32, seed=0)]
    g0 = [p.detach().clone() for p in list(net_g.parameters())[:50]]
    d0 = [p.detach().clone() for p in net_d.parameters()]
    outs = [st.step(batch) for _ in range(3)]
    torch.cuda.synchronize()
    for out in outs:
        assert torch.isfinite(out["loss_gen_all"]) and torch.isfinite(out["loss_mel"])
        assert torch.isfinite(out["loss_disc"])
    assert any(not torch.equal(a, b) for a, b in zip(g0, net_g.parameters()))
    assert any(not torch.equal(a, b) for a, b in zip(d0, net_d.parameters()))


@pytest.mark.gpu
def test_bucketed_rccl_allreduce_in_captured_step(device):
    """The overlapped bucketed G all-reduce inside a captured hipGraph on
    RCCL (a one-rank nccl group on this GPU: the side stream, its event fork
    / join and the RCCL kernels are all captured and replayed): replays stay
    finite and end bit-identical to the flat all-reduce's capture (one rank:
    both are the identity on the gradients)."""
    hps = tiny_hps()
    hps.train.fp16_run = False  # fp32: no fp16 rounding chaos between the two runs
    batch = [t.to(device) for t in _batch(hps, 4, seed=0)]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0,
                            world_size=1)
    old_det = torch.backends.cudnn.deterministic
    # (MIOpen's default find picks run-dependent solvers for the STFT
    # discriminators' convs: profiles/r05_determinism.txt)
    torch.backends.cudnn.deterministic = True
    try:
        res = {}
        for mode in (True, "flat"):
            st = _make(hps, device, seed=0, capturable=True, allreduce=mode)
            assert (st._gbuckets is not None) == (mode is True)
            st.capture(batch, warmup=2)
            for _ in range(2):
                out = st.replay()
            torch.cuda.synchronize()
            assert torch.isfinite(out["loss_gen_all"]) and torch.isfinite(out["loss_disc"])
            res[mode] = torch.cat([p.detach().flatten() for p in st.net_g.parameters()])
        assert torch.equal(res[True], res["flat"])
    finally:
        torch.backends.cudnn.deterministic = old_det
        dist.destroy_process_group()
