"""Shape census of the HIP training convs (forward and data-gradient
launches, train_ops._run) in one eager train_stft step at B=32: per shape,
calls, HIP-event time and TF/s; then the wgrad launches the same way.
python tools/train_conv_census.py"""
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from vits_amd import train_ops  # noqa: E402
from vits_amd.train import TrainStep, build_models, default_hps, synthetic_batch  # noqa: E402

rec = collections.defaultdict(list)
orig_run, orig_wgrad = train_ops._run, train_ops.wgrad


def run(x, layer, n_out, in_slope=1.0, gmask=None, gmask_slope=1.0, io16=False, res=None):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    y = orig_run(x, layer, n_out, in_slope, gmask, gmask_slope, io16, res)
    e.record()
    # 16-byte staging needs time-contiguous rows, T % 4 == 0, 4-element
    # aligned strides and base (csrc/conv1d_impl.h launch_tile)
    v4 = (x.stride(2) == 1 and x.stride(1) % 4 == 0 and x.stride(0) % 4 == 0
          and x.shape[2] % 4 == 0 and x.data_ptr() % (4 * x.element_size()) == 0)
    key = ("fwd" if gmask is None else "dgrad", layer.m, layer.cin, layer.k, layer.dil, n_out,
           x.shape[0], layer.tile, f"v4={int(v4)} tin={x.shape[2]} {tuple(x.stride())}")
    rec[key].append((s, e, 2 * x.shape[0] * layer.m * n_out * layer.cin * layer.k))
    return y


def wgrad(dy, x, k, dil, pad, slope, **kw):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    out = orig_wgrad(dy, x, k, dil, pad, slope, **kw)
    e.record()
    key = ("wgrad", dy.shape[1], x.shape[1], k, dil, dy.shape[2], x.shape[0], 0, "")
    rec[key].append((s, e, 2 * x.shape[0] * dy.shape[1] * dy.shape[2] * x.shape[1] * k))
    return out


dev = torch.device("cuda:0")
hps = default_hps()
torch.manual_seed(1234)
g, d = build_models(hps, dev)
st = TrainStep(hps, g, d, dev, log_mels=False)
batch = [t.to(dev) for t in synthetic_batch(hps, 32, seed=0)]
st.step(batch)
torch.cuda.synchronize()
train_ops._run, train_ops.wgrad = run, wgrad
st.step(batch)
torch.cuda.synchronize()
rows = []
for key, v in rec.items():
    ms = sum(s.elapsed_time(e) for s, e, _ in v)
    fl = sum(f for _, _, f in v)
    rows.append((ms, key, len(v), fl / ms / 1e9))
tot = sum(r[0] for r in rows)
print(f"total {tot:.2f} ms over {sum(r[2] for r in rows)} launches")
for ms, key, n, tf in sorted(rows, reverse=True)[:45]:
    kind, m, cin, k, dil, n_out, B, tile, st = key
    print(f"{ms:7.3f} ms {n:4d}x {tf:7.1f} TF/s  {kind:5s} m={m:4d} cin={cin:4d} k={k:2d} d={dil} "
          f"T={n_out:6d} B={B:4d} tile={tile} {st}")
