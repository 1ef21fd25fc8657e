"""Per-shape table of the train_stft step's HIP convs (forward / input
gradient, every conv1d_launch via ops.ConvTimer) and weight gradients
(train_ops.wgrad, timed with HIP events on the launch stream), from one eager
step at B=32 (base config, fp16 autocast).  Rows: launches, ms, TF/s
(algorithmic: 2 * Cout * Cin * k * T * B), fraction of the fp16 dense peak.
Usage: python tools/train_conv_table.py [--batch 32]."""
import argparse
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vits_amd import ops, train_ops  # noqa: E402
from vits_amd.train import TrainStep, build_models, default_hps, synthetic_batch  # noqa: E402

PEAK = 2500.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--top", type=int, default=60)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    hps = default_hps()
    torch.manual_seed(hps.train.seed)
    net_g, net_d = build_models(hps, dev)
    st = TrainStep(hps, net_g, net_d, dev)
    batch = [t.to(dev) for t in synthetic_batch(hps, a.batch, tx=100, ty=500, seed=0)]
    for _ in range(2):
        st.step(batch)
    torch.cuda.synchronize()

    wrec = []
    orig = train_ops.wgrad

    def timed_wgrad(dy, x, k, dil, pad_left, *args, **kw):
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        out = orig(dy, x, k, dil, pad_left, *args, **kw)
        e.record()
        B, cout, n = dy.shape
        cin = x.shape[1]
        wrec.append((f"wgrad co{cout} ci{cin} k{k} d{dil} T{n} B{B} {str(dy.dtype)[6:]}", s, e,
                     2 * B * cout * cin * k * n))
        return out

    train_ops.wgrad = timed_wgrad
    try:
        with ops.ConvTimer() as timer:
            st.step(batch)
        torch.cuda.synchronize()
    finally:
        train_ops.wgrad = orig
    rows = collections.defaultdict(lambda: [0, 0.0, 0])
    for lab, ms, fl in timer.per_launch():
        r = rows[lab.replace("conv ", "conv  ")]
        r[0] += 1
        r[1] += ms
        r[2] += fl
    for lab, s, e, fl in wrec:
        r = rows[lab]
        r[0] += 1
        r[1] += s.elapsed_time(e)
        r[2] += fl
    tot_ms = sum(r[1] for r in rows.values())
    tot_fl = sum(r[2] for r in rows.values())
    print(f"{sum(r[0] for r in rows.values())} launches, {tot_ms:.2f} ms, "
          f"{tot_fl / tot_ms / 1e9:.1f} TF/s ({tot_fl / tot_ms / 1e9 / PEAK:.3f} of fp16 dense)")
    for kind in ("conv", "wgrad"):
        sub = {k: v for k, v in rows.items() if k.startswith(kind)}
        ms = sum(v[1] for v in sub.values())
        fl = sum(v[2] for v in sub.values())
        print(f"  {kind}: {sum(v[0] for v in sub.values())} launches {ms:.2f} ms "
              f"{fl / max(ms, 1e-9) / 1e9:.1f} TF/s")
    print(f"{'n':>4} {'ms':>8} {'TF/s':>7} {'frac':>6}  shape")
    for lab, (n, ms, fl) in sorted(rows.items(), key=lambda kv: -kv[1][1])[:a.top]:
        tf = fl / max(ms, 1e-9) / 1e9
        print(f"{n:4d} {ms:8.3f} {tf:7.1f} {tf / PEAK:6.3f}  {lab}")


if __name__ == "__main__":
    main()
