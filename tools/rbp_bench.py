"""Split-fp32 fused ResBlock2 pair (csrc/resblock_f32p.hip) vs the two-conv
path on the bench workload's 256/128/64-channel stages (B=16, Ty=500): per
(stage, dilation) the three branches (k = 3, 7, 11) as the engine launches
them - two-conv: one grouped c1 launch + one grouped c2 launch; fused: one
grouped pair launch - and each branch alone.  HIP events; TF/s over the
pairs' algorithmic FLOPs.  ONLY=C128 filters."""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import torch  # noqa: E402

from vits_amd import ops  # noqa: E402
from vits_amd.ops import make_desc, make_out  # noqa: E402

dev = torch.device("cuda:0")
B, Ty = 16, 500
reps = int(os.environ.get("REPS", "5"))
only = os.environ.get("ONLY")


def timeit(fn):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


tot = {"two": 0.0, "fused": 0.0}
for C, T in ((256, 8 * Ty), (128, 48 * Ty), (64, 96 * Ty), (32, 192 * Ty)):
    for d in (1, 3, 5):
        name = f"C{C}.d{d}"
        if only and only not in name:
            continue
        x = torch.randn(B, C, T, device=dev) * 0.5
        cond = torch.randn(B, C, device=dev) * 0.3
        br = []
        for k in (3, 7, 11):
            w1 = torch.randn(C, C, k, device=dev) / (C * k) ** 0.5
            w2 = torch.randn(C, C // 2, k, device=dev) / (C * k / 2) ** 0.5
            c1 = ops.to_lowp(ops.pack_conv(w1, torch.zeros(C, device=dev), dilation=d, gate=True),
                             ops.WDT_F32S, min_rows=0)
            c2 = ops.to_lowp(ops.pack_conv(w2, torch.zeros(C, device=dev)), ops.WDT_F32S,
                             min_rows=0)
            gb = torch.empty(B, C // 2, T, device=dev)
            y = torch.empty(B, C, T, device=dev)
            d1 = make_desc(c1, x, make_out(gb), in_slope=0.1, cond=cond)
            d2 = make_desc(c2, gb, make_out(y, res=x))
            pd = ops.resblock_pair_desc(c1, c2, x, y, cond=cond)
            br.append((k, d1, d2, pd))
        fl = sum(ops.resblock_pair_flops(b[3], B) for b in br)
        t2 = timeit(lambda: ops.conv1d_launch_seq([tuple(b[1] for b in br), tuple(b[2] for b in br)],
                                                  B, dev))
        tf = timeit(lambda: ops.resblock_pair_launch(tuple(b[3] for b in br), B, dev, ops.WDT_F32P))
        tot["two"] += t2
        tot["fused"] += tf
        print(f"{name:8s} group k3+7+11  two-conv {t2*1e3:7.1f} us {fl/t2/1e9:6.1f} TF/s"
              f"   fused {tf*1e3:7.1f} us {fl/tf/1e9:6.1f} TF/s", flush=True)
        for k, d1, d2, pd in br:
            f1 = ops.resblock_pair_flops(pd, B)
            a = timeit(lambda: ops.conv1d_launch_seq([d1, d2], B, dev))
            b = timeit(lambda: ops.resblock_pair_launch(pd, B, dev, ops.WDT_F32P))
            print(f"   k{k:<2d}  two-conv {a*1e3:7.1f} us {f1/a/1e9:6.1f} TF/s"
                  f"   fused {b*1e3:7.1f} us {f1/b/1e9:6.1f} TF/s", flush=True)
print(f"TOTAL (groups) two-conv {tot['two']:.3f} ms  fused {tot['fused']:.3f} ms")
# the 32-channel stage's shipped exact-fp32 path (resblock.hip pairs for k <= 7,
# two exact convs for k = 11) beside the split-fp32 fused pair
C, T = 32, 192 * Ty
if not only or "C32" in only:
    tex = tsp = 0.0
    for d in (1, 3, 5):
        x = torch.randn(B, C, T, device=dev) * 0.5
        cond = torch.randn(B, C, device=dev) * 0.3
        for k in (3, 7, 11):
            w1 = torch.randn(C, C, k, device=dev) / (C * k) ** 0.5
            w2 = torch.randn(C, C // 2, k, device=dev) / (C * k / 2) ** 0.5
            e1 = ops.pack_conv(w1, torch.zeros(C, device=dev), dilation=d, gate=True)
            e2 = ops.pack_conv(w2, torch.zeros(C, device=dev))
            s1 = ops.to_lowp(e1, ops.WDT_F32S, min_rows=0)
            s2 = ops.to_lowp(e2, ops.WDT_F32S, min_rows=0)
            y = torch.empty(B, C, T, device=dev)
            if ops.resblock_pair_supported(e1, e2, T):
                pe = ops.resblock_pair_desc(e1, e2, x, y, cond=cond)
                te = timeit(lambda: ops.resblock_pair_launch(pe, B, dev))
            else:
                gb = torch.empty(B, C // 2, T, device=dev)
                ds = [make_desc(e1, x, make_out(gb), in_slope=0.1, cond=cond),
                      make_desc(e2, gb, make_out(y, res=x))]
                te = timeit(lambda: ops.conv1d_launch_seq(ds, B, dev))
            ps = ops.resblock_pair_desc(s1, s2, x, y, cond=cond)
            ts = timeit(lambda: ops.resblock_pair_launch(ps, B, dev, ops.WDT_F32P))
            f1 = ops.resblock_pair_flops(ps, B)
            tex += te
            tsp += ts
            print(f"C32.k{k}d{d}  exact (shipped) {te*1e3:7.1f} us {f1/te/1e9:6.1f} TF/s"
                  f"   split fused {ts*1e3:7.1f} us {f1/ts/1e9:6.1f} TF/s", flush=True)
    print(f"TOTAL C32 exact {tex:.3f} ms  split fused {tsp:.3f} ms")
