"""Per-launch conv / fused-pair timing of the bench's infer_p2 step (B=16,
Tx=100, Ty=500, fp32): HIP events around every launch (ops.ConvTimer), the
algorithmic FLOPs of each, TF/s and the share of the step's conv time.
Shows which launches hold the dominant kernel's roofline fraction down."""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import torch  # noqa: E402

import bench  # noqa: E402
from vits_amd.ops import ConvTimer  # noqa: E402

PEAK = 157.3
dev = torch.device("cuda:0")
steps = int(os.environ.get("STEPS", "5"))
model = bench.build_model(dev)
inputs = bench.make_inputs(16, 100, 500, dev, seed=1234)
with torch.no_grad():
    for _ in range(3):
        model.infer_p2(*inputs)
    torch.cuda.synchronize()
    with ConvTimer() as timer:
        for _ in range(steps):
            model.infer_p2(*inputs)
    rows = timer.per_launch()
n = len(rows) // steps
agg = []
for i in range(n):
    lab = rows[i][0]
    ms = sorted(rows[i + j * n][1] for j in range(steps))[steps // 2]
    agg.append((i, lab, ms, rows[i][2]))
tot_ms = sum(a[2] for a in agg)
tot_fl = sum(a[3] for a in agg)
print(f"{n} launches/step, {tot_ms:.3f} ms, {tot_fl / tot_ms / 1e9:.1f} TF/s "
      f"({tot_fl / tot_ms / 1e9 / PEAK:.3f} of fp32 MFMA)")
lost = []
for i, lab, ms, fl in agg:
    tf = fl / ms / 1e9
    # time above what the launch would take at the step-average rate
    lost.append((ms - fl / (tot_fl / tot_ms), i, lab, ms, tf))
    print(f"{i:3d} {ms * 1e3:8.1f} us {tf:6.1f} TF/s {ms / tot_ms * 100:5.1f}%  {lab}")
print("\nlargest time over the average rate:")
for over, i, lab, ms, tf in sorted(lost, reverse=True)[:15]:
    print(f"{i:3d} +{over * 1e3:7.1f} us  {ms * 1e3:8.1f} us {tf:6.1f} TF/s  {lab}")
