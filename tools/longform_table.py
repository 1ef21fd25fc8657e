"""Per-launch conv table of the C5 long-form step (bf16 model, B=4,
Tx=500, Ty=2500) - bench.conv_kernel_table on that workload - plus the
whole-step time, to see where the long-form leg's time goes."""
import os
import sys
import time

import torch

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import bench  # noqa: E402
from vits_amd.ops import ConvTimer  # noqa: E402

dev = torch.device("cuda:0")
dt = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[
    os.environ.get("DT", "bf16")]
m = bench.build_model(dev).to(dt)
inputs = bench.make_inputs(4, 500, 2500, dev, seed=4321)
with torch.no_grad():
    for _ in range(2):
        m.infer_p2(*inputs)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        m.infer_p2(*inputs)
    torch.cuda.synchronize()
    print(f"eager step {(time.perf_counter() - t0) / 5 * 1e3:.3f} ms")
    with ConvTimer() as timer:
        for _ in range(3):
            m.infer_p2(*inputs)
    rows = bench.conv_kernel_table(timer, 3)
    if dt != torch.float32:  # output SNR against the fp32 model on the same inputs
        out = m.infer_p2(*inputs).float()
        m32 = bench.build_model(dev)
        ref = m32.infer_p2(*inputs).float()
        snr = 10 * torch.log10((ref ** 2).sum() / ((out - ref) ** 2).sum().clamp_min(1e-30))
        print(f"snr vs fp32 {float(snr):.2f} dB")
tot = sum(r["ms_per_step"] for r in rows)
print(f"conv total {tot:.3f} ms/step over {len(rows)} shapes")
for r in rows:
    print(f"{r['kernel'][:84]:84s} {r['arith']:9s} {r['launches_per_step']:5} {r['ms_per_step']:8.4f} "
          f"{r['achieved']:8.1f} {r['frac']:.3f}")
