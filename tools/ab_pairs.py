"""A/B of the headline infer_p2 step (bench.py's workload: B=16, Tx=100,
Ty=500, fp32) under fused-pair rules, interleaved in one process:
  none   - every split-fp32 pair on the two-conv path
  rule   - ops.F32P_PAIR_MAX_K as shipped
  all    - every 64/128/256 pair fused
Prints ms per step (min / median over ROUNDS rounds of STEPS steps)."""
import os
import statistics
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import torch  # noqa: E402

from bench import build_model, make_inputs  # noqa: E402
from vits_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
steps = int(os.environ.get("STEPS", "20"))
rounds = int(os.environ.get("ROUNDS", "4"))
model = build_model(dev)
inputs = make_inputs(16, 100, 500, dev, seed=1234)
shipped = dict(ops.F32P_PAIR_MAX_K)
variants = {"none": {}, "rule": shipped, "all": {64: 15, 128: 15, 256: 15}}
extra = os.environ.get("EXTRA")  # e.g. "c128k11=64:11,128:11"
if extra:
    name, spec = extra.split("=")
    variants[name] = {int(a): int(b) for a, b in (kv.split(":") for kv in spec.split(","))}
res = {v: [] for v in variants}
outs = {}
with torch.no_grad():
    for r in range(rounds):
        for v, rule in variants.items():
            ops.F32P_PAIR_MAX_K = rule
            for _ in range(3):
                model.infer_p2(*inputs)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                o = model.infer_p2(*inputs)
            torch.cuda.synchronize()
            res[v].append((time.perf_counter() - t0) / steps * 1e3)
            if r == 0:
                outs[v] = o[0].clone() if isinstance(o, tuple) else o.clone()
for v, ts in res.items():
    eq = torch.equal(outs[v], outs["none"])
    print(f"{v:8s} min {min(ts):7.3f} ms  median {statistics.median(ts):7.3f} ms  "
          f"bitwise==none {eq}", flush=True)
