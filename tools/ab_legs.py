"""A/B of bench.py's train (C4, B=32, captured) and long-form (C5, bf16,
captured) legs under python-side settings, one arm per process:
  python tools/ab_legs.py [--legs train,longform]
VITS_AMD_LIB picks the library build (tools/ab_build.sh).
Prints one JSON line."""
import argparse
import json
import os
import sys
import types

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--legs", default="train,longform")
ap.add_argument("--pair16-256", type=int, default=None,
                help="ops.PAIR16_256_MAX_K (0: the 256-channel stage's two-conv path)")
a = ap.parse_args()
if a.pair16_256 is not None:
    from vits_amd import ops
    ops.PAIR16_256_MAX_K = a.pair16_256
dev = torch.device("cuda:0")
out = {"lib": os.environ.get("VITS_AMD_LIB", "default"), "pair16_256": a.pair16_256}
legs = a.legs.split(",")
if "train" in legs:
    args = types.SimpleNamespace(train_eager=False, train_batch=32, tx=100, ty=500,
                                 train_warmup=3, train_steps=10, no_cpu_baseline=True)
    r = bench.train_leg(args, dev, 0, 1, None, 32, cpu_base=False)
    out["train_ms"] = r["ms_per_step"]
if "longform" in legs:
    model = bench.build_model(dev)
    r = bench.longform_leg(model, dev, 0)
    out["longform_ms"] = r["ms_per_step"]
    out["longform_conv_ms"] = r["roofline"]["conv_ms_per_step"]
print(json.dumps(out), flush=True)
