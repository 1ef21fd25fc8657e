"""Where the train_stft step's small torch ops (copies, casts, elementwise)
come from: one eager step under a TorchDispatchMode that records every aten
op with the vits_amd source line that issued it (forward and backward), and
the bytes it writes.  python tools/glue_prof.py --batch 32 > out.txt"""
import argparse
import collections
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

from vits_amd.train import TrainStep, build_models, default_hps, synthetic_batch  # noqa: E402

SKIP = ("view", "as_strided", "_reshape_alias", "detach", "t.default", "transpose", "permute",
        "expand", "slice", "select", "unsqueeze", "squeeze", "split", "chunk", "unbind",
        "empty", "_unsafe_view", "alias", "lift_fresh", "is_same_size", "_to_copy.default?")


class Rec(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.agg = collections.defaultdict(lambda: [0, 0])

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        name = str(func)
        if any(s in name for s in SKIP):
            return out
        where = "?"
        for fr in reversed(traceback.extract_stack()[:-1]):
            if "/vits_amd/" in fr.filename:
                where = f"{fr.filename.split('/vits_amd/')[-1]}:{fr.lineno} {fr.name}"
                break
        if where == "?":
            # backward: the forward site of the autograd node being run
            # (anomaly mode stores each node's forward traceback)
            node = torch._C._current_autograd_node()
            if node is not None:
                tb = node.metadata.get("traceback_", [])
                lines = tb if isinstance(tb, list) else str(tb).splitlines()
                site = "?"
                for ln in lines:
                    ln = str(ln)
                    if "/vits_amd/" in ln and "line" in ln:
                        site = ln.strip().split("/vits_amd/")[-1].replace('", line ', ":")
                where = f"bwd[{node.name()}] {site}"
        nbytes = 0
        for o in (out if isinstance(out, (tuple, list)) else (out,)):
            if isinstance(o, torch.Tensor):
                nbytes += o.numel() * o.element_size()
        a = self.agg[(name, where)]
        a[0] += nbytes
        a[1] += 1
        return out


ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=32)
ap.add_argument("--top", type=int, default=70)
ap.add_argument("--by", choices=("bytes", "count"), default="bytes")
args = ap.parse_args()
dev = torch.device("cuda:0")
hps = default_hps()
torch.manual_seed(1234)
g, d = build_models(hps, dev)
st = TrainStep(hps, g, d, dev, log_mels=True)
batch = [t.to(dev) for t in synthetic_batch(hps, args.batch, seed=0)]
st.step(batch)
torch.cuda.synchronize()
rec = Rec()
with rec, torch.autograd.detect_anomaly(check_nan=False):
    st.step(batch)
torch.cuda.synchronize()
tot = sum(v[0] for v in rec.agg.values())
print(f"ops {sum(v[1] for v in rec.agg.values())}, bytes written {tot / 2**20:.1f} MiB")
key = 0 if args.by == "bytes" else 1
for (name, where), (b, n) in sorted(rec.agg.items(), key=lambda kv: -kv[1][key])[:args.top]:
    print(f"{b / 2**20:9.1f} MiB {n:5d}  {name:40s} {where}")
