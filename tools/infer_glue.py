"""Every torch (aten) op of one eager headline infer_p2 step (B=16, Tx=100,
Ty=500, fp32) by its innermost vits_amd call site - the small copy / fill /
elementwise kernels around the HIP launches.   python tools/infer_glue.py"""
import collections
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

from bench import build_model, make_inputs  # noqa: E402

HERE = os.path.join("vits_amd", "")
SKIP = {"empty", "empty_strided", "view", "_unsafe_view", "as_strided", "detach", "slice",
        "select", "t", "transpose", "permute", "unsqueeze", "squeeze", "expand", "reshape",
        "alias", "split", "split_with_sizes", "unbind", "narrow", "lift_fresh", "_to_copy_meta"}


class Count(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.c = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = func.__name__.split(".")[0]
        if name not in SKIP and any(isinstance(a, torch.Tensor) and a.is_cuda for a in args):
            site = "?"
            for f in reversed(traceback.extract_stack(limit=40)):
                if HERE in f.filename:
                    site = f"{os.path.basename(f.filename)}:{f.lineno} {f.name}"
                    break
            self.c[(name, site)] += 1
        return func(*args, **(kwargs or {}))


dev = torch.device("cuda:0")
model = build_model(dev)
inputs = make_inputs(16, 100, 500, dev, seed=1234)
with torch.no_grad():
    model.infer_p2(*inputs)
    torch.cuda.synchronize()
    m = Count()
    with m:
        model.infer_p2(*inputs)
torch.cuda.synchronize()
print(f"aten ops on the GPU in one step: {sum(m.c.values())}")
for (name, site), n in m.c.most_common(60):
    print(f"{n:5d}  {name:24s} {site}")
