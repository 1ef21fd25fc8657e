"""Where the train step's small torch kernels come from: one eager
train_stft step (B=32, base config, fp16 autocast) under a TorchDispatchMode
that counts every aten op of the glue kinds (copy / cast / fill / add / mul /
leaky_relu ...) by the innermost vits_amd call site (backward included: the
autograd engine runs on this thread).   python tools/glue_sites.py"""
import collections
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

from vits_amd.train import TrainStep, build_models, default_hps, synthetic_batch  # noqa: E402

GLUE = ("copy_", "_to_copy", "fill_", "zero_", "zeros", "zeros_like", "add", "add_", "mul",
        "mul_", "leaky_relu", "leaky_relu_backward", "sub", "div", "where", "cat", "sum",
        "neg", "clamp", "abs", "pow", "exp", "masked_fill", "index", "index_put_", "clone",
        "contiguous", "empty_like", "ones_like", "mean", "sigmoid", "tanh", "threshold_backward",
        "_foreach_add_", "lerp_", "addcmul_", "addcdiv_", "sqrt", "rsqrt", "reciprocal",
        "tanh_backward", "sigmoid_backward", "native_layer_norm", "native_layer_norm_backward")
HERE = os.path.join("vits_amd", "")


class Count(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.c = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = func.__name__.split(".")[0]
        if name in GLUE and any(isinstance(a, torch.Tensor) and a.is_cuda for a in args):
            site = "?"
            node = torch._C._current_autograd_node()
            if node is not None:
                # backward: the forward op's site from anomaly mode's traceback
                tb = node.metadata.get("traceback_", [])
                lines = "".join(tb).splitlines() if tb else []
                for ln in reversed(lines):
                    if HERE in ln and 'File "' in ln:
                        f = ln.split('File "')[1]
                        site = "bwd " + os.path.basename(f.split('"')[0]) + ":" + \
                            f.split("line ")[1].split(",")[0] + " " + type(node).__name__
                        break
                else:
                    site = "bwd ? " + type(node).__name__
            else:
                for f in reversed(traceback.extract_stack(limit=30)):
                    if HERE in f.filename and "glue_sites" not in f.filename:
                        site = f"{os.path.basename(f.filename)}:{f.lineno} {f.name}"
                        break
            self.c[(name, site)] += 1
        return func(*args, **(kwargs or {}))


dev = torch.device("cuda:0")
hps = default_hps()
torch.manual_seed(hps.train.seed)
net_g, net_d = build_models(hps, dev)
st = TrainStep(hps, net_g, net_d, dev)
batch = [t.to(dev) for t in synthetic_batch(hps, 32, tx=100, ty=500, seed=0)]
st.step(batch)
torch.cuda.synchronize()
torch.autograd.set_multithreading_enabled(False)
m = Count()
with torch.autograd.detect_anomaly(check_nan=False), m:
    st.step(batch)
torch.cuda.synchronize()
tot = sum(m.c.values())
print(f"glue ops in one step: {tot}")
for (name, site), n in m.c.most_common(80):
    print(f"{n:5d}  {name:22s} {site}")
