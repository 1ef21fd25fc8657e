"""Where the train step's small torch kernels come from: one eager
train_stft step (B=32, base config, fp16 autocast) under torch.profiler,
the glue ops (fill / copy / cast / add / mul / leaky_relu ...) grouped by
their Python call site (5 frames).  Output: a text table (stdout)."""
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vits_amd.train import TrainStep, build_models, default_hps, synthetic_batch  # noqa: E402

dev = torch.device("cuda:0")
hps = default_hps()
torch.manual_seed(hps.train.seed)
net_g, net_d = build_models(hps, dev)
st = TrainStep(hps, net_g, net_d, dev)
batch = [t.to(dev) for t in synthetic_batch(hps, 32, tx=100, ty=500, seed=0)]
for _ in range(2):
    st.step(batch)
torch.cuda.synchronize()
print("warm", flush=True)
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True,
             record_shapes=False) as prof:
    st.step(batch)
    torch.cuda.synchronize()
GLUE = ("aten::fill_", "aten::zero_", "aten::copy_", "aten::add", "aten::add_", "aten::mul",
        "aten::mul_", "aten::leaky_relu", "aten::leaky_relu_backward", "aten::sub", "aten::div",
        "aten::where", "aten::cat", "aten::sum", "aten::neg", "aten::clamp", "aten::abs",
        "aten::sqrt", "aten::pow", "aten::exp", "aten::masked_fill", "aten::index",
        "aten::index_put_", "aten::ones_like", "aten::zeros_like", "aten::fill_",
        "aten::_foreach_add_", "aten::mean")
rows = []
for e in prof.key_averages(group_by_stack_n=6):
    if e.key in GLUE and e.count > 0:
        rows.append((e.count, e.device_time_total / 1e3 if hasattr(e, "device_time_total")
                     else e.cuda_time_total / 1e3, e.key, e.stack))
rows.sort(key=lambda r: -r[0])
tot = sum(r[0] for r in rows)
print(f"glue calls {tot}", flush=True)
for cnt, ms, key, stack in rows[:70]:
    frames = " <- ".join(s.split("/")[-1][:70] for s in (stack or [])[:4])
    print(f"{cnt:5d} {ms:8.3f} ms {key:28s} {frames}")
