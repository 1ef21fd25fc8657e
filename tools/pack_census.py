"""Which convs still pack their 16-bit weight images per call (not served by
train_ops.prepacked): one eager train_stft step (B=32, base config, fp16
autocast) with train_ops.PACK_TRACE on, the per-call packs counted by call
site.    python tools/pack_census.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import collections  # noqa: E402

from vits_amd import train_ops  # noqa: E402

train_ops.PACK_TRACE = collections.Counter()
from vits_amd.train import TrainStep, build_models, default_hps, synthetic_batch  # noqa: E402

dev = torch.device("cuda:0")
hps = default_hps()
torch.manual_seed(hps.train.seed)
net_g, net_d = build_models(hps, dev)
st = TrainStep(hps, net_g, net_d, dev)
batch = [t.to(dev) for t in synthetic_batch(hps, 32, tx=100, ty=500, seed=0)]
st.step(batch)
train_ops.PACK_TRACE.clear()
st.step(batch)
torch.cuda.synchronize()
tot = sum(train_ops.PACK_TRACE.values())
print(f"per-call packs in one step: {tot}")
for (kind, shape, site), n in train_ops.PACK_TRACE.most_common(40):
    print(f"{n:5d}  {kind:7s} {str(shape):18s} {site}")
