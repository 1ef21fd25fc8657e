"""Which WN residual/skip updates of one eager train_stft step fall back to
torch ops (train_ops.wn_update returning None), and why: dtypes,
contiguity and the autocast state of each call.
    python tools/wn_fallback_debug.py"""
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from vits_amd import modules, train_ops  # noqa: E402
from vits_amd.train import TrainStep, build_models, default_hps, synthetic_batch  # noqa: E402

seen = collections.Counter()
orig = train_ops.wn_update


def wn_update(x, rs, mask, out):
    r = orig(x, rs, mask, out)
    if r is None:
        wdt = train_ops.autocast_wdtype() if x.device.type == "cuda" else None
        seen[(f"wdt={wdt}", f"x={x.dtype},{tuple(x.shape)},c={x.is_contiguous()}",
              f"rs={rs.dtype},c={rs.is_contiguous()}", f"mask={mask.dtype},c={mask.is_contiguous()}",
              f"out={None if out is None else (out.dtype, out.is_contiguous())}")] += 1
    return r


train_ops.wn_update = wn_update
modules.train_ops.wn_update = wn_update
dev = torch.device("cuda:0")
hps = default_hps()
torch.manual_seed(1234)
g, d = build_models(hps, dev)
st = TrainStep(hps, g, d, dev, log_mels=False)
batch = [t.to(dev) for t in synthetic_batch(hps, 8, seed=0)]
st.step(batch)
torch.cuda.synchronize()
for k, n in seen.most_common():
    print(n, *k)
print("WN_DEBUG_DONE")
