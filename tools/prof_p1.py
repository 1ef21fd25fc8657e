"""infer_p1 at B=1, Tx=100 (10 calls) — for rocprofv3 kernel stats."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda:0")
m = bench.build_model(dev)
g = torch.Generator().manual_seed(11)
x = torch.randn(1, 100, 256, generator=g).to(dev)
emo = torch.randn(1, 1024, generator=g).to(dev)
sid = torch.tensor([1], device=dev)
with torch.no_grad():
    for _ in range(11):
        m.infer_p1(x, emo, sid)
torch.cuda.synchronize()
