"""neg_cent at the C3 shape (B=64, C=192, t_t=500, t_s=100), 20 calls: run
under rocprofv3 --kernel-trace --stats for the kernel's device time."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from vits_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator(device="cpu").manual_seed(7)
z = torch.randn(64, 192, 500, generator=g).to(dev)
m = torch.randn(64, 192, 100, generator=g).to(dev)
lg = (torch.randn(64, 192, 100, generator=g) * 0.5).to(dev)
for _ in range(20):
    ops.neg_cent(z, m, lg)
torch.cuda.synchronize()
