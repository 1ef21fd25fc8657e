"""MR-STFT magnitude forward split by resolution group (bench.kernels_leg
shape: B=64, L=9216, y and y_hat): the n <= 1024 resolutions, n = 2048
alone, all five - device time per call from hipGraph replays."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from vits_amd import ops  # noqa: E402
from vits_amd.stft_loss import MultiResolutionSTFTLoss  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(7)
B, L = 64, 9216
y = (torch.randn(B, L, generator=g) * 0.1).to(dev)
yd = (torch.randn(B, L, generator=g) * 0.1).to(dev)
loss = MultiResolutionSTFTLoss().to(dev)
specs = [(f.window, f.fft_size, f.hop_size, f.win_size, None, 1e-7) for f in loss.stft_losses]
out = {}
for name, sel in (("n<=1024", [s for s in specs if s[1] <= 1024]),
                  ("n=2048", [s for s in specs if s[1] == 2048]), ("all", specs)):
    ms = bench._graph_ms(lambda sel=sel: ops.stft_mag_multi([y] * len(sel) + [yd] * len(sel),
                                                            sel + sel))
    out[name] = round(ms * 1e3, 1)
print(json.dumps({"us": out, "VITS_STFT_FWD": os.environ.get("VITS_STFT_FWD", "1")}), flush=True)
