"""Run the MR-STFT magnitude launches a few times (for rocprofv3 --pmc):
the n <= 1024 group and n = 2048, B=64, L=9216, y and y_hat."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vits_amd import ops  # noqa: E402
from vits_amd.stft_loss import MultiResolutionSTFTLoss  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(7)
y = (torch.randn(64, 9216, generator=g) * 0.1).to(dev)
loss = MultiResolutionSTFTLoss().to(dev)
specs = [(f.window, f.fft_size, f.hop_size, f.win_size, None, 1e-7) for f in loss.stft_losses]
for _ in range(3):
    ops.stft_mag_multi([y] * 5 + [y] * 5, specs + specs)
torch.cuda.synchronize()
print("ok", flush=True)
