"""Multi-resolution STFT loss (reference ``stft_loss.py``) on the HIP STFT
magnitude kernel.

The magnitudes come from ``vits_stft_mag_forward`` (LDS radix-2 FFT) and
back-propagate through ``vits_stft_mag_backward`` (adjoint FFT + windowed
overlap-add + reflect fold), so ``y_hat`` gets its gradient without
torch.stft.  The loss reductions are small torch ops.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .modules import TorchSTFT


class STFTLoss(TorchSTFT):
    """(sc, log-mag L1, x_mag, y_mag) at one resolution (stft_loss.py:15-44)."""

    def __init__(self, fft_size, hop_size, win_size):
        super().__init__(fft_size, hop_size, win_size)

    def spec2mag(self, real, imag):
        return torch.sqrt(real ** 2 + imag ** 2 + 1e-7)

    def forward(self, x, y):
        x_mag = self.mag(x, eps=1e-7)
        y_mag = self.mag(y, eps=1e-7)
        sc_loss = torch.norm(y_mag - x_mag, p="fro") / torch.norm(y_mag, p="fro")
        mag_loss = F.l1_loss(torch.log(x_mag), torch.log(y_mag))
        return sc_loss, mag_loss, x_mag, y_mag


class MultiResolutionSTFTLoss(nn.Module):
    """Mean over resolutions (stft_loss.py:47-95).  Default resolutions
    (128,32,128) ... (2048,512,2048) as the reference."""

    def __init__(self, fft_sizes=[128, 256, 512, 1024, 2048], hop_sizes=[32, 64, 128, 256, 512],
                 win_sizes=[128, 256, 512, 1024, 2048]):
        super().__init__()
        assert len(fft_sizes) == len(hop_sizes) == len(win_sizes)
        self.stft_losses = nn.ModuleList(
            [STFTLoss(fs, ss, wl) for fs, ss, wl in zip(fft_sizes, hop_sizes, win_sizes)])

    def forward(self, x, y):
        sc_loss, mag_loss = 0.0, 0.0
        xs_mag, ys_mag = [], []
        for f in self.stft_losses:
            sc_l, mag_l, x_mag, y_mag = f(x, y)
            sc_loss = sc_loss + sc_l
            mag_loss = mag_loss + mag_l
            xs_mag.append(x_mag)
            ys_mag.append(y_mag)
        n = len(self.stft_losses)
        return sc_loss / n, mag_loss / n, xs_mag, ys_mag
