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
        """All 2 x len(resolutions) magnitude transforms run as one HIP launch
        (and one for their backward); the per-resolution losses are the
        reference's (STFTLoss.forward, stft_loss.py:35-44)."""
        from . import ops

        R = len(self.stft_losses)
        specs = [(f.window, f.fft_size, f.hop_size, f.win_size, None, 1e-7) for f in self.stft_losses]
        if R <= 8 and x.is_cuda:
            mags = ops.stft_mag_multi([x] * R + [y] * R, specs + specs)
            xs_mag, ys_mag = mags[:R], mags[R:]
        else:
            xs_mag = [f.mag(x, eps=1e-7) for f in self.stft_losses]
            ys_mag = [f.mag(y, eps=1e-7) for f in self.stft_losses]
        sc_loss, mag_loss = 0.0, 0.0
        for x_mag, y_mag in zip(xs_mag, ys_mag):
            sc_loss = sc_loss + torch.norm(y_mag - x_mag, p="fro") / torch.norm(y_mag, p="fro")
            mag_loss = mag_loss + F.l1_loss(torch.log(x_mag), torch.log(y_mag))
        return sc_loss / R, mag_loss / R, xs_mag, ys_mag
