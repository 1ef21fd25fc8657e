"""Multi-wave / multi-STFT discriminator (reference ``mrd.py``) — host-side
PyTorch modules so that the ``train_stft.py`` step (BASELINE configs 3/4) is
complete.  Not on the HIP hot path (adversarial-only, §8(f)
"next" #1); kept structurally identical so ``D_*.pth`` checkpoints (spectral
norm ``weight_orig/weight_u/weight_v`` keys) load unchanged.

Reference: WaveDiscriminator mrd.py:15-55, MultiWaveDiscriminator 58-91,
STFTDiscriminator 94-156, MultiSTFTDiscriminator 159-188,
MultiWaveSTFTDiscriminator 200-236.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.nn import Conv1d, Conv2d, LeakyReLU
from torch.nn.utils import spectral_norm, weight_norm

LRELU_SLOPE = 0.2


def _xavier_reset(module):
    def _reset(m):
        if isinstance(m, (Conv1d, Conv2d)):
            nn.init.xavier_uniform_(m.weight, gain=nn.init.calculate_gain("leaky_relu", LRELU_SLOPE))
            if m.bias is not None:
                m.bias.data.fill_(0.0)

    module.apply(_reset)


class WaveDiscriminator(nn.Module):
    def __init__(self, in_channels, kernel_size=5, layers=10, conv_channels=64, use_weight_norm=False):
        super().__init__()
        fnorm = weight_norm if use_weight_norm else spectral_norm
        convs = [fnorm(Conv1d(in_channels, conv_channels, 1)), LeakyReLU(LRELU_SLOPE)]
        for i in range(layers - 2):
            convs += [fnorm(Conv1d(conv_channels, conv_channels, kernel_size, padding=0, dilation=i + 2)),
                      LeakyReLU(LRELU_SLOPE)]
        convs += [fnorm(Conv1d(conv_channels, 1, 1))]
        self.convs = nn.Sequential(*convs)
        _xavier_reset(self)

    def forward(self, x):
        return self.convs(x).squeeze(1)


class MultiWaveDiscriminator(nn.Module):
    def __init__(self, num_dwt=5, kernel_size=5, layers=10, conv_channels=64, use_weight_norm=False):
        super().__init__()
        self.num_dwt = num_dwt
        self.discriminators = nn.ModuleList([
            WaveDiscriminator(2 ** i, kernel_size, layers, conv_channels + i * 32,
                              use_weight_norm=use_weight_norm) for i in range(num_dwt)])

    def forward(self, x):
        outs = []
        for i, d in enumerate(self.discriminators, 1):
            outs.append(d(x))
            if i == self.num_dwt:
                break
            b, c, t = x.shape
            period = 2 ** i
            if t % period != 0:
                n_pad = period - (t % period)
                x = F.pad(x, (0, n_pad), "reflect")
                t = t + n_pad
            x = x.view(b, period, -1)
        return outs


class STFTDiscriminator(nn.Module):
    def __init__(self, fft_size=1024, hop_size=256, win_size=1024, window="hann_window",
                 num_layers=4, kernel_size=3, stride=1, conv_channels=256, use_weight_norm=False):
        super().__init__()
        assert (kernel_size - 1) % 2 == 0, "Not support even number kernel size."
        self.fft_size, self.hop_size, self.win_size = fft_size, hop_size, win_size
        fnorm = weight_norm if use_weight_norm else spectral_norm
        nf = fft_size // 2 + 1
        s0 = int(nf ** (1.0 / float(num_layers)))
        k0, k1, cc = s0 * 2 + 1, kernel_size, conv_channels
        convs = [fnorm(Conv2d(1, cc, (k0, k1), stride=(s0, stride), padding=[0, k1 // 2])),
                 LeakyReLU(LRELU_SLOPE)]
        nf = int((nf - k0) / s0 + 1)
        for _ in range(num_layers - 2):
            convs += [fnorm(Conv2d(cc, cc, (k0, k1), stride=(s0, stride), padding=[0, k1 // 2])),
                      LeakyReLU(LRELU_SLOPE)]
            nf = int((nf - k0) / s0 + 1)
        convs += [fnorm(Conv2d(cc, 1, (nf, 1), stride=(1, 1), padding=0))]
        self.convs = nn.Sequential(*convs)
        _xavier_reset(self)

    def forward(self, x):
        return self.convs(x.unsqueeze(1)).squeeze_(1).squeeze_(2)


class MultiSTFTDiscriminator(nn.Module):
    def __init__(self, fft_sizes=[128, 256, 512, 1024], hop_sizes=[32, 64, 128, 256],
                 win_sizes=[128, 256, 512, 1024], num_layers=[5, 6, 7, 8], kernel_sizes=[5, 5, 5, 5],
                 conv_channels=[64, 64, 64, 64], use_weight_norm=False):
        super().__init__()
        self.discriminators = nn.ModuleList([
            STFTDiscriminator(fft_size=f, hop_size=h, win_size=w, num_layers=n, kernel_size=k,
                              conv_channels=c, use_weight_norm=use_weight_norm)
            for f, h, w, n, k, c in zip(fft_sizes, hop_sizes, win_sizes, num_layers, kernel_sizes,
                                        conv_channels)])

    def forward(self, xs):
        return [d(x) for x, d in zip(xs, self.discriminators)]


class MultiWaveSTFTDiscriminator(nn.Module):
    def __init__(self,
                 multi_wave_discriminator_params={"num_dwt": 5, "kernel_size": 5, "layers": 10,
                                                  "conv_channels": 64, "use_weight_norm": False},
                 multi_stft_discriminator_params={"fft_sizes": [128, 256, 512, 1024, 2048],
                                                  "hop_sizes": [32, 64, 128, 256, 512],
                                                  "win_sizes": [128, 256, 512, 1024, 2048],
                                                  "num_layers": [5, 6, 7, 8, 9],
                                                  "kernel_sizes": [5, 5, 5, 5, 5],
                                                  "conv_channels": [64, 64, 64, 64, 64],
                                                  "use_weight_norm": False}):
        super().__init__()
        self.mwd = MultiWaveDiscriminator(**multi_wave_discriminator_params)
        self.mfd = MultiSTFTDiscriminator(**multi_stft_discriminator_params)

    def forward(self, x, m):
        """x [B, 1, t] waveform, m list of STFT magnitudes [B, F, T] (the
        MR-STFT loss's outputs, train_stft.py:198-199)."""
        return self.mwd(x) + self.mfd(m)
