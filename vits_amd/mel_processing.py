"""Linear / mel spectrograms (reference ``mel_processing.py``) on the HIP STFT.

* ``spectrogram_torch``  = reflect-pad (n_fft-hop)/2, STFT(center=False,
  hann(win) centred in n_fft), sqrt(|X|^2 + 1e-6)   (mel_processing.py:58-77)
  -> one ``vits_stft_mag_forward`` call with pad=(n_fft-hop)/2.
* ``spec_to_mel_torch`` / ``mel_spectrogram_torch`` add the Slaney mel basis
  and log(clamp(., 1e-5))                          (mel_processing.py:80-119).

The mel basis is librosa.filters.mel(sr, n_fft, n_mels, fmin, fmax) with
Slaney scale and Slaney area normalisation; librosa is not a dependency, the
formula is restated in ``mel_filterbank`` (host-side numpy, computed once
per (device, config) and cached, as the reference caches its basis).
"""
from __future__ import annotations

import numpy as np
import torch

from . import ops

MAX_WAV_VALUE = 32768.0
_mel_basis: dict = {}
_hann_window: dict = {}


def _hz_to_mel(f):
    f = np.asanyarray(f, dtype=np.float64)
    f_sp = 200.0 / 3
    mels = f / f_sp
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-10) / min_log_hz) / logstep,
                    mels)


def _mel_to_hz(m):
    m = np.asanyarray(m, dtype=np.float64)
    f_sp = 200.0 / 3
    freqs = f_sp * m
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), freqs)


def mel_filterbank(sr: int, n_fft: int, n_mels: int = 128, fmin: float = 0.0,
                   fmax=None) -> np.ndarray:
    """[n_mels, 1 + n_fft//2] float32 Slaney mel basis (librosa semantics)."""
    if fmax is None:
        fmax = float(sr) / 2
    weights = np.zeros((n_mels, 1 + n_fft // 2), dtype=np.float32)
    fftfreqs = np.fft.rfftfreq(n=n_fft, d=1.0 / sr)
    mel_f = _mel_to_hz(np.linspace(_hz_to_mel(fmin), _hz_to_mel(fmax), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = np.subtract.outer(mel_f, fftfreqs)
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        weights[i] = np.maximum(0, np.minimum(lower, upper))
    enorm = 2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels])
    weights *= enorm[:, np.newaxis]
    return weights


librosa_mel_fn = mel_filterbank


def dynamic_range_compression_torch(x, C=1, clip_val=1e-5):
    return torch.log(torch.clamp(x, min=clip_val) * C)


def dynamic_range_decompression_torch(x, C=1):
    return torch.exp(x) / C


def spectral_normalize_torch(magnitudes):
    return dynamic_range_compression_torch(magnitudes)


def spectral_de_normalize_torch(magnitudes):
    return dynamic_range_decompression_torch(magnitudes)


def _window(win_size, device):
    key = (win_size, str(device))
    if key not in _hann_window:
        _hann_window[key] = torch.hann_window(win_size).to(device=device, dtype=torch.float32)
    return _hann_window[key]


def _basis(sampling_rate, n_fft, num_mels, fmin, fmax, device):
    key = (sampling_rate, n_fft, num_mels, fmin, fmax, str(device))
    if key not in _mel_basis:
        mel = mel_filterbank(sr=sampling_rate, n_fft=n_fft, n_mels=num_mels, fmin=fmin, fmax=fmax)
        _mel_basis[key] = torch.from_numpy(mel).to(device=device)
    return _mel_basis[key]


def spectrogram_torch(y, n_fft, sampling_rate, hop_size, win_size, center=False):
    """[B, L] -> [B, n_fft//2+1, frames] magnitude (mel_processing.py:58-77)."""
    if center:
        raise NotImplementedError("the reference always calls center=False")
    pad = int((n_fft - hop_size) / 2)
    # (looked up at call time: a module imported while a test patches
    # ops.stft_mag must not keep the patch after it is undone)
    return ops.stft_mag(y, _window(win_size, y.device), n_fft, hop_size, win_size, pad=pad,
                        eps=1e-6)


def spec_to_mel_torch(spec, n_fft, num_mels, sampling_rate, fmin, fmax):
    basis = _basis(sampling_rate, n_fft, num_mels, fmin, fmax, spec.device).to(spec.dtype)
    return spectral_normalize_torch(torch.matmul(basis, spec))


def mel_spectrogram_torch(y, n_fft, num_mels, sampling_rate, hop_size, win_size, fmin, fmax,
                          center=False):
    spec = spectrogram_torch(y, n_fft, sampling_rate, hop_size, win_size, center)
    basis = _basis(sampling_rate, n_fft, num_mels, fmin, fmax, y.device)
    return spectral_normalize_torch(torch.matmul(basis, spec))
