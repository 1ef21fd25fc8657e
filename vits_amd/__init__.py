"""vits_amd — MI355X (gfx950) native VITS forward/inference hot path.

Drop-in for the reference's SynthesizerTrn / monotonic_align / STFT-loss
surface; the hot kernels live in libvits_amd.so (vits_amd/csrc, C-ABI in
include/vits_amd.h).
"""
__version__ = "0.1.0"
