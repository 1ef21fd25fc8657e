"""Filelist dataset + ``.spec.pt`` cache (reference data_utils.py:15-102,
mel_processing.py:58-77).

CPU: the loader's filter / seed-1234 shuffle / item layout on a synthetic
filelist (PCM16 wavs, raw float32 vec / emo files, as the reference's
``load_binfn`` / ``load_wav_to_torch`` read them), with caches written in the
reference's format from a torch.stft restatement of ``spectrogram_torch``;
a missing cache raises.  GPU: ``build_spec_cache`` (HIP STFT, batched over
equal-length utterances) against that restatement, and the loader reading
the caches it wrote.  The reference loader itself is not importable here
(soundfile and librosa are absent): parity is against the restated
``spectrogram_torch`` (torch.stft, fp32), tolerance 1e-4 relative to the
spectrum's peak.
"""
import os
import random

import numpy as np
import pytest
import torch

HOP, NFFT, WIN, SR, C = 192, 512, 512, 16000, 8


def _ref_spectrogram(y):
    """mel_processing.py:58-77 restated with torch.stft on the CPU (fp32)."""
    pad = int((NFFT - HOP) / 2)
    y = torch.nn.functional.pad(y.unsqueeze(1), (pad, pad), mode="reflect").squeeze(1)
    spec = torch.stft(y, NFFT, hop_length=HOP, win_length=WIN, window=torch.hann_window(WIN),
                      center=False, normalized=False, onesided=True, return_complex=True)
    return torch.sqrt(spec.real ** 2 + spec.imag ** 2 + 1e-6)


def _hps():
    from vits_amd.utils import get_hparams_from_dict

    return get_hparams_from_dict({
        "train": {"segment_size": 8 * HOP},
        "data": {"sampling_rate": SR, "filter_length": NFFT, "hop_length": HOP,
                 "win_length": WIN, "text_channels": C, "min_wav_len": 0,
                 "max_wav_len": 40 * HOP}})


def _make_filelist(tmp_path, n=7, seed=0):
    from scipy.io import wavfile

    rng = np.random.default_rng(seed)
    lines = []
    for i in range(n):
        # lengths: a few equal ones (one batched STFT launch), one too short
        # for segment_size, one too long for max_wav_len, one 1-token text
        L = [20 * HOP, 20 * HOP, 31 * HOP + 57, 5 * HOP, 45 * HOP, 24 * HOP, 20 * HOP][i % 7]
        ntok = 1 if i == 5 else int(rng.integers(3, 12))
        wav = (rng.standard_normal(L) * 6000).clip(-32768, 32767).astype(np.int16)
        wavfn = str(tmp_path / f"u{i}.wav")
        wavfile.write(wavfn, SR, wav)
        vecfn = str(tmp_path / f"u{i}.vec")
        rng.standard_normal((ntok, C)).astype(np.float32).tofile(vecfn)
        emofn = str(tmp_path / f"u{i}.emo")
        rng.standard_normal(1024).astype(np.float32).tofile(emofn)
        lines.append("|".join([vecfn, wavfn, emofn, str(i % 3)]))
    fl = tmp_path / "filelist.txt"
    fl.write_text("\n".join(lines) + "\n")
    return str(fl), lines


def test_loader_filter_shuffle_and_cache(tmp_path):
    from vits_amd.data_utils import (TextAudioSpeakerCollate, TextAudioSpeakerLoader,
                                     _spec_filename)
    from vits_amd.utils import load_wav_to_torch

    fl, lines = _make_filelist(tmp_path)
    hps = _hps()
    # the reference's filter and shuffle, restated (data_utils.py:35-56)
    keep = []
    for line in lines:
        vecfn, wavfn, emofn, sid = line.split("|")
        ntok = os.path.getsize(vecfn) // (4 * C)
        L = load_wav_to_torch(wavfn)[0].numel()
        if 2 < ntok < 384 and 8 * HOP < L < 40 * HOP:
            keep.append([vecfn, wavfn, emofn, sid])
    expect_lengths = [load_wav_to_torch(w)[0].numel() // HOP for _, w, _, _ in keep]
    random.seed(1234)
    shuffled = list(keep)
    random.shuffle(shuffled)

    # no caches yet: the loader refuses rather than computing on the CPU
    ds = TextAudioSpeakerLoader(fl, hps)
    assert ds.lengths == expect_lengths
    assert ds.filepaths_sid == shuffled
    with pytest.raises(FileNotFoundError, match="build_spec_cache"):
        ds[0]

    # caches in the reference's format: torch.save of the [F, T] tensor
    for _, wavfn, _, _ in keep:
        w = load_wav_to_torch(wavfn)[0]
        torch.save(_ref_spectrogram(w.unsqueeze(0))[0], _spec_filename(wavfn))
    for i in range(len(ds)):
        vec, spec, wav, emo, sid = ds[i]
        vecfn, wavfn, emofn, s = shuffled[i]
        assert vec.shape[1] == C and vec.dtype == torch.float32
        assert spec.shape == (NFFT // 2 + 1, wav.shape[1] // HOP)
        assert wav.shape[0] == 1 and abs(wav.abs().max().item() - 1.0) < 1e-6
        assert emo.shape == (1024,) and sid.tolist() == [int(s)]
    batch = TextAudioSpeakerCollate()([ds[i] for i in range(len(ds))])
    assert batch[2].shape[1] == NFFT // 2 + 1


@pytest.mark.gpu
def test_build_spec_cache_gpu_matches_spectrogram(tmp_path, device):
    from vits_amd.data_utils import TextAudioSpeakerLoader, _spec_filename, build_spec_cache
    from vits_amd.utils import load_filepaths_and_sid, load_wav_to_torch

    fl, _ = _make_filelist(tmp_path, n=7, seed=3)
    hps = _hps()
    n = build_spec_cache(fl, hps, device=device)
    assert n == 7
    assert build_spec_cache(fl, hps, device=device) == 0  # already cached
    for _, wavfn, _, _ in load_filepaths_and_sid(fl):
        got = torch.load(_spec_filename(wavfn), weights_only=True)
        ref = _ref_spectrogram(load_wav_to_torch(wavfn)[0].unsqueeze(0))[0]
        assert got.shape == ref.shape and got.dtype == torch.float32
        err = (got - ref).abs().max().item() / ref.abs().max().item()
        assert err < 1e-4, (wavfn, err)
    ds = TextAudioSpeakerLoader(fl, hps)
    _, spec, wav, _, _ = ds[0]
    assert spec.shape[1] == wav.shape[1] // HOP
    # spec_device= computes a missing cache on the GPU inside the loader
    os.remove(_spec_filename(ds.filepaths_sid[1][1]))
    ds2 = TextAudioSpeakerLoader(fl, hps, spec_device=device)
    spec2 = ds2[1][1]
    ref2 = _ref_spectrogram(load_wav_to_torch(ds.filepaths_sid[1][1])[0].unsqueeze(0))[0]
    assert (spec2 - ref2).abs().max().item() / ref2.abs().max().item() < 1e-4
    assert os.path.exists(_spec_filename(ds.filepaths_sid[1][1]))


def test_wav_header_any_pcm_width(tmp_path):
    """build_spec_cache's header pass (data_utils._wav_header): sample rate
    and sample count for 16-bit / float WAVs and for 24-bit PCM, which
    scipy's memory-mapped read refuses."""
    import struct

    import numpy as np
    from scipy.io import wavfile

    from vits_amd.data_utils import _wav_header

    p = tmp_path / "a.wav"
    wavfile.write(p, 16000, (np.arange(12345) % 300).astype(np.int16))
    assert _wav_header(str(p)) == (16000, 12345)
    p = tmp_path / "b.wav"
    wavfile.write(p, 22050, np.zeros(777, np.float32))
    assert _wav_header(str(p)) == (22050, 777)
    n = 1001
    data = b"".join(struct.pack("<i", i * 100)[:3] for i in range(n)) + b"\0"
    fmt = struct.pack("<HHIIHH", 1, 1, 16000, 16000 * 3, 3, 24)
    riff = (b"RIFF" + struct.pack("<I", 4 + 8 + len(fmt) + 8 + len(data)) + b"WAVE" + b"fmt "
            + struct.pack("<I", len(fmt)) + fmt + b"LIST" + struct.pack("<I", 3) + b"abc\0"
            + b"data" + struct.pack("<I", 3 * n) + data)
    p = tmp_path / "c.wav"
    p.write_bytes(riff)
    assert _wav_header(str(p)) == (16000, n)


def test_wav_header_truncated_or_placeholder_size(tmp_path):
    """A data chunk whose header size is larger than the file (truncated) or
    a streaming placeholder (0 / 0xFFFFFFFF) is counted from the bytes that
    are actually there."""
    import struct

    from vits_amd.data_utils import _wav_header

    fmt = struct.pack("<HHIIHH", 1, 1, 16000, 32000, 2, 16)
    pcm = b"\1\0" * 500
    for declared in (0, 0xFFFFFFFF, 2 * 900):
        riff = (b"RIFF" + struct.pack("<I", 0) + b"WAVE" + b"fmt " + struct.pack("<I", len(fmt))
                + fmt + b"data" + struct.pack("<I", declared) + pcm)
        p = tmp_path / f"t{declared}.wav"
        p.write_bytes(riff)
        assert _wav_header(str(p)) == (16000, 500), declared
