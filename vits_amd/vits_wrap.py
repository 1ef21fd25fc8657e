"""VITSWrap text-to-speech wrapper (reference ``vits_wrap.py``).

``speaking(dict) -> dict`` keeps the reference contract (vits_wrap.py:168-218):
chunked text -> front-end -> ``EmoVITS.infer`` -> pitch / sampling-rate
resampling -> int16 PCM with a RIFF header, plus segment info, front/back-end
times (ms) and RTF.  The reference's text front-end (``textparser``) is a
private package absent from the reference tree, so it is *pluggable*: pass
any object with ``__call__(utt_id, text) -> (utt_id, segtext, vec[N, c])``,
``max_utt_length`` and ``update()``.  librosa is replaced by
``scipy.signal.resample_poly`` for the resampling steps.
"""
from __future__ import annotations

import struct
import time
from fractions import Fraction

import numpy as np
import torch

from .infer import EmoVITS


def _gen_wav_header(sample_num, sample_rate=8000, bit_num=16):
    """44-byte PCM RIFF header (vits_wrap.py:16-26)."""
    h = b"RIFF" + struct.pack("i", sample_num * 2 + 44 - 8)
    h += b"WAVEfmt \x10\x00\x00\x00\x01\x00\x01\x00"
    h += struct.pack("i", sample_rate) + struct.pack("i", sample_rate * bit_num // 8)
    h += struct.pack("H", bit_num // 8) + struct.pack("H", bit_num)
    h += b"data" + struct.pack("i", sample_num * 2)
    return h


def _resample(wav, orig_sr, target_sr):
    from scipy.signal import resample_poly

    if orig_sr == target_sr:
        return wav
    fr = Fraction(int(target_sr), int(orig_sr)).limit_denominator(1000)
    return resample_poly(wav, fr.numerator, fr.denominator).astype(np.float32)


class VITSWrap(object):
    default_spkid = 1
    default_volume = 1.0
    default_speed = 1.0
    default_pitch = 1.0
    default_tail_silece = 0.0

    def __init__(self, ckpt_path: str = None, device: torch.device = None, loglv: int = 0, *,
                 textparser=None, speecher: EmoVITS = None):
        if textparser is None:
            raise ValueError("VITSWrap needs a text front-end (the reference's private `textparser` "
                             "is not available): pass textparser=...")
        self.loglv = loglv
        self.textparser = textparser
        self.speecher = speecher if speecher is not None else EmoVITS(ckpt_path, device=device)
        self.asv = None  # optional bandwidth extension (fbandext) is not part of the reference tree
        self.default_sampling_rate = self.speecher.sampling_rate
        self.max_utt_length = getattr(self.textparser, "max_utt_length", 256)

    def update(self):
        if hasattr(self.textparser, "update"):
            self.textparser.update()
        self.speecher.update()
        if torch.cuda.is_available():
            torch.cuda.empty_cache()

    def _parse_input(self, inputs):
        volume = max(0.0, min(1.0, float(inputs.get("volume", self.default_volume))))
        speed = max(0.5, min(2.0, float(inputs.get("speed", self.default_speed))))
        pitch = max(0.5, min(2.0, float(inputs.get("pitch", self.default_pitch))))
        sampling_rate = min(48000, max(8000, int(inputs.get("sampling_rate", self.default_sampling_rate))))
        tail_silence = float(inputs.get("tail_silence", self.default_tail_silece))
        speed /= pitch
        utt_id = inputs.get("id", str(time.time()).replace(".", "_"))
        return (inputs, utt_id, inputs.get("text", "。"), int(inputs.get("spkid", self.default_spkid)),
                volume, speed, pitch, sampling_rate, tail_silence, inputs.get("emotion"))

    def _split_utt_text(self, utt_id, utt_text):
        """Split long input at sentence punctuation into chunks of at most
        max_utt_length characters (vits_wrap.py:101-166, simplified: the
        reference's punctuation ranking is front-end specific)."""
        puncs = "。！？；!?;，,、 "
        out_id, out_txt, i = [], [], 0
        while utt_text:
            if len(utt_text) <= self.max_utt_length:
                out_id.append(f"{utt_id}-{i}")
                out_txt.append(utt_text)
                break
            cut = max(utt_text.rfind(p, 0, self.max_utt_length) for p in puncs)
            cut = self.max_utt_length if cut <= 0 else cut + 1
            out_id.append(f"{utt_id}-{i}")
            out_txt.append(utt_text[:cut])
            utt_text = utt_text[cut:]
            i += 1
        return out_id, out_txt

    @torch.no_grad()
    def speaking(self, inputs: dict) -> dict:
        inputs, utt_id, utt_text, spkid, volume, speed, pitch, sampling_rate, tail_silence, emotion = \
            self._parse_input(inputs)
        ids, texts = self._split_utt_text(utt_id, utt_text)
        batch_wav, batch_wavlen = [], 0
        segment_info, start_ms, end_ms = [], 0.0, 0.0
        t_front, t_back = 0.0, 0.0
        for uid, text in zip(ids, texts):
            t0 = time.time()
            uid, segtext, vec = self.textparser(uid, text)
            t1 = time.time()
            t_front += t1 - t0
            wav, emotion = self.speecher.infer(spkid, vec, emotion, duration_rate=speed)
            batch_wavlen += len(wav)
            if pitch != 1.0:
                wav = _resample(wav, int(self.default_sampling_rate / pitch), self.default_sampling_rate)
            if sampling_rate != self.default_sampling_rate:
                wav = _resample(wav, self.default_sampling_rate, sampling_rate)
            wav = np.clip(wav * volume * 32767, -32768, 32767).astype(np.int16)
            if tail_silence > 0:
                wav = np.pad(wav, [0, int(tail_silence * sampling_rate)])
            batch_wav.append(wav)
            t_back += time.time() - t1
            end_ms += len(wav) / sampling_rate * 1000
            segment_info.append({"start_ms": start_ms, "end_ms": end_ms, "input_text": text,
                                 "segtext": segtext.printer() if hasattr(segtext, "printer") else str(segtext)})
            start_ms = end_ms
        rtf = (t_front + t_back) / max(1e-9, batch_wavlen / self.default_sampling_rate)
        pcm = b"".join(w.tobytes() for w in batch_wav)
        out = inputs
        out["wav"] = _gen_wav_header(len(pcm) // 2, sampling_rate, 16) + pcm
        out["sr"] = sampling_rate
        out["segment_info"] = segment_info
        out["time_used_frontend"] = t_front * 1000
        out["time_used_backend"] = t_back * 1000
        out["rtf"] = rtf
        return out
