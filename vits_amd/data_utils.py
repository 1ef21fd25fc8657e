"""Batching side of the data pipeline (reference ``data_utils.py``).

* ``DistributedBucketSampler`` — the per-rank length-bucketed sharding that
  DDP training relies on (data_utils.py:166-262): buckets by boundaries, pads
  every bucket to a multiple of world*batch by repetition, deterministic
  per-epoch shuffles, rank r takes ids[r::world].
* ``TextAudioSpeakerCollate`` — zero-pad collate sorted by spec length
  (data_utils.py:105-163).
* ``TextAudioSpeakerLoader`` — the reference's filelist dataset
  (data_utils.py:15-102): ``vec|wav|emo|sid`` lines, length filter, the
  seed-1234 shuffle, items ``(vec[N,c], spec[F,T], wav[1,L], emo[1024],
  sid[1])`` with the linear spectrogram read from the ``<wav>.spec.pt``
  cache (data_utils.py:73-81).
* ``build_spec_cache`` — the MI355X side of that cache: the reference
  computes a missing spectrogram with ``torch.stft`` inside one of its 8
  forked CPU loader workers and saves it; here the whole filelist's missing
  caches are computed up front in the main process on the GPU (one HIP STFT
  launch per run of equal-length utterances) and written in the reference's
  ``.spec.pt`` format, so the workers only ever load.  A loader worker never
  initialises HIP (a forked child of a HIP process cannot use the device).
* ``SyntheticTextAudioSpeaker`` — a fixed-shape synthetic dataset for the
  benchmarks (BASELINE configs 3/4).
"""
from __future__ import annotations

import os
import random

import torch

from .utils import load_binfn, load_filepaths_and_sid, load_wav_to_torch


def _spec_filename(wavfn: str) -> str:
    return wavfn[:-len(".wav")] + ".spec.pt"


class TextAudioSpeakerLoader(torch.utils.data.Dataset):
    """``data_utils.py:15-102``.  ``spec_device``: when a ``.spec.pt`` cache
    is missing, compute it with the HIP spectrogram on that device and save it
    (for ``num_workers=0`` use); without it a missing cache raises and names
    ``build_spec_cache`` (the reference would fall back to a CPU
    ``torch.stft`` in the worker)."""

    def __init__(self, filepaths_sid, hparams, spec_device=None):
        self.filepaths_sid = load_filepaths_and_sid(filepaths_sid)
        self.sampling_rate = hparams.data.sampling_rate
        self.filter_length = hparams.data.filter_length
        self.hop_length = hparams.data.hop_length
        self.win_length = hparams.data.win_length
        self.text_channels = hparams.data.text_channels
        self.segment_size = hparams.train.segment_size
        self.min_text_len = getattr(hparams.data, "min_text_len", 2)
        self.max_text_len = getattr(hparams.data, "max_text_len", 384)
        self.min_wav_len = max(self.segment_size, getattr(hparams.data, "min_wav_len", 0))
        self.max_wav_len = getattr(hparams.data, "max_wav_len", 10 * self.sampling_rate)
        self.spec_device = spec_device
        self._filter()
        random.seed(1234)
        random.shuffle(self.filepaths_sid)

    def _filter(self):
        """Keep ``min_text_len < N < max_text_len`` and ``min_wav_len < L <
        max_wav_len``; ``lengths`` = L // hop for the bucket sampler
        (data_utils.py:39-56)."""
        kept, lengths = [], []
        for vecfn, wavfn, emofn, sid in self.filepaths_sid:
            vec = load_binfn(vecfn, self.text_channels)
            wav, _ = load_wav_to_torch(wavfn)
            if self.min_text_len < len(vec) < self.max_text_len and \
                    self.min_wav_len < len(wav) < self.max_wav_len:
                kept.append([vecfn, wavfn, emofn, sid])
                lengths.append(len(wav) // self.hop_length)
        self.filepaths_sid = kept
        self.lengths = lengths

    def get_item(self, filepaths_sid):
        vecfn, wavfn, emofn, sid = filepaths_sid
        return (self.get_text(vecfn), *self.get_audio(wavfn), self.get_emo(emofn),
                self.get_sid(sid))

    def get_audio(self, filename):
        audio_norm, sampling_rate = load_wav_to_torch(filename)
        if sampling_rate != self.sampling_rate:
            raise ValueError("{} {} SR doesn't match target {} SR".format(
                filename, sampling_rate, self.sampling_rate))
        assert len(audio_norm) >= self.segment_size
        audio_norm = audio_norm.unsqueeze(0)
        spec_filename = _spec_filename(filename)
        if os.path.exists(spec_filename):
            spec = torch.load(spec_filename, weights_only=True)
        elif self.spec_device is not None:
            spec = _spectrogram(audio_norm, self, self.spec_device)[0]
            torch.save(spec, spec_filename)
        else:
            raise FileNotFoundError(
                f"{spec_filename}: no spectrogram cache; run "
                "vits_amd.data_utils.build_spec_cache(filelist, hps) once before training "
                "(or pass spec_device= for num_workers=0)")
        return spec, audio_norm

    def get_text(self, vecfn):
        return torch.from_numpy(load_binfn(vecfn, self.text_channels))

    def get_emo(self, emofn):
        return torch.from_numpy(load_binfn(emofn, 1024).flatten())

    def get_sid(self, sid):
        return torch.LongTensor([int(sid)])

    def __getitem__(self, index):
        return self.get_item(self.filepaths_sid[index])

    def __len__(self):
        return len(self.filepaths_sid)


def _spectrogram(wavs, hp, device):
    """[n, L] peak-normalised audio -> [n, F, L // hop] on the HIP STFT
    (``mel_processing.spectrogram_torch``), returned on the CPU."""
    from .mel_processing import spectrogram_torch

    y = wavs.to(device=device, dtype=torch.float32)
    spec = spectrogram_torch(y, hp.filter_length, hp.sampling_rate, hp.hop_length,
                             hp.win_length, center=False)
    return spec.cpu()


def _wav_header(fn: str):
    """(sample rate, sample count over all channels) of a RIFF/WAVE file from
    its header alone: the 'fmt ' chunk's rate and bits per sample and the
    'data' chunk's byte size (any PCM width - 24-bit included, which scipy's
    memory-mapped read refuses - and WAVE_FORMAT_EXTENSIBLE).  Files the
    parser does not recognise are read whole by scipy instead."""
    import struct

    try:
        with open(fn, "rb") as f:
            riff = f.read(12)
            if len(riff) == 12 and riff[:4] in (b"RIFF", b"RIFX") and riff[8:12] == b"WAVE":
                en = "<" if riff[:4] == b"RIFF" else ">"
                sr = bits = None
                while True:
                    hdr = f.read(8)
                    if len(hdr) < 8:
                        break
                    cid, size = hdr[:4], struct.unpack(en + "I", hdr[4:])[0]
                    if cid == b"fmt ":
                        fmt = f.read(size + (size & 1))
                        sr = struct.unpack(en + "I", fmt[4:8])[0]
                        bits = struct.unpack(en + "H", fmt[14:16])[0]
                    elif cid == b"data" and sr is not None and bits:
                        # a truncated file, or a streamed one with a
                        # placeholder size (0 / 0xFFFFFFFF): what is there
                        left = os.path.getsize(fn) - f.tell()
                        if size == 0 or size > left:
                            size = left
                        return int(sr), int(size // ((bits + 7) // 8))
                    else:
                        f.seek(size + (size & 1), 1)
    except (OSError, struct.error):
        pass
    from scipy.io import wavfile

    sr, data = wavfile.read(fn)
    return int(sr), int(data.size)


def build_spec_cache(filepaths_sid, hparams, device="cuda", overwrite=False, max_batch=64):
    """Write the ``.spec.pt`` cache of every utterance of a filelist that
    lacks one (``data_utils.py:73-81``), on the GPU.  Utterances of equal
    sample count share one batched HIP STFT launch (up to ``max_batch``).
    Each file holds the ``[F, T]`` float32 tensor the reference's
    ``torch.save(spec, ...)`` writes.  The first pass reads only each WAV's
    header (sample rate, sample count: ``_wav_header``); audio is loaded ``max_batch`` utterances at a time in the
    compute loop, so host memory stays bounded by one batch whatever the
    dataset size.  Returns the number of files written."""

    hp = hparams.data
    todo: dict = {}
    for _vecfn, wavfn, _emofn, _sid in load_filepaths_and_sid(filepaths_sid):
        fn = _spec_filename(wavfn)
        if overwrite or not os.path.exists(fn):
            sr, n = _wav_header(wavfn)
            if sr != hp.sampling_rate:
                raise ValueError("{} {} SR doesn't match target {} SR".format(
                    wavfn, sr, hp.sampling_rate))
            todo.setdefault(n, []).append((fn, wavfn))
    written = 0
    for _n, items in sorted(todo.items()):
        for i in range(0, len(items), max_batch):
            chunk = items[i:i + max_batch]
            loaded = [(fn, load_wav_to_torch(w)[0]) for fn, w in chunk]
            # (a header that disagrees with the samples read: its own batch)
            by_len: dict = {}
            for fn, w in loaded:
                by_len.setdefault(w.numel(), []).append((fn, w))
            del loaded
            for group in by_len.values():
                spec = _spectrogram(torch.stack([w for _, w in group]), hp, device)
                for (fn, _), s in zip(group, spec):
                    torch.save(s.clone(), fn)
                    written += 1
    return written


class DistributedBucketSampler(torch.utils.data.distributed.DistributedSampler):
    def __init__(self, dataset, batch_size, boundaries, num_replicas=None, rank=None, shuffle=True):
        super().__init__(dataset, num_replicas=num_replicas, rank=rank, shuffle=shuffle)
        self.lengths = dataset.lengths
        self.batch_size = batch_size
        self.boundaries = list(boundaries)
        self.buckets, self.num_samples_per_bucket = self._create_buckets()
        self.total_size = sum(self.num_samples_per_bucket)
        self.num_samples = self.total_size // self.num_replicas

    def _bucket_of(self, length):
        for i in range(len(self.boundaries) - 1):
            if self.boundaries[i] < length <= self.boundaries[i + 1]:
                return i
        return -1

    def _create_buckets(self):
        buckets = [[] for _ in range(len(self.boundaries) - 1)]
        for i, length in enumerate(self.lengths):
            b = self._bucket_of(length)
            if b != -1:
                buckets[b].append(i)
        for i in range(len(buckets) - 1, 0, -1):
            if not buckets[i]:
                buckets.pop(i)
                self.boundaries.pop(i + 1)
        total = self.num_replicas * self.batch_size
        per_bucket = [len(b) + (total - len(b) % total) % total for b in buckets]
        return buckets, per_bucket

    def __iter__(self):
        g = torch.Generator()
        g.manual_seed(self.epoch)
        if self.shuffle:
            orders = [torch.randperm(len(b), generator=g).tolist() for b in self.buckets]
        else:
            orders = [list(range(len(b))) for b in self.buckets]
        batches = []
        for bucket, ids, n_target in zip(self.buckets, orders, self.num_samples_per_bucket):
            rem = n_target - len(bucket)
            ids = ids + ids * (rem // len(bucket)) + ids[:rem % len(bucket)]
            ids = ids[self.rank::self.num_replicas]
            for j in range(len(ids) // self.batch_size):
                batches.append([bucket[i] for i in ids[j * self.batch_size:(j + 1) * self.batch_size]])
        if self.shuffle:
            order = torch.randperm(len(batches), generator=g).tolist()
            batches = [batches[i] for i in order]
        self.batches = batches
        assert len(self.batches) * self.batch_size == self.num_samples
        return iter(self.batches)

    def __len__(self):
        return self.num_samples // self.batch_size


class TextAudioSpeakerCollate:
    """Items are (text[N,c], spec[F,T], wav[1,L], emo[1024], sid)."""

    def __init__(self, return_ids=False):
        self.return_ids = return_ids

    def __call__(self, batch):
        _, order = torch.sort(torch.LongTensor([x[1].size(1) for x in batch]), dim=0, descending=True)
        B = len(batch)
        mt = max(len(x[0]) for x in batch)
        ms = max(x[1].size(1) for x in batch)
        mw = max(x[2].size(1) for x in batch)
        text = torch.zeros(B, mt, batch[0][0].size(1))
        spec = torch.zeros(B, batch[0][1].size(0), ms)
        wav = torch.zeros(B, 1, mw)
        emo = torch.zeros(B, 1024)
        sid = torch.zeros(B, dtype=torch.long)
        tl = torch.zeros(B, dtype=torch.long)
        sl = torch.zeros(B, dtype=torch.long)
        wl = torch.zeros(B, dtype=torch.long)
        for i, k in enumerate(order.tolist()):
            t, s, w, e, spk = batch[k]
            text[i, :t.size(0)] = t
            tl[i] = t.size(0)
            spec[i, :, :s.size(1)] = s
            sl[i] = s.size(1)
            wav[i, :, :w.size(1)] = w
            wl[i] = w.size(1)
            emo[i] = e
            sid[i] = int(spk)
        out = (text, tl, spec, sl, wav, wl, emo, sid)
        return out + (order,) if self.return_ids else out


class SyntheticTextAudioSpeaker(torch.utils.data.Dataset):
    """Fixed-shape synthetic utterances: text
    vectors randn(Tx, c), spec rand(F, Ty), wav clip(randn*0.1), emo randn,
    speaker id = index % n_speakers."""

    def __init__(self, n, tx=100, ty=500, text_channels=256, spec_channels=513, hop=192,
                 n_speakers=2048, seed=1234, ty_min=None):
        self.n, self.tx, self.ty, self.c, self.f, self.hop = n, tx, ty, text_channels, spec_channels, hop
        self.n_speakers, self.seed = n_speakers, seed
        g = torch.Generator().manual_seed(seed)
        lo = ty if ty_min is None else ty_min
        self.ty_per = torch.randint(lo, ty + 1, (n,), generator=g).tolist()
        self.lengths = [t * hop for t in self.ty_per]

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed + 7919 * i)
        ty = self.ty_per[i]
        tx = max(1, min(self.tx, ty))
        text = torch.randn(tx, self.c, generator=g)
        spec = torch.rand(self.f, ty, generator=g)
        wav = (torch.randn(1, ty * self.hop, generator=g) * 0.1).clamp(-1, 1)
        emo = torch.randn(1024, generator=g)
        return text, spec, wav, emo, i % self.n_speakers
