"""Batching side of the data pipeline (reference ``data_utils.py``).

* ``DistributedBucketSampler`` — the per-rank length-bucketed sharding that
  DDP training relies on (data_utils.py:166-262): buckets by boundaries, pads
  every bucket to a multiple of world*batch by repetition, deterministic
  per-epoch shuffles, rank r takes ids[r::world].
* ``TextAudioSpeakerCollate`` — zero-pad collate sorted by spec length
  (data_utils.py:105-163).
* ``SyntheticTextAudioSpeaker`` — a fixed-shape synthetic dataset for the
  benchmarks (BASELINE configs 3/4: the reference's filelists, wav reading and
  ``.spec.pt`` caches are outside the hot path).
"""
from __future__ import annotations

import torch


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
