"""EmoVITS inference wrapper (reference ``infer.py``), on the HIP engine.

Same constructor and ``infer`` contract as ``infer.py:12-184``: speaker-id
mapping files ``*.map``, per-speaker emotion banks ``{spk}.emo`` next to the
checkpoint, an fp16 model (``.half()`` like the reference: its convs run on
the fp16-MFMA kernel variant with fp32 accumulation), a fixed noise
buffer sliced at a random offset per call.  Differences: the noise buffer
lives on the device (no host->device copy per call) and the CLI writes WAVs
with scipy instead of soundfile.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

from . import ops, utils
from .commons import infer_path
from .export import load_model


class EmoVITS(object):
    def __init__(self, checkpoint_path=None, device=None, *, loglv=0, hps=None, model=None,
                 graph_cache=0, graph=True, max_graphs=16):
        """graph: synthesise each utterance as ONE hipGraph replay
        (SynthesizerTrn.capture_infer_bucketed: the durations, the output
        length and the path computed on the device, no host sync before the
        waveform copy), graphs cached per (text bucket, frame bucket), at
        most ``max_graphs``; graph=False: the reference's eager sequence
        (infer_p1 -> host durations -> infer_p2)."""
        self.loglv = loglv
        self.graph_cache = int(graph_cache)
        self._p1_graphs = {}
        self.graph = bool(graph)
        self.max_graphs = int(max_graphs)
        self._graphs = {}
        self._ty_bucket = {}
        if checkpoint_path is None and model is None:
            checkpoint_path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "checkpoint",
                                           "checkpoint.pth")
        self.res_root_path = os.path.dirname(checkpoint_path) if checkpoint_path else "."
        if hps is None:
            hps = utils.get_hparams_from_file(os.path.join(self.res_root_path, "config.json"))
        self.hps = hps
        self.sampling_rate = hps.data["sampling_rate"]
        self.hop_size = hps.data["hop_length"]
        self.text_channels = hps.data["text_channels"]
        self.inter_channels = hps.model["inter_channels"]
        self.num_speaker = hps.data["n_speakers"]
        self.noise_scale = hps.data["noise_scale"]

        self.spkid_mapping, self.spkid_mapping_mtime = {}, {}
        for map_path in utils.find_files(self.res_root_path, "*.map"):
            self._load_spkid_mapping(map_path)
        self.spk_emo_embed, self.spk_emo_embed_mtime = {}, {}
        for emo_path in utils.find_files(self.res_root_path, "*.emo"):
            self._load_spk_emo_embed(int(os.path.splitext(os.path.basename(emo_path))[0]))

        if isinstance(device, str):
            device = torch.device(device)
        self.device = device if device is not None else torch.device("cuda")
        if model is None:
            model = load_model(checkpoint_path, hps)
        model.remove_weight_norm()
        self.model = model.half().eval().to(self.device)
        self.noise = (torch.randn(1 * self.inter_channels * 4096) * self.noise_scale).half().to(self.device)
        self.inference = self.infer
        if self.device.type != "cuda":
            self.graph = False

    # -- speaker / emotion banks (infer.py:77-133) ----------------------------
    def _load_spkid_mapping(self, mapfn):
        if not os.path.exists(mapfn):
            return
        with open(mapfn, "rt") as f:
            for line in f:
                line = line.strip()
                if not line or line[0] == "#":
                    continue
                arr = line.split()
                if len(arr) != 2 or not (arr[0].isdigit() and arr[1].isdigit()):
                    continue
                self.spkid_mapping[int(arr[0])] = int(arr[1])
        self.spkid_mapping_mtime[mapfn] = int(os.stat(mapfn).st_mtime)

    def _load_spk_emo_embed(self, spkid: int):
        emo_path = os.path.join(self.res_root_path, f"{spkid}.emo")
        if os.path.exists(emo_path):
            emb = torch.from_numpy(np.fromfile(emo_path, dtype=np.float32).reshape(-1, 1024)).half()
            self.spk_emo_embed[spkid] = emb
            self.spk_emo_embed_mtime[emo_path] = int(os.stat(emo_path).st_mtime)
            return emb
        return None

    def _get_spk_emo_embed(self, emo: tuple):
        if isinstance(emo[0], (int, np.integer)):
            emb = self.spk_emo_embed.get(int(emo[0]))
            if emb is None:
                emb = self._load_spk_emo_embed(int(emo[0]))
            assert emb is not None, f"no emotion bank for speaker {emo[0]}"
        elif isinstance(emo[0], np.ndarray):
            emb = torch.from_numpy(emo[0].reshape(-1, 1024).astype(np.float32)).half()
        else:
            raise ValueError("emo[0] must be int or ndarray")
        eid = -1 if len(emo) == 1 else int(emo[1])
        if eid < 0 or eid > emb.size(0):
            eid = np.random.randint(0, emb.size(0))
        return emb[eid]

    def update(self):
        for map_path in list(self.spkid_mapping_mtime.keys()):
            if not os.path.exists(map_path):
                self.spkid_mapping_mtime.pop(map_path)
                continue
            if int(os.stat(map_path).st_mtime) != self.spkid_mapping_mtime[map_path]:
                self._load_spkid_mapping(map_path)
        for emo_path in list(self.spk_emo_embed_mtime.keys()):
            if not os.path.exists(emo_path):
                self.spk_emo_embed_mtime.pop(emo_path)
                continue
            if int(os.stat(emo_path).st_mtime) != self.spk_emo_embed_mtime[emo_path]:
                self._load_spk_emo_embed(int(os.path.splitext(os.path.basename(emo_path))[0]))

    # -- synthesis (infer.py:135-184) ------------------------------------------
    @torch.no_grad()
    def _infer_p1(self, text_t, emo, sid):
        """infer_p1, optionally replayed from a per-length hipGraph (captured
        on first use of a token count, at most `graph_cache` lengths kept).
        Off by default: on MI355X the B=1 text side is GPU-bound (3.3 ms
        eager vs 3.3 ms replayed at Tx=100), so capture only adds latency."""
        t_x = text_t.shape[1]
        if self.graph_cache <= 0:
            return self.model.infer_p1(text_t, emo, sid)
        run = self._p1_graphs.pop(t_x, None)
        if run is None:
            run = self.model.capture_infer_p1(t_x)
            while len(self._p1_graphs) >= self.graph_cache:
                self._p1_graphs.pop(next(iter(self._p1_graphs)))
        self._p1_graphs[t_x] = run  # most recently used last
        return tuple(t.clone() for t in run(text_t, emo, sid))

    def infer(self, spkid, text, emo, *, duration_rate=1.0):
        x_length = text.shape[0]
        spkid = self.spkid_mapping.get(spkid, spkid)
        assert spkid < self.num_speaker, f"spkid={spkid} must be less than {self.num_speaker}"
        sid = torch.tensor([spkid], dtype=torch.long, device=self.device)
        if isinstance(emo, torch.Tensor):
            emo = emo.half()
        else:
            if emo is None:
                emo = (spkid, -1)
            if isinstance(emo[0], (int, np.integer)):
                emo = tuple([self.spkid_mapping.get(emo[0], emo[0]) if emo[0] != 0 else spkid,
                             -1 if len(emo) == 1 else emo[1]])
            emo = self._get_spk_emo_embed(emo).unsqueeze(0)
        text_t = torch.from_numpy(np.ascontiguousarray(text)).half().to(self.device).unsqueeze(0)
        emo = emo.to(self.device)

        if self.graph and x_length <= 4096:
            return self._infer_graph(text_t, emo, sid, duration_rate), emo
        m_p, s_p, logw, g = self._infer_p1(text_t, emo, sid)
        w = torch.exp(logw) * duration_rate
        w_ceil = torch.ceil(w)
        y_length = int(torch.clamp_min(torch.sum(w_ceil), 1).item())
        nl = self.inter_channels * y_length
        start = np.random.randint(max(1, self.noise.size(0) - nl))
        noise = self.noise[start:start + nl].view(1, self.inter_channels, y_length)
        attn = infer_path(w_ceil.float(), x_length, y_length).half()
        wav = self.model.infer_p2(attn, m_p, s_p, g, noise)
        return wav.float().view(-1).cpu().numpy(), emo


    # text tokens are padded to a multiple of TX_BUCKET (masked encoder);
    # frame buckets are powers of two from 256 up to the noise buffer's 4096
    TX_BUCKET = 32

    def _infer_graph(self, text_t, emo, sid, duration_rate):
        """One replay of the whole-utterance graph; the one host sync is the
        waveform copy (y_len read with it).  A bucket that turns out too
        small (y_len > frames) is re-run once at a large enough bucket,
        which this text bucket keeps from then on."""
        t_x = text_t.shape[1]
        xb = -(-t_x // self.TX_BUCKET) * self.TX_BUCKET
        while True:
            tyb = self._ty_bucket.get((xb, duration_rate), 256)
            key = (xb, tyb, float(duration_rate))
            run = self._graphs.pop(key, None)
            if run is None:
                while len(self._graphs) >= self.max_graphs:
                    self._graphs.pop(next(iter(self._graphs)))
                run = self.model.capture_infer_bucketed(
                    xb, tyb, noise_len=self.noise.numel(), padded_text=True,
                    length_scale=duration_rate)
                run.static["noise"].copy_(self.noise.float())
            self._graphs[key] = run  # most recently used last
            # infer.py:173's np.random.randint(len - nl), drawn on the device
            # from raw words of numpy's own generator: the same start as the
            # reference, and the generator ends where the reference's does
            pool, state = ops.numpy_draw_pool()
            wav, y_len = run(text_t, emo, sid, noise_start=pool, x_length=t_x)
            n, used = (int(v) for v in y_len[:, 0].tolist())  # (synchronises)
            if n <= tyb and used == -2:
                # every word of the pool was rejected (p < 2^-32): numpy's
                # randint would go on drawing - advance past the pool and
                # replay with the next words of the same stream
                ops.numpy_draw_commit(state, ops.ED_DRAWS)
                continue
            if n <= tyb:
                if used < 0:
                    np.random.set_state(state)
                    raise ValueError(f"utterance of {n} frames does not fit the "
                                     f"{self.noise.numel()}-sample noise buffer")
                ops.numpy_draw_commit(state, used)
                return wav[0, 0, :n * self.hop_size].float().cpu().numpy()
            np.random.set_state(state)  # re-run at a larger bucket: same draw
            if tyb >= 4096:
                raise RuntimeError(f"utterance of {n} frames exceeds the 4096-frame noise buffer")
            self._ty_bucket[(xb, duration_rate)] = min(4096, 1 << (n - 1).bit_length())


def main(argv=None):
    import argparse
    import time

    from scipy.io import wavfile

    ap = argparse.ArgumentParser(description="Decode text vectors with vits_amd (EmoVITS).")
    ap.add_argument("--scpfn", "--scp", required=True)
    ap.add_argument("--spkid", "--sid", default=None, type=int)
    ap.add_argument("--outdir", required=True)
    ap.add_argument("--checkpoint", "--ckpt", default=None)
    ap.add_argument("--device", default=None)
    args = ap.parse_args(argv)
    os.makedirs(args.outdir, exist_ok=True)
    model = EmoVITS(args.checkpoint, args.device, loglv=1)
    total_rtf, n = 0.0, 0
    with open(args.scpfn) as fid:
        for line in fid:
            line = line.strip()
            if not line or line[0] == "#":
                continue
            parts = line.split("|")
            utt_id = os.path.splitext(os.path.basename(parts[0]))[0]
            spkid = int(args.spkid) if args.spkid is not None else (int(parts[-1]) if len(parts) > 1 else 1)
            start = time.time()
            text = np.fromfile(parts[0], dtype=np.float32).reshape(-1, model.text_channels)
            wav, _ = model.infer(spkid, text, None)
            wavfile.write(os.path.join(args.outdir, f"{utt_id}.wav"), model.sampling_rate,
                          np.clip(wav * 32767, -32768, 32767).astype(np.int16))
            total_rtf += (time.time() - start) / (len(wav) / model.sampling_rate)
            n += 1
    sys.stderr.write(f"Finished generation of {n} utterances (RTF = {total_rtf / max(1, n):.03f}).\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
