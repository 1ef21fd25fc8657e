"""Checkpoint loading / greedy-soup export (reference ``export.py``).

``load_model`` keeps the reference contract (export.py:22-61): build
``SynthesizerTrn`` from ``hps`` (``config.json`` beside the checkpoint when
``hps`` is None), load ``G_*.pth`` (or a directory of them, averaging the last
``greedy`` files), return the module.  Checkpoints load with
``torch.load(weights_only=True)``.  TorchScript / ONNX conversion
(export.py:159-226) is out of scope: the HIP plans are the deployment format.
"""
from __future__ import annotations

import argparse
import glob
import logging
import os
import sys

import torch

from . import utils
from .models import SynthesizerTrn


def find_checkpoint_path(dir_path, regex="G_*.pth"):
    f_list = glob.glob(os.path.join(dir_path, regex))
    f_list.sort(key=lambda f: int("".join(filter(str.isdigit, f)) or 0))
    return f_list


def build_generator(hps) -> SynthesizerTrn:
    return SynthesizerTrn(hps.data.text_channels, hps.data.filter_length // 2 + 1,
                          hps.train.segment_size // hps.data.hop_length,
                          n_speakers=hps.data.n_speakers, **hps.model)


def load_model(checkpoint, hps=None, *, greedy=5, is_dis=0):
    if is_dis:
        raise NotImplementedError("discriminators are outside the vits_amd hot path (SURVEY.md §2)")
    if hps is None:
        dirname = checkpoint if os.path.isdir(checkpoint) else os.path.dirname(checkpoint)
        hps = utils.get_hparams_from_file(os.path.join(dirname, "config.json"))
    model = build_generator(hps)
    ckpt_paths = [checkpoint] if not os.path.isdir(checkpoint) else find_checkpoint_path(checkpoint)
    logging.info(f"Load [{ckpt_paths[-1]}]")
    avg = torch.load(ckpt_paths[-1], map_location="cpu", weights_only=True)["model"]
    if greedy > 0 and len(ckpt_paths) > 1:
        n = 1
        for ckpt in ckpt_paths[max(0, len(ckpt_paths) - greedy):-1]:
            logging.info(f"Load [{ckpt}] for averaging.")
            states = torch.load(ckpt, map_location="cpu", weights_only=True)["model"]
            for k in avg.keys():
                avg[k] = avg[k] + states[k]
            n += 1
        for k in avg.keys():
            avg[k] = torch.true_divide(avg[k], n)
    model.load_state_dict(avg)
    return model


def main(argv=None):
    ap = argparse.ArgumentParser(description="Export a vits_amd generator checkpoint (greedy soup).")
    ap.add_argument("--outdir", "-o", required=True)
    ap.add_argument("--checkpoint", "--ckpt", required=True)
    ap.add_argument("--config", "--conf", default=None)
    ap.add_argument("--greedy-soup", "--greedy", default=5, type=int)
    args = ap.parse_args(argv)
    os.makedirs(args.outdir, exist_ok=True)
    if args.config is None:
        d = args.checkpoint if os.path.isdir(args.checkpoint) else os.path.dirname(args.checkpoint)
        args.config = os.path.join(d, "config.json")
    hps = utils.get_hparams_from_file(args.config)
    model = load_model(args.checkpoint, hps, greedy=args.greedy_soup)
    torch.save({"model": model.state_dict()}, os.path.join(args.outdir, "checkpoint.pth"))
    with open(args.config) as fi, open(os.path.join(args.outdir, "config.json"), "w") as fo:
        fo.write(fi.read())
    return 0


if __name__ == "__main__":
    sys.exit(main())
