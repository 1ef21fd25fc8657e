"""Host-side helpers: config tree, checkpoint I/O, deterministic weight fill.

Mirrors the parts of the reference ``utils.py`` that sit on the inference /
training drivers' call path (``HParams`` ``utils.py:249-278``,
``get_hparams_from_file`` ``utils.py:205-211``, ``load_checkpoint``
``utils.py:19-45``, ``save_checkpoint`` ``utils.py:47-57``,
``latest_checkpoint_path`` ``utils.py:71-78``).  TensorBoard / matplotlib /
soundfile helpers are out of scope.

``deterministic_fill_`` is the key-hashed weight generator used everywhere a
model needs reproducible weights without shipping a checkpoint: the golden
fixture generator applies it to the *reference* model, tests and ``bench.py``
apply it to ours, so both sides hold bit-identical parameters.
"""
from __future__ import annotations

import glob
import json
import os
import zlib

import numpy as np
import torch


# --------------------------------------------------------------------------
# config tree
# --------------------------------------------------------------------------
class HParams:
    """Attribute/dict hybrid over a nested JSON config (``utils.py:249-278``)."""

    def __init__(self, **kwargs):
        for k, v in kwargs.items():
            if isinstance(v, dict):
                v = HParams(**v)
            self[k] = v

    def keys(self):
        return self.__dict__.keys()

    def items(self):
        return self.__dict__.items()

    def values(self):
        return self.__dict__.values()

    def __len__(self):
        return len(self.__dict__)

    def __getitem__(self, key):
        return getattr(self, key)

    def __setitem__(self, key, value):
        return setattr(self, key, value)

    def __contains__(self, key):
        return key in self.__dict__

    def get(self, key, default=None):
        return self.__dict__.get(key, default)

    def __repr__(self):
        return self.__dict__.__repr__()


def get_hparams_from_file(config_path: str) -> HParams:
    with open(config_path, "r") as f:
        config = json.load(f)
    return HParams(**config)


def get_hparams_from_dict(config: dict) -> HParams:
    return HParams(**json.loads(json.dumps(config)))


# --------------------------------------------------------------------------
# checkpoints (format is a drop-in contract: SURVEY.md §8(b))
# --------------------------------------------------------------------------
def latest_checkpoint_path(dir_path: str, regex: str = "G_*.pth"):
    f_list = glob.glob(os.path.join(dir_path, regex))
    if not f_list:
        return None
    f_list.sort(key=lambda f: int("".join(filter(str.isdigit, f)) or 0))
    return f_list[-1]


def _unwrap(model):
    return model.module if hasattr(model, "module") else model


def load_checkpoint(checkpoint_path, model, optimizer=None, adapt=False):
    """Load ``{'model', 'iteration', 'optimizer'}``; missing keys keep the
    current init (``utils.py:33-39``).  ``adapt`` loads weights only."""
    assert os.path.isfile(checkpoint_path), checkpoint_path
    ckpt = torch.load(checkpoint_path, map_location="cpu", weights_only=True)
    iteration = ckpt.get("iteration", 1)
    if optimizer is not None and not adapt and ckpt.get("optimizer") is not None:
        optimizer.load_state_dict(ckpt["optimizer"])
    saved = ckpt["model"]
    target = _unwrap(model)
    state = target.state_dict()
    new_state = {}
    for k, v in state.items():
        if k in saved and saved[k].shape == v.shape:
            new_state[k] = saved[k]
        else:
            new_state[k] = v
    target.load_state_dict(new_state)
    lr = optimizer.param_groups[0]["lr"] if optimizer is not None else None
    return model, optimizer, lr, iteration


def save_checkpoint(model, optimizer, iteration, checkpoint_path):
    torch.save(
        {
            "model": _unwrap(model).state_dict(),
            "iteration": iteration,
            "optimizer": optimizer.state_dict() if optimizer is not None else None,
        },
        checkpoint_path,
    )


# --------------------------------------------------------------------------
# deterministic weights
# --------------------------------------------------------------------------
def _key_rng(key: str, seed: int) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64([zlib.crc32(key.encode()), seed]))


def deterministic_tensor(key: str, shape, seed: int = 1234) -> torch.Tensor:
    """Value for parameter ``key`` of ``shape``; depends only on (key, shape,
    seed).  Scales keep activations O(1) through the residual stacks so that
    parity is checked on non-degenerate data (no tanh saturation, no zeros)."""
    shape = tuple(int(s) for s in shape)
    rng = _key_rng(key, seed)
    leaf = key.rsplit(".", 1)[-1]
    n = int(np.prod(shape)) if shape else 1
    if leaf == "weight_g" and ".ups." in key:
        # ConvTranspose weight-norm is per *input* channel (dim 0 of
        # [in, out, k]); a larger gain keeps the upsampled signal O(0.1).
        a = rng.uniform(1.0, 1.6, size=n)
    elif leaf == "weight_g":
        a = rng.uniform(0.35, 0.75, size=n)
    elif leaf == "weight_v":
        a = rng.standard_normal(n)
    elif leaf in ("gamma",) or (leaf == "weight" and len(shape) == 1):
        a = 1.0 + 0.05 * rng.standard_normal(n)
    elif leaf in ("beta", "bias"):
        a = 0.05 * rng.standard_normal(n)
    elif leaf == "alpha":
        a = 1.0 + 0.05 * rng.standard_normal(n)
    elif key.endswith("emb_g.weight"):
        a = 0.5 * rng.standard_normal(n)
    elif key.endswith("conv_post.weight"):
        a = (1.0 / np.sqrt(float(np.prod(shape[1:])))) * rng.standard_normal(n)
    elif leaf == "weight":
        fan_in = int(np.prod(shape[1:])) if len(shape) > 1 else 1
        a = (0.8 / np.sqrt(max(fan_in, 1))) * rng.standard_normal(n)
    else:
        a = 0.05 * rng.standard_normal(n)
    return torch.from_numpy(a.astype(np.float32).reshape(shape))


@torch.no_grad()
def deterministic_fill_(module: torch.nn.Module, seed: int = 1234) -> torch.nn.Module:
    """Overwrite every parameter (not buffers) of ``module`` by key."""
    for key, p in module.named_parameters():
        p.copy_(deterministic_tensor(key, p.shape, seed).to(p.device, p.dtype))
    return module


def find_files(root_dir, query="*.wav", include_root_dir=True):
    """Recursive glob (reference ``utils.find_files`` ``utils.py:281``)."""
    files = []
    for root, _, filenames in os.walk(root_dir, followlinks=True):
        for filename in filenames:
            import fnmatch

            if fnmatch.fnmatch(filename, query):
                files.append(os.path.join(root, filename))
    if not include_root_dir:
        files = [f.replace(root_dir + "/", "") for f in files]
    return files
