"""Host-side helpers: config tree, checkpoint I/O, deterministic weight fill.

Mirrors the parts of the reference ``utils.py`` that sit on the inference /
training drivers' call path (``HParams`` ``utils.py:249-278``,
``get_hparams_from_file`` ``utils.py:205-211``, ``load_checkpoint``
``utils.py:19-45``, ``save_checkpoint`` ``utils.py:47-57``,
``latest_checkpoint_path`` ``utils.py:71-78``, ``get_hparams``
``utils.py:152-191``, ``get_logger`` ``utils.py:234-246``, ``summarize``
``utils.py:60-68``, ``plot_*`` ``utils.py:81-133``), same signatures and
return values, so ``from vits_amd import utils`` serves the reference's
``train*.py`` unpacking patterns.

``deterministic_fill_`` is the key-hashed weight generator used everywhere a
model needs reproducible weights without shipping a checkpoint: the golden
fixture generator applies it to the *reference* model, tests and ``bench.py``
apply it to ours, so both sides hold bit-identical parameters.
"""
from __future__ import annotations

import argparse
import glob
import json
import logging
import os
import subprocess
import zlib

import numpy as np
import torch

logger = logging.getLogger("vits_amd")


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


def load_checkpoint(checkpoint_path, model, optimizer=None, *, adapt=False):
    """Same contract as the reference (``utils.py:19-45``): returns
    ``(model, optimizer, iteration)``; ``adapt`` loads weights only and
    reports iteration 1; a key missing from the checkpoint keeps the current
    init (``utils.py:33-39``); the load is strict otherwise (a shape mismatch
    raises, as ``load_state_dict(strict=True)`` does in the reference).
    Unlike the reference the file is read with ``weights_only=True``."""
    assert os.path.isfile(checkpoint_path), checkpoint_path
    ckpt = torch.load(checkpoint_path, map_location="cpu", weights_only=True)
    if "iteration" in ckpt and not adapt:
        iteration = ckpt["iteration"]
    else:
        iteration = 1
    if "optimizer" in ckpt and ckpt["optimizer"] is not None and optimizer is not None \
            and not adapt:
        optimizer.load_state_dict(ckpt["optimizer"])
    saved = ckpt["model"]
    target = _unwrap(model)
    new_state = {}
    for k, v in target.state_dict().items():
        if k in saved:
            new_state[k] = saved[k]
        else:
            logger.info("%s is not in the checkpoint", k)
            new_state[k] = v
    target.load_state_dict(new_state, strict=True)
    logger.info("Loaded checkpoint '%s' (iteration %s)", checkpoint_path, iteration)
    return model, optimizer, iteration


def portable_optimizer_state(optimizer):
    """``optimizer.state_dict()`` with every param group's ``lr`` /
    ``initial_lr`` as a Python float: a graph-capturable TrainStep keeps its
    learning rates as device tensors, which the reference's optimizers cannot
    consume (radam.py:92 passes ``-step_size * group['lr']`` as a number;
    torch's foreach AdamW rejects a tensor lr without capturable)."""
    sd = optimizer.state_dict()
    for g in sd["param_groups"]:
        for k in ("lr", "initial_lr"):
            if isinstance(g.get(k), torch.Tensor):
                g[k] = float(g[k])
    return sd


def pin_optimizer_state(optimizer):
    """Make ``optimizer.load_state_dict`` write IN PLACE into the tensors a
    captured hipGraph reads: a tensor ``lr`` / ``initial_lr`` keeps its object
    (the loaded value is copied into it) and existing state tensors (moments,
    device step counters) receive the loaded values instead of being
    replaced.  Without this a resumed run (load_checkpoint, then capture or
    an earlier capture replayed) would bake the checkpoint's float lr into
    the graph or update orphaned moments."""
    snap = {}

    def pre(opt, state_dict):
        snap["lr"] = [(g.get("lr"), g.get("initial_lr")) for g in opt.param_groups]
        snap["state"] = {p: dict(st) for p, st in opt.state.items()}
        return None

    def post(opt):
        for g, (lr, ilr) in zip(opt.param_groups, snap.get("lr", [])):
            for k, prev in (("lr", lr), ("initial_lr", ilr)):
                if isinstance(prev, torch.Tensor) and k in g and g[k] is not prev:
                    prev.fill_(float(g[k]))
                    g[k] = prev
        for p, st in opt.state.items():
            old = snap.get("state", {}).get(p, {})
            for k, new in list(st.items()):
                prev = old.get(k)
                if isinstance(prev, torch.Tensor) and prev is not new:
                    if isinstance(new, torch.Tensor) and new.numel() == prev.numel():
                        prev.copy_(new.reshape(prev.shape))
                        st[k] = prev
                    elif not isinstance(new, torch.Tensor) and prev.numel() == 1:
                        prev.fill_(float(new))
                        st[k] = prev
        snap.clear()

    optimizer.register_load_state_dict_pre_hook(pre)
    optimizer.register_load_state_dict_post_hook(post)
    return optimizer


def save_checkpoint(model, optimizer, iteration, checkpoint_path):
    """``utils.py:47-57``: ``{'model', 'iteration', 'optimizer'}`` (learning
    rates stored as floats, ``portable_optimizer_state``)."""
    logger.info("Saving model and optimizer state at iteration %s to %s",
                iteration, checkpoint_path)
    torch.save(
        {
            "model": _unwrap(model).state_dict(),
            "iteration": iteration,
            "optimizer": portable_optimizer_state(optimizer) if optimizer is not None else None,
        },
        checkpoint_path,
    )


# --------------------------------------------------------------------------
# CLI / logging / file helpers the training drivers call
# --------------------------------------------------------------------------
def get_hparams(init=True, argv=None) -> HParams:
    """``utils.py:152-191``: ``-c -m -a -d --ckptG --ckptD``; copies the
    config to ``./logs/<model>/config.json`` (``init``) or reads it back."""
    parser = argparse.ArgumentParser()
    parser.add_argument("-c", "--config", type=str, default="./configs/base.json",
                        help="JSON file for configuration")
    parser.add_argument("-m", "--model", type=str, required=True, help="Model name")
    parser.add_argument("-a", "--adapt", action="store_true",
                        help="Adaptative training or not, default=False.")
    parser.add_argument("-d", "--use-dur-dis", action="store_true",
                        help="Use duration discriminator or not, default=False.")
    parser.add_argument("--ckptG", type=str, required=False,
                        help="original VITS G checkpoint path")
    parser.add_argument("--ckptD", type=str, required=False,
                        help="original VITS D checkpoint path")
    args = parser.parse_args(argv)
    model_dir = os.path.join("./logs", args.model)
    os.makedirs(model_dir, exist_ok=True)
    config_save_path = os.path.join(model_dir, "config.json")
    if init:
        with open(args.config, "r") as f:
            data = f.read()
        with open(config_save_path, "w") as f:
            f.write(data)
    else:
        with open(config_save_path, "r") as f:
            data = f.read()
    hparams = HParams(**json.loads(data))
    hparams.model_dir = model_dir
    hparams.adapt = args.adapt
    hparams.use_dur_dis = args.use_dur_dis
    hparams.ckptG = args.ckptG
    hparams.ckptD = args.ckptD
    return hparams


def get_hparams_from_dir(model_dir) -> HParams:
    """``utils.py:194-202``."""
    with open(os.path.join(model_dir, "config.json"), "r") as f:
        hparams = HParams(**json.load(f))
    hparams.model_dir = model_dir
    return hparams


def get_logger(model_dir, filename="train.log"):
    """``utils.py:234-246``: file logger ``<model_dir>/<filename>``; also
    becomes this module's logger, as in the reference."""
    global logger
    logger = logging.getLogger(os.path.basename(model_dir))
    logger.setLevel(logging.DEBUG)
    formatter = logging.Formatter("%(asctime)s\t%(name)s\t%(levelname)s\t%(message)s")
    os.makedirs(model_dir, exist_ok=True)
    h = logging.FileHandler(os.path.join(model_dir, filename))
    h.setLevel(logging.DEBUG)
    h.setFormatter(formatter)
    logger.addHandler(h)
    return logger


def check_git_hash(model_dir):
    """``utils.py:214-231``: record / compare the source tree's git hash."""
    source_dir = os.path.dirname(os.path.dirname(os.path.realpath(__file__)))
    if not os.path.exists(os.path.join(source_dir, ".git")):
        logger.warning("%s is not a git repository, therefore hash value comparison "
                       "will be ignored.", source_dir)
        return
    cur_hash = subprocess.getoutput(f"git -C {source_dir} rev-parse HEAD")
    path = os.path.join(model_dir, "githash")
    if os.path.exists(path):
        with open(path) as f:
            saved_hash = f.read()
        if saved_hash != cur_hash:
            logger.warning("git hash values are different. %s(saved) != %s(current)",
                           saved_hash[:8], cur_hash[:8])
    else:
        with open(path, "w") as f:
            f.write(cur_hash)


def summarize(writer, global_step, scalars={}, histograms={}, images={}, audios={},
              audio_sampling_rate=22050):
    """``utils.py:60-68`` over any TensorBoard-``SummaryWriter``-like object."""
    for k, v in scalars.items():
        writer.add_scalar(k, v, global_step)
    for k, v in histograms.items():
        writer.add_histogram(k, v, global_step)
    for k, v in images.items():
        writer.add_image(k, v, global_step, dataformats="HWC")
    for k, v in audios.items():
        writer.add_audio(k, v, global_step, audio_sampling_rate)


def _figure_to_numpy(fig):
    # the reference's ``np.fromstring(fig.canvas.tostring_rgb())`` is gone from
    # current matplotlib/numpy; buffer_rgba gives the same HxWx3 image
    fig.canvas.draw()
    data = np.asarray(fig.canvas.buffer_rgba())[..., :3].copy()
    return data


def plot_spectrogram_to_numpy(spectrogram):
    """``utils.py:81-104``."""
    import matplotlib

    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    fig, ax = plt.subplots(figsize=(10, 2))
    im = ax.imshow(spectrogram, aspect="auto", origin="lower", interpolation="none")
    plt.colorbar(im, ax=ax)
    plt.xlabel("Frames")
    plt.ylabel("Channels")
    plt.tight_layout()
    data = _figure_to_numpy(fig)
    plt.close(fig)
    return data


def plot_alignment_to_numpy(alignment, info=None):
    """``utils.py:107-133``."""
    import matplotlib

    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    fig, ax = plt.subplots(figsize=(6, 4))
    im = ax.imshow(alignment.transpose(), aspect="auto", origin="lower",
                   interpolation="none")
    fig.colorbar(im, ax=ax)
    xlabel = "Decoder timestep"
    if info is not None:
        xlabel += "\n\n" + info
    plt.xlabel(xlabel)
    plt.ylabel("Encoder timestep")
    plt.tight_layout()
    data = _figure_to_numpy(fig)
    plt.close(fig)
    return data


def load_wav_to_torch(full_path):
    """``utils.py:136-139``: float32 samples peak-normalised to 1.  soundfile is
    absent from this image, so PCM / float WAV is read with scipy."""
    from scipy.io import wavfile

    sr, x = wavfile.read(full_path)
    if x.dtype.kind == "i":
        x = x.astype(np.float32) / float(np.iinfo(x.dtype).max + 1)
    elif x.dtype.kind == "u":
        x = (x.astype(np.float32) - 128.0) / 128.0
    x = x.astype(np.float32)
    x /= np.abs(x).max()
    return torch.from_numpy(x), sr


def load_filepaths_and_sid(filename, split="|"):
    """``utils.py:142-145``."""
    with open(filename, encoding="utf-8") as f:
        return [line.strip().split(split) for line in f]


def load_binfn(filename, dim):
    """``utils.py:148-149``: raw float32 text vectors ``[N, dim]``."""
    return np.fromfile(filename, dtype=np.float32).reshape(-1, dim)


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


@torch.no_grad()
def deterministic_fill_sn_(module: torch.nn.Module, seed: int = 1234) -> torch.nn.Module:
    """Overwrite the spectral-norm power-iteration buffers (``*_u`` / ``*_v``
    beside a ``*_orig`` parameter, torch.nn.utils.spectral_norm) by key with
    unit vectors, so a reference module and this one start their power
    iterations from the same state (mrd.py's D, train_stft.py:86)."""
    params = dict(module.named_parameters())
    for key, b in module.named_buffers():
        stem, _, leaf = key.rpartition("_")
        if leaf in ("u", "v") and stem + "_orig" in params:
            t = deterministic_tensor(key, b.shape, seed).double()
            b.copy_((t / t.norm().clamp_min(1e-12)).to(b.device, b.dtype))
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
