"""How chaotic the fp16 golden train step's gradients are under different
weight-fill gains of the generator (tests/test_train_step_golden.py _chaotic:
parameters whose torch-fp16-autocast gradient moves by more than cos 0.999
under a one-ulp parameter perturbation).  Prints, per candidate gain set, the
chaotic parameter count of G.  Run on the GPU box:
    python tools/chaos_probe.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import test_train_step_golden as T  # noqa: E402

CANDIDATES = {
    "fill": {},
    "c_stft 0": {"c_stft": 0.0},
}


class _MP:
    def __init__(self):
        self._undo = []

    def setattr(self, obj, name, value):
        self._undo.append((obj, name, getattr(obj, name)))
        setattr(obj, name, value)

    def context(self):
        return self

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        for obj, name, old in reversed(self._undo):
            setattr(obj, name, old)
        self._undo = []
        return False


def main():
    dev = torch.device("cuda:0")
    G, cfg = T._load()
    n_g = len(G["g_keys"])
    orig = T._make_step
    y0 = G["y"].copy()
    for name, gains in CANDIDATES.items():
        G["y"] = y0 * gains.get("y", 1.0)
        cfg["step"]["c_stft"] = gains.get("c_stft", 25.0)
        gains = {k: v for k, v in gains.items() if k not in ("y", "c_stft")}
        def make(cfg_, device, fp16, gains=gains):
            st = orig(cfg_, device, fp16)
            with torch.no_grad():
                for n, p in st.net_g.named_parameters():
                    for (pre, suf), f in gains.items():
                        if n.startswith(pre) and n.endswith(suf):
                            p.mul_(f)
            return st
        T._make_step = make
        try:
            chaotic, _, _ = T._chaotic(G, cfg, dev, _MP())
        except AssertionError as e:  # e.g. the fp16 step overflowed at this gain
            print(f"{name:22s} failed: {e}", flush=True)
            continue
        finally:
            T._make_step = orig
        n_gc = sum(1 for k in chaotic if k.startswith("g."))
        n_dc = sum(1 for k in chaotic if k.startswith("d."))
        print(f"{name:22s} chaotic G {n_gc:4d} / {n_g} ({n_gc / n_g:.2f}), D {n_dc}", flush=True)
        if name in ("fill", "c_stft 0"):
            import collections
            by = collections.Counter(".".join(k.split(".")[1:3]) for k in chaotic)
            tot = collections.Counter(".".join(("g." + str(k)).split(".")[1:3]) for k in G["g_keys"])
            for pre, n in sorted(tot.items()):
                print(f"    {pre:28s} {by.get(pre, 0):4d} / {n}")


if __name__ == "__main__":
    main()
