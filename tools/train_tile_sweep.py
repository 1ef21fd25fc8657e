"""Tile sweep of the 16-bit training conv (forward + input gradient launches,
vits_amd.train_ops.Conv1dHip) on the train_stft step's conv shapes: each
shape timed with every tile of the forward kernel (MI355X).
    python tools/train_tile_sweep.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from vits_amd import train_ops  # noqa: E402
from vits_amd._lib import TILE_128x128, TILE_32x256, TILE_64x128, TILE_64x256  # noqa: E402

SHAPES = [  # name, B, cin, cout, k, dil, pad, T, slope
    ("wn_in", 32, 256, 512, 5, 1, 2, 500, 1.0),
    ("wn_in dgrad", 32, 512, 256, 5, 1, 2, 500, 1.0),
    ("wn_rs", 32, 256, 512, 1, 1, 0, 500, 1.0),
    ("rb1 c1 k3", 32, 256, 256, 3, 1, 1, 384, 0.1),
    ("rb1 c1 k11d5", 32, 256, 256, 11, 5, 25, 384, 0.1),
    ("rb2 c1 k7d3", 32, 128, 128, 7, 3, 9, 2304, 0.1),
    ("rb3 c1 k7", 32, 64, 64, 7, 1, 3, 4608, 0.1),
    ("rb4 c1 k3", 32, 32, 32, 3, 1, 1, 9216, 0.1),
    ("mwd0 k5d5", 32, 64, 64, 5, 5, 0, 9216, 0.2),
    ("mwd2 k5d5", 32, 128, 128, 5, 5, 0, 2304, 0.2),
    ("mwd4 k5d9", 32, 192, 192, 5, 9, 0, 576, 0.2),
    ("ffn1", 32, 256, 1024, 5, 1, 2, 100, 1.0),
]
TILES = {"128x128": TILE_128x128, "64x256": TILE_64x256, "64x128": TILE_64x128,
         "32x256": TILE_32x256}


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


def main():
    dev = torch.device("cuda:0")
    orig = train_ops._pick_tile_bf16
    for name, B, cin, cout, k, dil, pad, T, slope in SHAPES:
        x = torch.randn(B, cin, T, device=dev)
        w = torch.randn(cout, cin, k, device=dev) / (cin * k) ** 0.5
        b = torch.zeros(cout, device=dev)
        n_out = T + 2 * pad - (k - 1) * dil
        flops = 2.0 * B * cout * cin * k * n_out
        row = {"shape": name, "default": None}
        for tname, t in [("default", None)] + list(TILES.items()):
            train_ops._pick_tile_bf16 = orig if t is None else (lambda m, kk, t=t: t)
            try:
                layer = train_ops._pack16(w, False, dil, pad, train_ops.TRAIN_WDTYPE, b)
                us = timeit(lambda: train_ops._run(x, layer, n_out, slope))
                row[tname] = round(flops / us / 1e6, 1)
            except Exception as ex:  # noqa: BLE001
                row[tname] = f"ERR {type(ex).__name__}"
        train_ops._pick_tile_bf16 = orig
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
