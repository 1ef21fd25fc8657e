"""Time one 16-bit-activation training conv forward (io16, the fp16 autocast
train step's Conv1dHip16 launch) at a given shape over K-chunk sizes and
tiles, to see what bounds it.  python tools/conv16_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from vits_amd import train_ops  # noqa: E402
from vits_amd._lib import TILE_64x128, TILE_64x256, TILE_128x128, WDT_F16  # noqa: E402

SHAPES = [  # B, cin, cout, k, dil, pad, T
    (32, 256, 512, 1, 1, 0, 500),
    (32, 256, 512, 5, 1, 2, 500),
    (32, 512, 256, 5, 1, 2, 500),
    (32, 96, 96, 5, 5, 0, 4552),
    (32, 128, 128, 11, 3, 15, 2304),
]


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    shapes = SHAPES
    one = "--one" in sys.argv  # "--one i": shape i at its default tile / kc only
    if one:
        shapes = [SHAPES[int(sys.argv[sys.argv.index("--one") + 1])]]
    for B, cin, cout, k, dil, pad, T in shapes:
        x = torch.randn(B, cin, T, device=dev).half()
        w = torch.randn(cout, cin, k, device=dev) / (cin * k) ** 0.5
        b = torch.randn(cout, device=dev)
        n_out = T + 2 * pad - (k - 1) * dil
        fl = 2 * B * cout * cin * k * n_out
        layer, _ = train_ops._pack16_pair(w, dil, pad, WDT_F16, b, n_out, T, io16=True)
        if "--torch" in sys.argv:
            w16, b16 = w.half(), b.half()
            ms = timeit(lambda: torch.nn.functional.conv1d(x, w16, b16, padding=pad, dilation=dil))
            print(f"  MIOpen conv1d fp16: {ms * 1e3:8.1f} us  {fl / ms / 1e9:7.1f} TF/s", flush=True)
            if k == 1:
                w2 = w16[:, :, 0]
                ms = timeit(lambda: torch.matmul(w2, x))
                print(f"  matmul W@X (batched): {ms * 1e3:8.1f} us  {fl / ms / 1e9:7.1f} TF/s",
                      flush=True)
                xt = x.transpose(0, 1).reshape(cin, B * T)
                ms = timeit(lambda: torch.matmul(w2, xt))
                print(f"  matmul W@X (one GEMM, [C][B*T]): {ms * 1e3:8.1f} us  "
                      f"{fl / ms / 1e9:7.1f} TF/s", flush=True)
            continue
        print(f"shape B{B} cin{cin} cout{cout} k{k} d{dil} T{T}: default tile {layer.tile} "
              f"kc {layer.kc}", flush=True)
        if one:
            ms = timeit(lambda: train_ops._run(x, layer, n_out, io16=True))
            print(f"  {ms * 1e3:8.1f} us  {fl / ms / 1e9:7.1f} TF/s", flush=True)
            continue
        for tile in (TILE_128x128, TILE_64x128, TILE_64x256):
            for kc in (16, 32, 48, 64):
                if layer.cin_pad % kc:
                    continue
                layer.tile, layer.kc = tile, kc
                try:
                    ms = timeit(lambda: train_ops._run(x, layer, n_out, io16=True))
                except Exception as ex:  # noqa: BLE001 - unsupported combination
                    print(f"  tile {tile} kc {kc}: {type(ex).__name__}", flush=True)
                    continue
                print(f"  tile {tile} kc {kc:3d}: {ms * 1e3:8.1f} us  {fl / ms / 1e9:7.1f} TF/s",
                      flush=True)


if __name__ == "__main__":
    main()
