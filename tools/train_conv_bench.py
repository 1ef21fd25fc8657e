"""Per-shape time of one training conv (forward + input grad + weight grad)
on the HIP path (vits_amd.train_ops) vs torch/MIOpen under fp16 autocast,
at the train_stft step's shapes (B=32 utterances, Ty=500 frames, 48-frame
decoder slices, 9216-sample discriminator segments).
    python tools/train_conv_bench.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from vits_amd import train_ops  # noqa: E402

SHAPES = [
    # name, B, cin, cout, k, dil, pad, T, slope
    ("wn_in enc_q", 32, 256, 512, 5, 1, 2, 500, 1.0),
    ("wn_res_skip", 32, 256, 512, 1, 1, 0, 500, 1.0),
    ("rb c1 st1 k11d5", 32, 256, 256, 11, 5, 25, 384, 0.1),
    ("rb c2 st1 k11", 32, 128, 256, 11, 1, 5, 384, 1.0),
    ("rb c1 st4 k7d3", 32, 32, 32, 7, 3, 9, 9216, 0.1),
    ("mwd0 k5d5", 32, 64, 64, 5, 5, 0, 9216, 0.2),
    ("mwd2 k5d5", 32, 128, 128, 5, 5, 0, 2304, 0.2),
    ("mwd4 k5d9", 32, 192, 192, 5, 9, 0, 576, 0.2),
]


def timeit(fn, n=10):
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
    rows = []
    for name, B, cin, cout, k, dil, pad, T, slope in SHAPES:
        x = torch.randn(B, cin, T, device=dev, requires_grad=True)
        w = (torch.randn(cout, cin, k, device=dev) / (cin * k) ** 0.5).requires_grad_(True)
        b = torch.zeros(cout, device=dev, requires_grad=True)
        T_out = T + 2 * pad - (k - 1) * dil
        dy = torch.randn(B, cout, T_out, device=dev)
        flops = 2 * B * cout * cin * k * T_out * 3

        def hip():
            y = train_ops.Conv1dHip.apply(x, w, b, dil, pad, slope, train_ops.TRAIN_WDTYPE)
            y.backward(dy)

        dy16 = dy.half()

        def ref():
            with torch.autocast("cuda", dtype=torch.float16):
                xa = F.leaky_relu(x, slope) if slope != 1.0 else x
                y = F.conv1d(xa, w, b, padding=pad, dilation=dil)
            y.backward(dy16)

        def wg():
            train_ops.wgrad(dy, x.detach(), k, dil, pad, slope)

        def fwd():
            train_ops.Conv1dHip.apply(x.detach(), w.detach(), b.detach(), dil, pad, slope,
                                      train_ops.TRAIN_WDTYPE)

        th = timeit(hip)
        tr = timeit(ref)
        tw = timeit(wg)
        tf = timeit(fwd)
        rows.append(dict(shape=name, hip_ms=round(th, 4), miopen_ms=round(tr, 4),
                         hip_tflops=round(flops / th / 1e9, 1),
                         miopen_tflops=round(flops / tr / 1e9, 1),
                         wgrad_ms=round(tw, 4), wgrad_tflops=round(flops / 3 / tw / 1e9, 1),
                         fwd_ms=round(tf, 4), fwd_tflops=round(flops / 3 / tf / 1e9, 1)))
        print(json.dumps(rows[-1]), flush=True)


if __name__ == "__main__":
    main()
