"""Weight-gradient kernel: atomic vs split-K (workspace + reduce) at the
training shapes, over chunks-per-workgroup settings (MI355X).
    python tools/wgrad_split_bench.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from vits_amd import _lib  # noqa: E402
from vits_amd._lib import ConvWgradDesc, check  # noqa: E402
from vits_amd.ops import _stream_ptr  # noqa: E402
from vits_amd.train_ops import TRAIN_WDTYPE  # noqa: E402

SHAPES = [  # name, B, cin, cout, k, dil, pad, T, slope
    ("wn_in enc_q", 32, 256, 512, 5, 1, 2, 500, 1.0),
    ("wn_res_skip", 32, 256, 512, 1, 1, 0, 500, 1.0),
    ("rb c1 st1 k11d5", 32, 256, 256, 11, 5, 25, 384, 0.1),
    ("rb c1 st4 k7d3", 32, 32, 32, 7, 3, 9, 9216, 0.1),
    ("mwd0 k5d5", 32, 64, 64, 5, 5, 0, 9216, 0.2),
    ("mwd2 k5d5", 32, 128, 128, 5, 5, 0, 2304, 0.2),
    ("mwd4 k5d9", 32, 192, 192, 5, 9, 0, 576, 0.2),
    ("mpd p2 l5", 64, 1024, 1024, 5, 1, 2, 57, 1.0),
]


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
    return s.elapsed_time(e) / n * 1e3  # us


def main():
    dev = torch.device("cuda:0")
    lib = _lib.load()
    only = os.environ.get("ONLY")  # one shape name (PMC passes: tools/pmc_wgrad.sh)
    for name, B, cin, cout, k, dil, pad, T, slope in SHAPES:
        if only and name != only:
            continue
        n_out = T + 2 * pad - (k - 1) * dil
        io16 = os.environ.get("IO16", "0") == "1"  # the training step's fp16 activations
        dt = torch.float16 if io16 else torch.float32
        x = torch.randn(B, cin, T, device=dev, dtype=dt)
        dy = torch.randn(B, cout, n_out, device=dev, dtype=dt)
        flops = 2.0 * B * cout * cin * k * n_out

        def desc(dw, db, cpw=0):
            d = ConvWgradDesc()
            d.dy, d.dy_bstride, d.dy_cstride, d.cout = dy.data_ptr(), dy.stride(0), dy.stride(1), cout
            d.x, d.x_bstride, d.x_cstride, d.cin = x.data_ptr(), x.stride(0), x.stride(1), cin
            d.tin, d.n_out, d.k, d.dil, d.pad_left = T, n_out, k, dil, pad
            d.in_slope = slope
            d.dw_t, d.dbias, d.wdtype, d.reserved = dw.data_ptr(), db.data_ptr(), TRAIN_WDTYPE, cpw
            d.io16 = int(io16)
            return d

        dw_t = torch.zeros(k, cout, cin, device=dev)
        db = torch.zeros(cout, device=dev)
        d0 = desc(dw_t, db)

        def atomic():
            dw_t.zero_()
            db.zero_()
            check(lib.vits_conv1d_wgrad(d0, B, _stream_ptr(dev)), "wgrad")

        ref_ms = timeit(atomic)
        ref = dw_t.permute(1, 2, 0).contiguous().clone()
        row = {"shape": name, "atomic_us": round(ref_ms, 1),
               "atomic_tflops": round(flops / ref_ms / 1e6, 1)}
        dw = torch.empty(cout, cin, k, device=dev)
        db2 = torch.empty(cout, device=dev)
        for cpw in (0, 4, 8, 16, 32, 64):
            d = desc(dw, db2, cpw)
            nws = int(lib.vits_conv1d_wgrad_workspace(d, B))
            ws = torch.empty(nws, device=dev)

            def split():
                check(lib.vits_conv1d_wgrad_split(d, B, ws.data_ptr(), nws, _stream_ptr(dev)),
                      "wgrad_split")

            us = timeit(split)
            err = float((dw - ref).abs().max() / ref.abs().max())
            berr = float((db2 - db).abs().max() / db.abs().max())
            row[f"split{cpw}_us"] = round(us, 1)
            row[f"split{cpw}_err"] = float(f"{max(err, berr):.1e}")
            row[f"split{cpw}_wsMB"] = round(nws * 4 / 2**20, 1)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
