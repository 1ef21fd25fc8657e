"""Per-shape forward time of the 16-bit-activation training conv
(train_ops._run with io16, the Conv1dHip16 forward / data-gradient launch)
at the train_stft step's shapes, plus an exactness check against torch's
fp32 conv on the same fp16 operands (max |err| / max |ref|).
    python tools/conv16_bench.py            (VITS_AMD_LIB selects the library)
Prints one line per shape and "TOTAL x TF/s over y ms" (tools/ab_report.py).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from vits_amd import train_ops  # noqa: E402

SHAPES = [
    # name, B, cin, cout, k, dil, pad, T, slope
    ("wn_in_k5", 32, 256, 512, 5, 1, 2, 500, 1.0),
    ("wn_in_dgrad", 32, 512, 256, 5, 1, 2, 500, 1.0),
    ("wn_rs_1x1", 32, 256, 512, 1, 1, 0, 500, 1.0),
    ("wn_rs_1x1_t", 32, 512, 256, 1, 1, 0, 500, 1.0),
    ("attn_1x1_T100", 32, 256, 256, 1, 1, 0, 100, 1.0),
    ("ffn_k5_T100", 32, 256, 1024, 5, 1, 2, 100, 1.0),
    ("rb_c1_st1_k3", 32, 256, 256, 3, 1, 1, 384, 0.1),
    ("rb_c1_st1_k11d5", 32, 256, 256, 11, 5, 25, 384, 0.1),
    ("rb_c2_st1_k11", 32, 128, 256, 11, 1, 5, 384, 1.0),
    ("rb_c1_st2_k7d3", 32, 128, 128, 7, 3, 9, 2304, 0.1),
    ("rb_c1_st4_k7d3", 32, 32, 32, 7, 3, 9, 9216, 0.1),
    ("mwd0_k5d5", 32, 64, 64, 5, 5, 10, 9216, 0.2),
    ("mwd2_k5d5", 32, 128, 128, 5, 5, 10, 2304, 0.2),
    ("mwd4_k5d9", 32, 192, 192, 5, 9, 18, 576, 0.2),
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
    tot_ms = tot_fl = 0.0
    worst = 0.0
    only = os.environ.get("ONLY")
    for name, B, cin, cout, k, dil, pad, T, slope in SHAPES:
        if only and name not in only.split(","):
            continue
        x = torch.randn(B, cin, T, device=dev).half()
        w = torch.randn(cout, cin, k, device=dev) / (cin * k) ** 0.5
        b = torch.randn(cout, device=dev) * 0.1
        n_out = T + 2 * pad - (k - 1) * dil
        layer = train_ops._pack16(w, False, dil, pad, train_ops.TRAIN_WDTYPE, b, n_out=n_out,
                                  io16=True)
        y = train_ops._run(x, layer, n_out, slope, io16=True)
        xa = F.leaky_relu(x.float(), slope).half().float() if slope != 1.0 else x.float()
        ref = F.conv1d(xa, w.half().float(), b, padding=pad, dilation=dil)
        err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
        worst = max(worst, err)
        ms = timeit(lambda: train_ops._run(x, layer, n_out, slope, io16=True))
        fl = 2.0 * B * cout * cin * k * n_out
        tot_ms += ms
        tot_fl += fl
        print(f"{name:18s} cin={cin} cout={cout} k={k} d={dil} T={T} tile={layer.tile} kc={layer.kc}"
              f"  {ms * 1e3:8.1f} us  err={err:.2e}  {fl / ms / 1e9:7.1f} TF/s", flush=True)
    print(f"TOTAL {tot_fl / tot_ms / 1e9:.1f} TF/s over {tot_ms:.3f} ms  worst_err={worst:.2e}")
    assert worst < 2e-3, worst


if __name__ == "__main__":
    main()
