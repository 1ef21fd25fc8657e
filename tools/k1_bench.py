"""1x1 training convs (fp16 activations): the HIP conv (Conv1dHip16) vs a
batched hipBLASLt GEMM (torch.matmul) vs MIOpen (F.conv1d), forward and
forward + backward, at the train_stft step's 1x1 shapes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from vits_amd import train_ops  # noqa: E402

dev = torch.device("cuda:0")
SHAPES = [(32, 256, 512, 500), (32, 512, 256, 500), (32, 256, 256, 500), (32, 256, 256, 100),
          (32, 256, 96, 500), (32, 96, 256, 500)]


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


for B, cin, cout, T in SHAPES:
    x = torch.randn(B, cin, T, device=dev).half().requires_grad_()
    w = (torch.randn(cout, cin, 1, device=dev) / cin ** 0.5).requires_grad_()
    b = torch.zeros(cout, device=dev, requires_grad=True)
    dy = torch.randn(B, cout, T, device=dev).half()

    def hip_f():
        with torch.no_grad():
            return train_ops.Conv1dHip16.apply(x, w, b, 1, 0, 1.0, train_ops.TRAIN_WDTYPE)

    def hip_fb():
        y = train_ops.Conv1dHip16.apply(x, w, b, 1, 0, 1.0, train_ops.TRAIN_WDTYPE)
        y.backward(dy)

    def mm_f():
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16):
            return torch.matmul(w[:, :, 0], x) + b[:, None]

    def mm_fb():
        with torch.autocast("cuda", dtype=torch.float16):
            y = torch.matmul(w[:, :, 0], x) + b[:, None]
        y.backward(dy)

    def mi_f():
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16):
            return F.conv1d(x, w, b)

    def mi_fb():
        with torch.autocast("cuda", dtype=torch.float16):
            y = F.conv1d(x, w, b)
        y.backward(dy)

    r = {n: timeit(f) for n, f in (("hip_f", hip_f), ("mm_f", mm_f), ("mi_f", mi_f),
                                   ("hip_fb", hip_fb), ("mm_fb", mm_fb), ("mi_fb", mi_fb))}
    print(f"B={B} {cin}->{cout} T={T}: " + " ".join(f"{k}={v:7.1f}us" for k, v in r.items()),
          flush=True)
