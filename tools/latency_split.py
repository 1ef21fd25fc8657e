"""B=1 serving latency split: infer_p1 vs infer_p2 (eager and hipGraph)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda:0")
m = bench.build_model(dev)
g = torch.Generator().manual_seed(11)
x = torch.randn(1, 100, 256, generator=g).to(dev)
emo = torch.randn(1, 1024, generator=g).to(dev)
sid = torch.tensor([1], device=dev)
attn, m_p, s_p, gg, noise = bench.make_inputs(1, 100, 500, dev)


def t(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


with torch.no_grad():
    print("infer_p1 ms", t(lambda: m.infer_p1(x, emo, sid)))
    print("infer_p2 ms", t(lambda: m.infer_p2(attn, m_p, s_p, gg, noise)))
    run = m.capture_infer_p2(1, 100, 500)
    print("infer_p2 graph ms", t(lambda: run(attn, m_p, s_p, gg, noise)))
    for B in (2, 4, 8):
        a2, mp2, sp2, g2, n2 = bench.make_inputs(B, 100, 500, dev)
        print(f"infer_p2 B={B} ms", t(lambda: m.infer_p2(a2, mp2, sp2, g2, n2)))
