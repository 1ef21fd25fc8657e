"""infer_p2 (B=16, Tx=100, Ty=500) of a bf16 model, 5 steps — for rocprofv3."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda:0")
m = bench.build_model(dev).to(torch.bfloat16)
inp = bench.make_inputs(16, 100, 500, dev)
with torch.no_grad():
    for _ in range(7):
        m.infer_p2(*inp)
torch.cuda.synchronize()
print("done")
