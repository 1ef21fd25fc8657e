"""bf16-MFMA path: waveform SNR of a bf16 model vs the fp32 path, and step
time of infer_p2 at B=16/Ty=500 and the C5 long-form shape."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from tests.common import snr_db  # noqa: E402

dev = torch.device("cuda:0")
m32 = bench.build_model(dev)
m16 = bench.build_model(dev).to(torch.bfloat16)
for B, Tx, Ty in [(16, 100, 500), (4, 500, 2500)]:
    inp = bench.make_inputs(B, Tx, Ty, dev)
    with torch.no_grad():
        a = m32.infer_p2(*inp)
        b = m16.infer_p2(*inp)
        torch.cuda.synchronize()
        ts = {}
        for name, m in (("fp32", m32), ("bf16", m16)):
            for _ in range(2):
                m.infer_p2(*inp)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(5):
                m.infer_p2(*inp)
            torch.cuda.synchronize()
            ts[name] = (time.perf_counter() - t0) / 5 * 1e3
    print(f"B={B} Ty={Ty}: out dtype {b.dtype}, SNR bf16 vs fp32 = {snr_db(b.float(), a):.1f} dB, "
          f"fp32 {ts['fp32']:.2f} ms, bf16 {ts['bf16']:.2f} ms", flush=True)
