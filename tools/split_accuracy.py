"""Error of the split-fp32 conv (VITS_WDT_F32S: fp32 operands as three exact
bf16 terms, six bf16 MFMAs) next to the exact-fp32 conv (f32-input MFMA),
both against an fp64 CPU convolution, on the decoder's conv shapes at one
utterance x 2048 steps.  Prints rms and max error relative to the output's
rms for each kernel."""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from vits_amd import ops  # noqa: E402
from vits_amd.ops import make_desc, make_out  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)
T = int(os.environ.get("T", "2048"))
worst = {0: 0.0, 3: 0.0}
for C in (256, 128, 64, 32):
    for k, d in ((3, 1), (3, 5), (7, 3), (11, 5), (11, 1)):
        x = torch.randn(1, C, T, dtype=torch.float64)
        w = torch.randn(C, C, k, dtype=torch.float64) / (C * k) ** 0.5
        ref = F.conv1d(x, w, padding=(k - 1) * d // 2, dilation=d)
        rms = ref.pow(2).mean().sqrt().item()
        line = f"C={C:3d} k={k:2d} d={d}"
        for wdt in (0, 3):
            with ops.pack_lowp(wdt):
                layer = ops.pack_conv(w.float().to(dev), None, dilation=d)
            y = torch.empty(1, C, T, device=dev)
            ops.conv1d_launch(make_desc(layer, x.float().to(dev), make_out(y)), 1, dev)
            err = (y.double().cpu() - ref)
            e_rms = err.pow(2).mean().sqrt().item() / rms
            e_max = err.abs().max().item() / rms
            worst[wdt] = max(worst[wdt], e_rms)
            line += f"  {'f32 ' if wdt == 0 else 'f32s'}: rms {e_rms:.2e} max {e_max:.2e}"
        print(line, flush=True)
print(f"worst rms error / output rms: exact f32 {worst[0]:.2e}, split f32 {worst[3]:.2e}")
