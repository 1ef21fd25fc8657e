"""DEBUG: split-fp32 conv error per MFMA term subset (desc.reserved mask)."""
import os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import torch
import torch.nn.functional as F
from vits_amd import ops
from vits_amd.ops import make_desc, make_out
dev = torch.device("cuda:0")
torch.manual_seed(0)
C, k, d, T = 64, 3, 1, 256
def bf(t):
    return t.to(torch.bfloat16).to(torch.float64)
for label, x, w in [
    ("bf16-exact inputs", bf(torch.randn(1, C, T, dtype=torch.float64)), bf(torch.randn(C, C, k, dtype=torch.float64) / 14)),
    ("x bf16, w fp32", bf(torch.randn(1, C, T, dtype=torch.float64)), torch.randn(C, C, k, dtype=torch.float64).float().double() / 14),
    ("x fp32, w bf16", torch.randn(1, C, T).double(), bf(torch.randn(C, C, k, dtype=torch.float64) / 14)),
    ("fp32 both", torch.randn(1, C, T).double(), torch.randn(C, C, k).double() / 14),
]:
    ref = F.conv1d(x, w, padding=(k - 1) * d // 2, dilation=d)
    rms = ref.pow(2).mean().sqrt().item()
    with ops.pack_lowp(3):
        layer = ops.pack_conv(w.float().to(dev), None, dilation=d)
    out = []
    for mask in (0, 32, 32 | 8 | 16, 32 | 8 | 16 | 4, 1 | 2, 4, 8, 16):
        y = torch.empty(1, C, T, device=dev)
        desc = make_desc(layer, x.float().to(dev), make_out(y))
        desc.reserved = mask
        ops.conv1d_launch(desc, 1, dev)
        e = (y.double().cpu() - ref).pow(2).mean().sqrt().item() / rms
        out.append(f"m{mask}:{e:.2e}")
    print(label, " ".join(out), flush=True)
