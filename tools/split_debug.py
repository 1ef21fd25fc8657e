"""DEBUG: split-fp32 conv vs torch fp32 on small shapes (V4 and scalar staging)."""
import os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import torch
import torch.nn.functional as F
from vits_amd import ops
dev = torch.device("cuda:0")
for (B, cin, cout, k, dil, T) in [(2, 192, 512, 7, 1, 100), (2, 192, 512, 7, 1, 101), (1, 256, 256, 3, 1, 101),
                                  (1, 256, 256, 3, 1, 100), (1, 256, 256, 11, 5, 101), (1, 256, 256, 7, 1, 2000)]:
    g = torch.Generator().manual_seed(1)
    x = torch.randn(B, cin, T, generator=g)
    w = torch.randn(cout, cin, k, generator=g) / (cin * k) ** 0.5
    ref = F.conv1d(x, w, padding=(k - 1) * dil // 2, dilation=dil)
    for wdt in (0, 3):
        with ops.pack_lowp(wdt):
            layer = ops.pack_conv(w.to(dev), None, dilation=dil)
        out = ops.conv1d(x.to(dev), layer).cpu()
        err = (out - ref).abs()
        print(B, cin, cout, k, dil, T, "wdt", wdt, "tile", layer.tile, "nan", int(torch.isnan(out).sum()),
              "maxerr", float(err[~torch.isnan(err)].max()) if (~torch.isnan(err)).any() else None,
              "bad cols", torch.nonzero((err > 1e-3).any(1).any(0)).flatten()[:8].tolist(), flush=True)
