import os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import torch
from vits_amd import ops
from vits_amd.ops import make_desc, make_out
dev = torch.device("cuda:0")
for (B, T) in [(16, 96000), (64, 24000), (512, 3000), (1, 1536000)]:
    for (cin, cout, k, gate) in [(16, 32, 3, False), (32, 32, 3, True)]:
        x = torch.randn(B, cin, T, device=dev)
        w = torch.randn(cout, cin, k, device=dev) * 0.05
        layer = ops.pack_conv(w, torch.zeros(cout, device=dev), gate=gate)
        y = torch.empty(B, layer.out_channels, T, device=dev)
        res = None if gate else torch.randn(B, cout, T, device=dev)
        cond = torch.randn(B, cout, device=dev) if gate else None
        d = make_desc(layer, x, make_out(y, res=res), in_slope=0.1, cond=cond)
        for _ in range(2): ops.conv1d_launch(d, B, dev)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(5): ops.conv1d_launch(d, B, dev)
        e.record(); torch.cuda.synchronize()
        ms = s.elapsed_time(e) / 5
        fl = 2 * B * T * cout * cin * k
        print(f"B={B:4d} T={T:7d} cin={cin} cout={cout} gate={gate}: {ms*1e3:7.1f} us {fl/ms/1e9:6.1f} TF/s")
