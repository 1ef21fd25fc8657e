"""Per-shape timing of the conv kernel on the decoder / flow shapes of the
bench workload (B=16, Ty=500).  Prints TFLOP/s per shape and overall."""
import os, sys, time, json
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import torch
from vits_amd import ops
from vits_amd.ops import make_desc, make_out

dev = torch.device("cuda:0")
B, Ty = 16, 500
shapes = []  # (name, cin, cout, k, dil, T, gate, upsample(u,K))
for st, (C, T) in enumerate([(256, 8 * Ty), (128, 48 * Ty), (64, 96 * Ty), (32, 192 * Ty)]):
    for k in (3, 7, 11):
        for d in (1, 3, 5):
            shapes.append((f"s{st}.c1.k{k}d{d}", C, C, k, d, T, True, None))
        shapes.append((f"s{st}.c2.k{k}", C // 2, C, k, 1, T, False, None))
shapes.append(("flow.in", 256, 512, 5, 1, Ty, True, None))
shapes.append(("flow.rs", 256, 512, 1, 1, Ty, False, None))
shapes.append(("flow.rsl", 256, 256, 1, 1, Ty, False, None))
shapes.append(("flow.post", 256, 96, 1, 1, Ty, False, None))
shapes.append(("flow.pre", 96, 256, 1, 1, Ty, False, None))
shapes.append(("up0", 512, 256, 16, 1, Ty, False, (8, 16)))
shapes.append(("up1", 256, 128, 12, 1, 8 * Ty, False, (6, 12)))
shapes.append(("pre", 192, 512, 7, 1, Ty, False, None))

only = os.environ.get("ONLY")
BF = os.environ.get("BF", "0") == "1"
WDT = int(os.environ.get("WDT", "1" if BF else "0"))  # 0 f32, 1 bf16, 3 split-f32
CHECK = os.environ.get("CHECK", "0") == "1"  # error vs the exact-f32 kernel and fp64
tiles = [int(t) for t in os.environ.get("TILES", "").split(",") if t]
kcms = [int(t) for t in os.environ.get("KCM", "1").split(",") if t]
reps = int(os.environ.get("REPS", "5"))
if os.environ.get("SPLITW"):  # 0: split fp32 with in-kernel weight splits (F32S)
    ops.SPLIT_W = os.environ["SPLITW"] == "1"
if os.environ.get("F32P_KC"):  # chunk channels of the split-fp32 128-row tiles (32 / 16)
    ops.F32P_MAX_KC = int(os.environ["F32P_KC"])
tot_fl, tot_ms = 0, 0
res = {}
for name, cin, cout, k, d, T, gate, up in shapes:
    if only and only not in name:
        continue
    x = torch.randn(B, cin, T, device=dev)
    if up:
        u, K = up
        w = torch.randn(cin, cout, K, device=dev) * 0.05
        with ops.pack_lowp(WDT):
            layer = ops.pack_conv_transpose(w, torch.zeros(cout, device=dev), u, (K - u) // 2)
        y = torch.empty(B, cout, T * u, device=dev)
        desc = make_desc(layer, x, make_out(y), in_slope=0.1, t_out=T * u)
        flops = 2 * B * cout * T * u * cin * (K // u)
    else:
        w = torch.randn(cout, cin, k, device=dev) * 0.05
        with ops.pack_lowp(WDT):
            layer = ops.pack_conv(w, torch.zeros(cout, device=dev), dilation=d, gate=gate)
        y = torch.empty(B, layer.out_channels, T, device=dev)
        res_t = None if gate else torch.randn(B, cout, T, device=dev)
        cond = torch.randn(B, cout, device=dev) if gate else None
        desc = make_desc(layer, x, make_out(y, res=res_t), in_slope=0.1, cond=cond)
        flops = 2 * B * cout * T * cin * k
    def timeit():
        for _ in range(2):
            ops.conv1d_launch(desc, B, dev)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            ops.conv1d_launch(desc, B, dev)
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / reps

    ms = timeit()
    alt = ""
    if tiles:
        t0, kc0 = desc.tile, desc.kc
        for t in tiles:
            if layer.m_pad % 128 == 0:
                best = None
                for mlt in kcms:
                    kc = kc0 * mlt
                    if layer.cin_pad % kc:
                        continue
                    desc.tile, desc.kc = t, kc
                    try:
                        v = flops / timeit() / 1e9
                    except Exception:  # noqa: BLE001
                        continue
                    if best is None or v > best[0]:
                        best = (v, kc)
                alt += f" t{t}=" + ("ERR" if best is None else f"{best[0]:6.1f}@{best[1]}")
        desc.tile, desc.kc = t0, kc0
    tf = flops / ms / 1e9
    res[name] = round(tf, 1)
    print(f"{name:18s} cin={cin:4d} cout={cout:4d} k={k:2d} d={d} T={T:6d} tile={layer.tile} kc={layer.kc}  {ms*1e3:8.1f} us  {tf:6.1f} TF/s{alt}", flush=True)
    tot_fl += flops
    tot_ms += ms
print(f"TOTAL {tot_fl/tot_ms/1e9:.1f} TF/s over {tot_ms:.2f} ms")
