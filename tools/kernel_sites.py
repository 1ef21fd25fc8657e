"""Every GPU kernel of one eager train_stft step (B=32, base config, fp16
autocast) attributed to the Python call site or autograd node that launched
it: one torch.profiler run; for each kernel, the launching op's nearest
vits_amd frame (forward) or enclosing autograd node (backward).  Prints
(dispatches, device ms, site, kernel family) sorted by dispatches, and a
per-family total.  Usage: python tools/kernel_sites.py [--batch 32]."""
import argparse
import collections
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vits_amd.train import TrainStep, build_models, default_hps, synthetic_batch  # noqa: E402


def family(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    for key in ("conv1d_mfma_kernel", "wgrad_reduce", "wgrad_kernel", "gate_bwd", "gate_fwd",
                "igemm", "SubTensorOp", "Cijk", "leaky_relu_backward", "leaky_relu",
                "float16_copy", "float16tofloat32", "direct_copy", "CUDAFunctor_add", "MulFunctor",
                "FillFunctor", "fillBuffer", "copyBuffer", "reduce_kernel", "multi_tensor_apply",
                "stft_", "wn_update", "pack16", "wnorm", "sn_", "radam", "mas_kernel",
                "neg_cent", "layer_norm", "softmax", "index", "cat"):
        if key.lower() in n.lower():
            return key
    return n.split("(")[0].split("<")[0][:40]


def site(ev) -> str:
    e = ev
    while e is not None:
        for fr in (e.stack or []):
            if "vits_amd" in fr or "/tools/" in fr:
                return fr.split("/")[-1][:60]
        if e.name.startswith("autograd::engine::evaluate_function:"):
            return "bwd " + e.name.split(":", 4)[-1].strip()[:50]
        e = e.cpu_parent
    return ev.name[:50]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--top", type=int, default=90)
    ap.add_argument("--shapes", action="store_true", help="print the input shapes per site")
    ap.add_argument("--set", action="append", default=[], help="module.CONST=int (A/B)")
    a = ap.parse_args()
    import importlib

    for kv in a.set:
        k, v = kv.split("=")
        mod, attr = k.rsplit(".", 1)
        m = importlib.import_module("vits_amd." + mod)
        setattr(m, attr, type(getattr(m, attr))(int(v)))
    dev = torch.device("cuda:0")
    torch.backends.cudnn.benchmark = True  # as bench.py's train legs (train_stft.py:26)
    hps = default_hps()
    torch.manual_seed(hps.train.seed)
    net_g, net_d = build_models(hps, dev)
    st = TrainStep(hps, net_g, net_d, dev)
    batch = [t.to(dev) for t in synthetic_batch(hps, a.batch, tx=100, ty=500, seed=0)]
    for _ in range(2):
        st.step(batch)
    torch.cuda.synchronize()
    print("warm", flush=True)
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True,
                 record_shapes=True) as prof:
        st.step(batch)
        torch.cuda.synchronize()
    rows = collections.defaultdict(lambda: [0, 0.0])
    fams = collections.defaultdict(lambda: [0, 0.0])
    shapes = collections.defaultdict(collections.Counter)
    for ev in prof.events():
        for k in getattr(ev, "kernels", []) or []:
            f = family(k.name)
            key = (site(ev), f)
            rows[key][0] += 1
            rows[key][1] += k.duration / 1e3
            fams[f][0] += 1
            fams[f][1] += k.duration / 1e3
            if a.shapes:
                shapes[key][str(getattr(ev, "input_shapes", ""))[:90]] += 1
    n = sum(v[0] for v in fams.values())
    ms = sum(v[1] for v in fams.values())
    print(f"kernels in one eager step: {n} dispatches, {ms:.2f} ms device time")
    print("-- by family")
    for f, (c, t) in sorted(fams.items(), key=lambda kv: -kv[1][0]):
        print(f"{c:6d} {t:9.3f} ms  {f}")
    print("-- by site")
    for (s, f), (c, t) in sorted(rows.items(), key=lambda kv: -kv[1][0])[:a.top]:
        print(f"{c:6d} {t:9.3f} ms  {f:22s} {s}")
        if a.shapes:
            for shp, n in shapes[(s, f)].most_common(3):
                print(f"{'':20s} {n:4d} x {shp}")


if __name__ == "__main__":
    main()
