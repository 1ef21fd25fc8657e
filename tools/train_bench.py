"""Time the train_stft step (BASELINE C3/C4) on one GPU: base.json shapes,
synthetic batch Tx=100 / Ty=500, fp16 autocast.  Usage:
    python tools/train_bench.py --batch 32 --steps 5 --warmup 2
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from vits_amd.train import TrainStep, build_models, default_hps, synthetic_batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-mels", action="store_true")
    ap.add_argument("--no-fused", action="store_true")
    ap.add_argument("--torch-prof", default=None, help="write a torch.profiler op table here")
    ap.add_argument("--graph", action="store_true", help="capture the step into a hipGraph")
    ap.add_argument("--cudnn-benchmark", action="store_true",
                    help="torch.backends.cudnn.benchmark = True (train_stft.py:26)")
    ap.add_argument("--variant", choices=["stft", "mel"], default="stft")
    ap.add_argument("--set", action="append", default=[],
                    help="module.CONST=int for an in-process A/B, e.g. discriminators.STFT_D_FUSED=0")
    args = ap.parse_args()
    import importlib

    for kv in args.set:
        k, v = kv.split("=")
        mod, attr = k.rsplit(".", 1)
        setattr(importlib.import_module("vits_amd." + mod), attr, type(getattr(
            importlib.import_module("vits_amd." + mod), attr))(int(v)))
    dev = torch.device("cuda:0")
    torch.backends.cudnn.benchmark = args.cudnn_benchmark
    hps = default_hps()
    torch.manual_seed(1234)
    g, d = build_models(hps, dev, args.variant)
    st = TrainStep(hps, g, d, dev, log_mels=not args.no_mels, fused_adamw=not args.no_fused,
                   capturable=args.graph, variant=args.variant)
    batch = [t.to(dev) for t in synthetic_batch(hps, args.batch, seed=0)]
    if args.graph:
        t0 = time.perf_counter()
        st.capture(batch)
        torch.cuda.synchronize()
        print(f"capture: {time.perf_counter() - t0:.3f}s", flush=True)
    step = (lambda b: st.replay()) if args.graph else st.step
    for i in range(args.warmup):
        t0 = time.perf_counter()
        step(batch)
        torch.cuda.synchronize()
        print(f"warmup {i}: {time.perf_counter() - t0:.3f}s", flush=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step(batch)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    if args.torch_prof:
        from torch.profiler import ProfilerActivity, profile

        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
            st.step(batch)  # eager, so ops and step: phases are attributed
            torch.cuda.synchronize()
        ka = prof.key_averages()
        with open(args.torch_prof, "w") as f:
            f.write(ka.table(sort_by="self_cuda_time_total", row_limit=60, max_name_column_width=90))
            f.write("\n\n")
            f.write(ka.table(sort_by="cuda_time_total", row_limit=60, max_name_column_width=90))
            f.write("\n\n")
            phases = [e for e in ka if e.key.startswith("step:")]
            for e in sorted(phases, key=lambda e: -e.device_time_total):
                f.write(f"{e.key:32s} device {e.device_time_total / 1e3:8.2f} ms  cpu {e.cpu_time_total / 1e3:8.2f} ms\n")
    print(json.dumps({"set": args.set, "variant": args.variant, "batch": args.batch, "s_per_step": dt, "utt_per_s": args.batch / dt,
                      "loss_g": float(out["loss_gen_all"]), "loss_d": float(out["loss_disc"]),
                      "max_mem_gb": torch.cuda.max_memory_allocated() / 2**30}), flush=True)


if __name__ == "__main__":
    main()
