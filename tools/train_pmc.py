"""Run the captured train_stft step R times (tools/run_train_profiles.sh
profiles this under rocprofv3 twice, with R=1 and R=2, and takes the
difference as the per-step kernel counters, which removes the eager
warm-up and the capture from the count)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--replays", type=int, default=1)
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = True  # as bench.py's train legs (train_stft.py:26)
    from vits_amd.train import TrainStep, build_models, default_hps, synthetic_batch

    dev = torch.device("cuda:0")
    hps = default_hps()
    torch.manual_seed(hps.train.seed)
    g, d = build_models(hps, dev)
    st = TrainStep(hps, g, d, dev, capturable=True)
    batch = [t.to(dev) for t in synthetic_batch(hps, a.batch, seed=0)]
    print("capturing", flush=True)
    st.capture(batch, warmup=1)
    torch.cuda.synchronize()
    for i in range(a.replays):
        out = st.replay()
        torch.cuda.synchronize()
        print("replay", i, flush=True)
    print("replays", a.replays, "loss_gen_all", float(out["loss_gen_all"]), flush=True)


if __name__ == "__main__":
    main()
