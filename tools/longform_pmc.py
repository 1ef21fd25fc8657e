"""C5 long-form step (bf16 model, B=4, Tx=500, Ty=2500, whole infer_p2 in
one hipGraph) replayed R times - profiled by tools/run_longform_profiles.sh
with R=1 and R=2 (per step = difference), as the train profile."""
import argparse
import os
import sys

import torch

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--replays", type=int, default=1)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    m = bench.build_model(dev).to(torch.bfloat16)
    inputs = bench.make_inputs(4, 500, 2500, dev, seed=4321)
    with torch.no_grad():
        run = m.capture_infer_p2(4, 500, 2500)
        torch.cuda.synchronize()
        print("captured", flush=True)
        for i in range(a.replays):
            run(*inputs)
            torch.cuda.synchronize()
            print("replay", i, flush=True)


if __name__ == "__main__":
    main()
