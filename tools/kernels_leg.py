"""bench.kernels_leg alone (MAS, neg_cent, MR-STFT magnitudes) - for A/B
runs of the training-side kernels."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

print(json.dumps(bench.kernels_leg(torch.device("cuda:0"))), flush=True)
