"""Host-side profile (cProfile) of the train_stft step on one GPU, B=32."""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from vits_amd.train import TrainStep, build_models, default_hps, synthetic_batch  # noqa: E402

dev = torch.device("cuda:0")
hps = default_hps()
torch.manual_seed(1234)
g, d = build_models(hps, dev)
st = TrainStep(hps, g, d, dev)
batch = [t.to(dev) for t in synthetic_batch(hps, 32, seed=0)]
for _ in range(3):
    st.step(batch)
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(3):
    st.step(batch)
torch.cuda.synchronize()
pr.disable()
ps = pstats.Stats(pr).sort_stats("cumulative")
ps.print_stats(45)
ps.sort_stats("tottime").print_stats(30)
