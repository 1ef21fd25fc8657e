"""Debug the captured train step: eager capturable steps, then capture and replays, printing losses."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from vits_amd.train import TrainStep, build_models, default_hps, synthetic_batch

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
dev = torch.device("cuda:0")
hps = default_hps()
torch.manual_seed(1234)
g, d = build_models(hps, dev)
st = TrainStep(hps, g, d, dev, capturable=True)
batch = [t.to(dev) for t in synthetic_batch(hps, B, seed=0)]
def show(tag, out):
    print(tag, {k: round(float(v), 4) for k, v in out.items()}, "scale", float(st.scaler.get_scale()), flush=True)
for i in range(3):
    show(f"eager{i}", st.step(batch))
out = st.capture(batch, warmup=1)
torch.cuda.synchronize()
show("captured", out)
for i in range(4):
    show(f"replay{i}", st.replay())
p = next(g.parameters())
print("param finite", bool(torch.isfinite(p).all()))
