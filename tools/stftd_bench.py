"""Time the 5 STFT discriminators (mrd.py:94-188) fwd+bwd at B=32 train
shapes under fp16 autocast: default (NCHW) vs channels_last input/weights."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from vits_amd.discriminators import MultiWaveSTFTDiscriminator

dev = torch.device("cuda:0")
cl = len(sys.argv) > 1 and sys.argv[1] == "cl"
d = MultiWaveSTFTDiscriminator().to(dev)
mfd = d.mfd
if cl:
    mfd = mfd.to(memory_format=torch.channels_last)
B = 32
Fs = [65, 129, 257, 513, 1025]; Ts = [289, 145, 73, 37, 19]
mags = [torch.rand(B, f, t, device=dev, requires_grad=True) for f, t in zip(Fs, Ts)]
def run():
    d._sn.apply(True)
    with torch.autocast("cuda", dtype=torch.float16):
        outs = []
        for x, sd in zip(mags, mfd.discriminators):
            h = x.unsqueeze(1)
            if cl:
                h = h.contiguous(memory_format=torch.channels_last)
            outs.append(sd.convs(h))
        loss = sum(o.float().mean() for o in outs)
    loss.backward()
for _ in range(3): run()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(10): run()
torch.cuda.synchronize()
print("channels_last" if cl else "nchw", os.environ.get("PYTORCH_MIOPEN_SUGGEST_NHWC"), f"{(time.perf_counter()-t0)/10*1e3:.2f} ms fwd+bwd")
