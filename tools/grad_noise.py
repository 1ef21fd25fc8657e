"""How noisy is each parameter's fp16 gradient in the golden train step?
torch16 vs torch16 with every parameter scaled by (1 +- 2^-11), and HIP16 vs
torch16, at several GradScaler scales (underflow of small fp16 gradients
is one candidate source of the noise).  python tools/grad_noise.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import tests.test_train_step_golden as T  # noqa: E402
from vits_amd import discriminators, train_ops  # noqa: E402

dev = torch.device("cuda:0")
G, cfg = T._load()
orig = T._make_step


def run(scale, hip, perturb=0.0):
    def mk(cfg_, device, fp16):
        st = orig(cfg_, device, fp16)
        st.scaler = torch.amp.GradScaler("cuda", init_scale=scale)
        return st

    T._make_step = mk
    aw, sd = train_ops.HIP_TRAIN, discriminators.STFT_D_HIP
    if not hip:
        train_ops.HIP_TRAIN = False
        discriminators.STFT_D_HIP = False
    try:
        st = T._make_step(cfg, dev, True)
        if perturb:
            gen = torch.Generator().manual_seed(123)
            with torch.no_grad():
                for net in (st.net_g, st.net_d):
                    for p in net.parameters():
                        sgn = torch.randint(0, 2, p.shape, generator=gen).to(p) * 2 - 1
                        p.mul_(1 + perturb * sgn)
        with T._Replay(G):
            st.step(T._batch(G, dev))
        torch.cuda.synchronize()
        ok = float(st.scaler.get_scale()) == scale
        return T._grads(st), ok
    finally:
        train_ops.HIP_TRAIN, discriminators.STFT_D_HIP = aw, sd
        T._make_step = orig


# (larger GradScaler scales overflow on this step: 1024 only)
scale = 1024.0
t16, ok1 = run(scale, False)
tp, ok2 = run(scale, False, 2.0 ** -11)
pp = T.grad_agreement(tp, t16, t16)
for variant in ("default", "GATE_FUSED=0"):
    saved = train_ops.GATE_FUSED
    if variant == "GATE_FUSED=0":
        train_ops.GATE_FUSED = False
    h16, ok3 = run(scale, True)
    train_ops.GATE_FUSED = saved
    ht = T.grad_agreement(h16, t16, t16)
    print(f"--- HIP {variant}", flush=True)
    cp = np.array([pp[k][0] for k in pp])
    ch = np.array([ht[k][0] for k in pp])
    print(f"scale {scale}: {len(pp)} params; stable(cos>=0.999) t16' {int((cp >= 0.999).sum())} "
          f"HIP {int((ch >= 0.999).sum())}; cos<0.9: t16' {int((cp < 0.9).sum())} "
          f"HIP {int((ch < 0.9).sum())}", flush=True)
    worst = sorted(pp, key=lambda k: 1 - ht[k][0])[-12:]
    for k in worst:
        print(f"   {k:50s} cos(HIP,t16) {ht[k][0]:.4f} r {ht[k][1]:.3f}  cos(t16',t16) "
              f"{pp[k][0]:.4f} r {pp[k][1]:.3f}", flush=True)
