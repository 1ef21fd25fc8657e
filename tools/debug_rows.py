"""Layer-by-layer check of the row-joined STFT-discriminator path
(train_ops.Conv2dRowsHip16) against torch conv2d on the real MWSD
sub-discriminators (random magnitudes of the train_stft shapes), fp16
autocast.  python tools/debug_rows.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from vits_amd import discriminators as D, train_ops  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)
net = D.MultiWaveSTFTDiscriminator().to(dev)
net._sn.apply(True)
B, L_wave = 2, 9216
for sub, (fft, hop) in zip(net.mfd.discriminators, [(128, 32), (256, 64), (512, 128), (1024, 256),
                                                    (2048, 512)]):
    Fq, T = fft // 2 + 1, L_wave // hop + 1
    m = torch.rand(B, Fq, T, device=dev) * 3
    with torch.autocast("cuda", dtype=torch.float16):
        D.STFT_D_ROWS = True
        a = sub(m)
        D.STFT_D_ROWS = False
        b = sub(m)
        D.STFT_D_ROWS = True
    assert a.shape == b.shape, (a.shape, b.shape)
    err = (a.float() - b.float()).abs().max().item() / b.float().abs().max().item()
    print(f"fft {fft}: out {tuple(a.shape)} vs {tuple(b.shape)} rel err {err:.3e}", flush=True)
    # layer by layer on the torch path's intermediates
    layers = list(sub.convs)
    wdt = train_ops.WDT_F16
    with torch.autocast("cuda", dtype=torch.float16):
        h = D.conv2d_freq(layers[0], m.unsqueeze(1), wdt)
    slope = 1.0
    lp = 2
    R = train_ops.ROW_PAD
    for i, l in enumerate(layers[1:], 1):
        if isinstance(l, torch.nn.LeakyReLU):
            slope = l.negative_slope
            continue
        Fin = h.shape[2]
        L = train_ops.rows_len(T, lp)
        hp = F.pad(h.half(), (lp, L - T - lp, R, R))
        y = train_ops.Conv2dRowsHip16.apply(hp, l.weight, l.bias, l.stride[0], l.padding[1], lp, T,
                                            slope, wdt)
        ref = F.conv2d(F.leaky_relu(h.float(), slope), l.weight.half().float(), l.bias.float(),
                       l.stride, l.padding)
        got = y[:, :, R:R + ref.shape[2], lp:lp + T].float()
        e = (got - ref).abs().max().item() / max(ref.abs().max().item(), 1e-30)
        print(f"   layer {i}: {tuple(h.shape)} -> {tuple(ref.shape)} k={tuple(l.kernel_size)} "
              f"s={tuple(l.stride)} err {e:.3e}", flush=True)
        h = ref.half()
        slope = 1.0
