"""Per-parameter breakdown of the train-step / MWSD golden comparisons on
the GPU (which tensors carry the largest deviations, fp32 and fp16)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import test_mwsd as TM  # noqa: E402
import test_train_step_golden as TG  # noqa: E402


def step_report(fp16, scale=256.0):
    dev = torch.device("cuda:0")
    G, cfg = TG._load()
    st = TG._make_step(cfg, dev, fp16)
    if fp16:
        st.scaler = torch.amp.GradScaler("cuda", init_scale=scale)
    g0 = {k: p.detach().clone() for k, p in st.net_g.named_parameters()}
    with TG._Replay(G):
        out = st.step(TG._batch(G, dev))
    torch.cuda.synchronize()
    print("fp16" if fp16 else "fp32", "scale", float(st.scaler.get_scale()) if fp16 else None)
    params = dict(st.net_g.named_parameters())
    rows = []
    gtot = float(G["grad_norm_g"])
    for k, (gn, gs, dsum, dabs) in zip([str(k) for k in G["g_keys"]], G["g_stats"]):
        p = params[k]
        g = p.grad.detach().double().cpu()
        delta = (p.detach().double() - g0[k].double()).cpu()
        rows.append((k, p.numel(), gn, abs(g.norm().item() - gn) / max(gn, 1e-30),
                     abs(delta.sum().item() - dsum) / max(dabs, 1e-30),
                     abs(delta.sum().item() - dsum)))
    print("worst gnorm rel:")
    for r in sorted([r for r in rows if r[2] > 1e-6 * gtot], key=lambda r: -r[3])[:8]:
        print(f"  {r[0]:60s} n={r[1]:7d} |g|={r[2]:.3e} (x{r[2] / gtot:.1e} of total) rel={r[3]:.2e} upd={r[4]:.2e}")
    print("worst update:")
    for r in sorted(rows, key=lambda r: -r[4])[:5]:
        print(f"  {r[0]:60s} n={r[1]:7d} |g|={r[2]:.3e} rel={r[3]:.2e} upd={r[4]:.2e} abs={r[5]:.2e}")
    tot_u = sum(r[5] for r in rows) / sum(float(s[3]) for s in G["g_stats"])
    print("aggregate update disagreement", tot_u)


def mwsd_report(torch_fp16=False):
    dev = torch.device("cuda:0")
    print("MWSD", "torch-autocast" if torch_fp16 else "HIP")
    G = TM._load()
    d = TM._build(dev)
    outs, lg, gy, gm = TM._run(d, G, dev, autocast=True, loss_scale=1024.0)
    for i, o in enumerate(outs):
        print("out", i, TM._nerr(o.detach().float().cpu().numpy(), G[f"out{i}"]))
    print("grad_y", TM._nerr(gy.cpu(), G["grad_y"]))
    for i, g in enumerate(gm):
        print("grad_mag", i, TM._nerr(g[:, :, :4].float().cpu().numpy(), G[f"grad_mag{i}_head"]),
              g.double().norm().item() / G[f"grad_mag{i}_stats"][0] - 1)
    params = dict(d.named_parameters())
    errs = []
    for k, (gn, gs, _, _) in zip(G["keys"], G["stats"]):
        g = params[str(k)].grad.double().cpu()
        errs.append((abs(g.norm().item() - gn) / gn, str(k)))
    print("worst param grad norms", sorted(errs)[-6:])


class TorchConvs:
    """autocast stays on, but every conv / gate takes torch's path (MIOpen
    fp16): the reference's own fp16 arithmetic on this GPU."""

    def __enter__(self):
        from vits_amd import train_ops
        self.m, self.f = train_ops, train_ops.autocast_wdtype
        train_ops.autocast_wdtype = lambda *a, **k: None
        import vits_amd.discriminators as D
        self.D, self.h = D, D.STFT_D_HIP
        D.STFT_D_HIP = False

    def __exit__(self, *e):
        self.m.autocast_wdtype = self.f
        self.D.STFT_D_HIP = self.h


if __name__ == "__main__":
    step_report(False)
    step_report(True, 1024.0)
    print("=== torch autocast convs (the reference's fp16 arithmetic)")
    with TorchConvs():
        step_report(True, 1024.0)
        mwsd_report(True)
    mwsd_report()
