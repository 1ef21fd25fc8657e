"""Is the HIP training step run-to-run deterministic, and if not, where does
it first diverge?  ("run two HIP steps in one process,
diff the gradients layer by layer, and name the nondeterministic kernel".)

Runs the golden train step (tests/golden/train_step.npz, fp16 autocast) N
times from identical parameters / inputs / recorded draws and records, per
run: every module output's checksum in forward order, the gradient flowing
into every module output in backward order, and every parameter gradient.
Prints the first forward / backward record and the parameters that differ
between run 0 and each later run.  MODE=torch runs the same step on torch's
autocast convs (the reference's arithmetic) for comparison; DET=1 turns on
torch.use_deterministic_algorithms(warn_only) and prints which torch ops
warn (it also makes MIOpen pick deterministic solvers).

    python tools/determinism.py [runs]
"""
import os
import sys
import warnings

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import tests.test_train_step_golden as T  # noqa: E402
from vits_amd import discriminators, train_ops  # noqa: E402

dev = torch.device("cuda:0")
MODE = os.environ.get("MODE", "hip")
FP16 = os.environ.get("FP16", "1") != "0"


def _ck(t):
    t = t.detach()
    if not t.is_floating_point():
        t = t.float()
    t = t.double()
    w = torch.arange(1, t.numel() + 1, device=t.device, dtype=torch.float64).view(t.shape)
    return (float(t.abs().sum()), float((t * w).sum()))


def one_run(G, cfg):
    torch.manual_seed(0)
    st = T._make_step(cfg, dev, FP16)
    fwd, bwd = [], []
    hooks = []
    for pre, net in (("g.", st.net_g), ("d.", st.net_d)):
        for name, m in net.named_modules():
            if not name:
                continue

            def fh(mod, inp, out, name=pre + name):
                outs = out if isinstance(out, (tuple, list)) else (out,)
                for i, o in enumerate(outs):
                    if isinstance(o, torch.Tensor) and o.is_floating_point():
                        fwd.append((f"{name}[{i}]", _ck(o)))
                        if o.requires_grad:
                            o.register_hook(lambda g, n=f"{name}[{i}]": bwd.append((n, _ck(g))))

            hooks.append(m.register_forward_hook(fh))
    with T._Replay(G):
        st.step(T._batch(G, dev))
    torch.cuda.synchronize()
    for h in hooks:
        h.remove()
    grads = {k: v.clone() for k, v in T._grads(st).items()}
    return fwd, bwd, grads


def first_diff(a, b, what):
    for i, ((na, ca), (nb, cb)) in enumerate(zip(a, b)):
        if na != nb:
            print(f"  {what}: record {i} names differ ({na} vs {nb})")
            return
        if ca != cb:
            print(f"  {what}: first difference at record {i}/{len(a)}: {na}  {ca} vs {cb}")
            for j in range(max(0, i - 3), i):
                print(f"      (identical before: {a[j][0]})")
            return
    print(f"  {what}: all {len(a)} records bit-identical")


def main():
    runs = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    G, cfg = T._load()
    if MODE == "torch":
        train_ops.HIP_TRAIN = False
        discriminators.STFT_D_HIP = False
    if os.environ.get("DET") == "1":
        torch.use_deterministic_algorithms(True, warn_only=True)
        warnings.simplefilter("always")
    res = []
    with warnings.catch_warnings(record=True) as wl:
        warnings.simplefilter("always")
        for r in range(runs):
            res.append(one_run(G, cfg))
    seen = set()
    for w in wl:
        msg = str(w.message).split("\n")[0][:200]
        if "nondeterministic" in msg.lower() or "deterministic" in msg.lower():
            if msg not in seen:
                seen.add(msg)
                print("  torch warns:", msg)
    print(f"mode={MODE} fp16={FP16}: {runs} runs", flush=True)
    f0, b0, g0 = res[0]
    for r in range(1, runs):
        f, b, g = res[r]
        print(f"run 0 vs run {r}:")
        first_diff(f0, f, "forward")
        first_diff(b0, b, "backward")
        diff = [k for k in g0 if not torch.equal(g0[k], g[k])]
        print(f"  parameter gradients differing: {len(diff)} of {len(g0)}")
        for k in diff[:25]:
            d = float((g0[k] - g[k]).norm() / max(float(g0[k].norm()), 1e-30))
            print(f"     {k:60s} rel {d:.2e}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
