"""Which side moves in test_generator_fused_weight_norm_matches_torch_hooks
with the fused gate: per-parameter rel. L2 of (fused WN vs hooks) with
train_ops.GATE_FUSED on / off, and the dtype torch._weight_norm returns under
fp16 autocast.   python tools/wn_gate_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch  # noqa: E402

from vits_amd import train_ops, wnorm  # noqa: E402
from test_train import _batch, _make, tiny_hps  # noqa: E402

DEV = torch.device("cuda:0")
with torch.autocast("cuda", dtype=torch.float16):
    v = torch.randn(8, 4, 3, device=DEV, requires_grad=True)
    g = torch.randn(8, 1, 1, device=DEV, requires_grad=True)
    print("torch._weight_norm under autocast ->", torch._weight_norm(v, g, 0).dtype, flush=True)

hps = tiny_hps()
x, x_len, spec, spec_len, _, _, emo, spk = [t.to(DEV) for t in _batch(hps, 4, seed=0)]
st = _make(hps, DEV, seed=0)


def run(fused_wn, gate):
    wnorm.FUSED_WN, train_ops.GATE_FUSED = fused_wn, gate
    st.net_g.zero_grad(set_to_none=True)
    torch.manual_seed(5)
    with st.autocast(), st._g_weights():
        y_hat = st.net_g(x, x_len, spec, spec_len, emo, spk)[0]
    cot = torch.randn(y_hat.shape, device=DEV, generator=torch.Generator(device=DEV).manual_seed(7))
    (y_hat.float() * cot).sum().backward()
    torch.cuda.synchronize()
    return {n: p.grad.detach().double().clone() for n, p in st.net_g.named_parameters()
            if p.grad is not None}


r = {(a, b): run(a, b) for a in (True, False) for b in (True, False)}
wnorm.FUSED_WN, train_ops.GATE_FUSED = True, True


def rel(a, b):
    return float((a - b).norm() / (b.norm() + 1e-30))


names = sorted(r[(True, True)], key=lambda n: -rel(r[(True, True)][n], r[(False, True)][n]))[:6]
for n in names:
    print(f"{n:40s} fusedWN/gate vs hooks/gate {rel(r[(True, True)][n], r[(False, True)][n]):.3e}  "
          f"fusedWN/nogate vs hooks/nogate {rel(r[(True, False)][n], r[(False, False)][n]):.3e}  "
          f"fusedWN gate vs nogate {rel(r[(True, True)][n], r[(True, False)][n]):.3e}  "
          f"hooks gate vs nogate {rel(r[(False, True)][n], r[(False, False)][n]):.3e}", flush=True)
