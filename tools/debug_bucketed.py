"""Where does the padded-text bucketed infer differ from the exact one?"""
import os
import sys

import torch

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "tests"))
from common import base_model  # noqa: E402
from vits_amd import engine  # noqa: E402

dev = torch.device("cuda:0")
m = base_model(dev)
g = torch.Generator().manual_seed(1)
t_x = 60
x = torch.randn(1, t_x, 256, generator=g).to(dev)
emo = torch.randn(1, 1024, generator=g).to(dev)
sid = torch.tensor([5], device=dev)
with torch.no_grad():
    m_p, s_p, logw, gg = m.infer_p1(x, emo, sid)
    xp = torch.zeros(1, 64, 256, device=dev)
    xp[:, :t_x] = x
    xl = torch.tensor([t_x], device=dev, dtype=torch.int32)
    h, m2, s2 = m.enc_p.forward_masked_hip(xp, xl, emo, m.emb_g(sid), exp_logs=True)
    lw2 = engine.get_plan(m.dp, engine.DurationPlan).run(h, m.emb_g(sid), lengths=xl)
    for name, a, b in (("m_p", m_p, m2[:, :, :t_x]), ("s_p", s_p, s2[:, :, :t_x]),
                       ("logw", logw, lw2[:, :, :t_x])):
        d = (a - b).abs().max().item()
        print(name, "equal" if torch.equal(a, b) else f"max diff {d:.3e} rel {d / a.abs().max().item():.3e}")
    # exact-text path vs graph at exact text
    noise = torch.randn(1, 192, 1024, device=dev) * 0.7
    w1, y1 = m.infer_bucketed(x, emo, sid, noise, 1024)
    run = m.capture_infer_bucketed(t_x, 1024)
    w2, y2 = run(x, emo, sid, noise)
    n = int(y1[0]) * 192
    print("graph(exact text) vs eager bucketed:", torch.equal(w1[..., :n], w2[..., :n]), int(y1[0]), int(y2[0]))
    w3, y3 = m.infer_bucketed(xp, emo, sid, noise, 1024, x_lengths=xl)
    print("padded eager vs exact eager:", torch.equal(w1[..., :n], w3[..., :n]), int(y3[0]),
          (w1[..., :n] - w3[..., :n]).abs().max().item())
