import sys, os
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R); sys.path.insert(0, os.path.join(R, "tests"))
import torch, torch.nn.functional as F
from common import *
from vits_amd import engine, ops
from vits_amd.ops import make_desc, make_out
dev = torch.device("cuda:0")
m = base_model(dev)
plan = engine.get_plan(m.enc_p, engine.TextEncoderPlan)
torch.manual_seed(0)
x = torch.randn(2, 12, 256, device=dev)
e = torch.empty(2, 256, 12, device=dev)
ops.conv1d_launch(make_desc(plan.emb, x.transpose(1, 2), make_out(e)), 2, dev)
ref = F.linear(x, m.enc_p.emb[0].weight, m.enc_p.emb[0].bias).transpose(1, 2)
print('emb', rel_err(e[0], ref[0]), rel_err(e[1], ref[1]))
emo = torch.randn(2, 1024, device=dev)
ev = ops.linear_rows(emo, plan.emo_w, plan.emo_b)
print('emo', rel_err(ev, F.linear(emo, m.enc_p.emo_proj.weight, m.enc_p.emo_proj.bias)))
h = torch.empty_like(e)
gam, bet, eps = plan.emb_ln
ops.layer_norm_channels(e, gam, bet, eps, out=h, post_add=ev, scale=plan.xscale, pos=plan._pe(12, dev), pos_alpha=plan.alpha.detach().float())
r = F.layer_norm(ref.transpose(1, 2), (256,), gam, bet, eps) + ev[:, None, :]
r = r * plan.xscale + m.enc_p.sin_table[:, :12] * m.enc_p.alpha
r = r.transpose(1, 2)
print('ln', rel_err(h[0], r[0]), rel_err(h[1], r[1]))
qkv = torch.empty(2, 768, 12, device=dev)
ops.conv1d_launch(make_desc(plan.layers[0]["qkv"], h, make_out(qkv)), 2, dev)
a = m.enc_p.encoder.attn_layers[0]
q = F.conv1d(h, a.conv_q.weight, a.conv_q.bias)
print('q', rel_err(qkv[0, :256], q[0]), rel_err(qkv[1, :256], q[1]))
att = torch.empty(2, 256, 12, device=dev)
engine._attention_into(qkv, 256, 2, None, att)
k = F.conv1d(h, a.conv_k.weight, a.conv_k.bias); v = F.conv1d(h, a.conv_v.weight, a.conv_v.bias)
ref_att = a.attention(q, k, v)[0]
print('att', rel_err(att[0], ref_att[0]), rel_err(att[1], ref_att[1]))
