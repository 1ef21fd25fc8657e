import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch
from common import *
from oracle import vits_oracle as V
from vits_amd import engine
dev = torch.device("cuda:0")
m = base_model(dev)
sd = oracle_sd(m)
gd = golden('base_inference.npz')
t = lambda k: torch.from_numpy(gd[k])
xl = t('x_lengths').long()
g = torch.nn.functional.embedding(t('sid').long(), sd['emb_g.weight'])
h, mm, ll, xm = V.text_encoder(sd, t('x'), t('emo'), g, 6, 2, 192, x_lengths=xl)
logw = V.duration_predictor(sd, h, g, xm)
gd_ = g.to(dev)
H, M, L = m.enc_p.forward_masked_hip(t('x').to(dev), xl.to(dev), t('emo').to(dev), gd_)
print('h', rel_err(H, h), 'm', rel_err(M, mm), 'logs', rel_err(L, ll))
for b in range(2):
    print(' b', b, 'h', rel_err(H[b], h[b]))
LW = engine.get_plan(m.dp, engine.DurationPlan).run(H, gd_, lengths=xl.to(dev).int())
print('logw', rel_err(LW, logw))
print(LW.cpu()[:, 0], logw[:, 0])
# unmasked encoder with full lengths equals masked?
H2, M2, L2 = m.enc_p.forward_masked_hip(t('x').to(dev), torch.tensor([12, 12], device=dev), t('emo').to(dev), gd_)
h2, m2, l2, xm2 = V.text_encoder(sd, t('x'), t('emo'), g, 6, 2, 192, x_lengths=torch.tensor([12, 12]))
print('full-length h', rel_err(H2, h2), 'm', rel_err(M2, m2))
