"""Which part of the train step breaks hipGraph capture?  usage: debug_graph_parts.py PART
PART: gfwd | gbwd | dfwdbwd | optg | full"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from vits_amd import commons
from vits_amd.train import TrainStep, build_models, default_hps, synthetic_batch

part = sys.argv[1]
B = 8
dev = torch.device("cuda:0")
hps = default_hps()
torch.manual_seed(1234)
g, d = build_models(hps, dev)
st = TrainStep(hps, g, d, dev, capturable=True)
batch = [t.to(dev) for t in synthetic_batch(hps, B, seed=0)]
g.__dict__["_device_slice_rng"] = True
g.__dict__["_align_noise_t"] = torch.tensor(0.01, device=dev)
x, x_lengths, spec, spec_lengths, y, y_lengths, emo, speakers = batch

def f_gfwd():
    with st.autocast():
        out = g(x, x_lengths, spec, spec_lengths, emo, speakers)
    return out[0]

def f_gbwd():
    with st.autocast():
        out = g(x, x_lengths, spec, spec_lengths, emo, speakers)
        yy = commons.slice_segments(y, out[3] * 192, 9216)
        sc, mag, ym, yhm = st.mstft(yy.squeeze(1), out[0].squeeze(1))
        loss = (sc + mag) * 25 + out[1].float().sum()
    st.scaler.scale(loss).backward()
    return loss.detach()

def f_dfwdbwd():
    yy = y[:, :, :9216].contiguous()
    with st.autocast():
        sc, mag, ym, yhm = st.mstft(yy.squeeze(1), yy.squeeze(1) * 0.5)
        outs = d(yy, ym)
        loss = sum(o.float().mean() for o in outs)
    st.scaler.scale(loss).backward()
    return loss.detach()

def f_optg():
    l = f_gbwd()
    st.scaler.unscale_(st.optim_g)
    st.scaler.step(st.optim_g)
    st.scaler.update()
    return l

def f_optd():
    l = f_dfwdbwd()
    st.scaler.unscale_(st.optim_d)
    gn = commons.clip_grad_value_(d.parameters(), None, as_tensor=True)
    st._step_d_sync_free()
    st.scaler.update()
    return l + 0 * gn

def f_mels():
    from vits_amd.mel_processing import mel_spectrogram_torch, spec_to_mel_torch
    h = hps.data
    with st.autocast():
        mel = spec_to_mel_torch(spec[:1].float(), h.filter_length, h.n_mel_channels, h.sampling_rate,
                                h.mel_fmin, h.mel_fmax)
        m2 = mel_spectrogram_torch(y[:1, 0, :9216].float(), h.filter_length, h.n_mel_channels,
                                   h.sampling_rate, h.hop_length, h.win_length, h.mel_fmin, h.mel_fmax)
    return mel.mean() + m2.mean()

def f_clip():
    l = f_gbwd()
    return commons.clip_grad_value_(g.parameters(), None, as_tensor=True) + 0 * l

fn = {"optd": f_optd, "mels": f_mels, "clip": f_clip, "gfwd": f_gfwd, "gbwd": f_gbwd, "dfwdbwd": f_dfwdbwd, "optg": f_optg,
      "full": lambda: st.step(batch)["loss_gen_all"]}[part]
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(2):
        r = fn()
        st.optim_g.zero_grad(set_to_none=True); st.optim_d.zero_grad(set_to_none=True)
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
print(part, "eager", float(r.float().mean()), flush=True)
gr = torch.cuda.CUDAGraph()
with torch.cuda.graph(gr):
    r = fn()
print(part, "captured", flush=True)
gr.replay(); torch.cuda.synchronize()
print(part, "replay", float(r.float().mean()), flush=True)
