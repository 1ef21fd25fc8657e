"""Kernel-level parity of libvits_amd against CPU fp32 references.

Floating-point ops are compared against torch CPU fp32 (the same library the
reference runs on) with tolerances stated per test; MAS is compared bit-exactly
against the C oracle (oracle/mas_oracle.c)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from vits_amd import ops

pytestmark = pytest.mark.gpu

RTOL = 1e-4  # fp32 MFMA vs CPU fp32: different summation order only


def _close(a, b, tol=RTOL, what=""):
    a = a.detach().float().cpu()
    b = b.detach().float().cpu()
    assert a.shape == b.shape, (what, a.shape, b.shape)
    scale = b.abs().max().item() + 1e-12
    err = (a - b).abs().max().item()
    assert err <= tol * scale, f"{what}: max err {err:.3e} vs scale {scale:.3e}"


@pytest.mark.parametrize("B,cin,cout,k,dil,T", [
    (1, 16, 32, 3, 1, 50), (2, 192, 512, 7, 1, 101), (3, 256, 256, 11, 5, 300),
    (2, 64, 64, 7, 3, 1000), (2, 16, 32, 11, 1, 777), (1, 513, 256, 1, 1, 64),
    (2, 256, 96, 1, 1, 130), (1, 96, 256, 1, 1, 33), (2, 32, 32, 3, 5, 2000),
])
@pytest.mark.parametrize("wdt", [ops.WDT_F32, ops.WDT_F32S])
def test_conv1d_store(device, B, cin, cout, k, dil, T, wdt):
    g = torch.Generator().manual_seed(B * 1000 + cin + k)
    x = torch.randn(B, cin, T, generator=g)
    w = torch.randn(cout, cin, k, generator=g) / (cin * k) ** 0.5
    b = torch.randn(cout, generator=g) * 0.1
    pad = (k * dil - dil) // 2
    ref = F.conv1d(F.leaky_relu(x, 0.1), w, b, padding=pad, dilation=dil)
    res = torch.randn(B, cout, T, generator=g)
    ref = ref + res
    with ops.pack_lowp(wdt):
        layer = ops.pack_conv(w.to(device), b.to(device), dilation=dil)
    out = ops.conv1d(x.to(device), layer, in_slope=0.1, residual=res.to(device))
    _close(out, ref, what="conv1d")


@pytest.mark.parametrize("B,C,k,dil,T", [(2, 256, 3, 1, 200), (1, 32, 11, 5, 900), (2, 128, 7, 3, 333)])
@pytest.mark.parametrize("wdt", [ops.WDT_F32, ops.WDT_F32S])
def test_conv1d_gate_cond(device, B, C, k, dil, T, wdt):
    g = torch.Generator().manual_seed(7 + C)
    x = torch.randn(B, C, T, generator=g)
    w = torch.randn(C, C, k, generator=g) / (C * k) ** 0.5
    b = torch.randn(C, generator=g) * 0.1
    cond = torch.randn(B, C, generator=g)
    pad = (k * dil - dil) // 2
    xt = F.conv1d(F.leaky_relu(x, 0.1), w, b, padding=pad, dilation=dil)
    xa, xb = xt.chunk(2, 1)
    sa, sb = cond.chunk(2, 1)
    ref = torch.tanh(xa + sa.unsqueeze(-1)) * torch.sigmoid(xb + sb.unsqueeze(-1))
    with ops.pack_lowp(wdt):
        layer = ops.pack_conv(w.to(device), b.to(device), dilation=dil, gate=True)
    out = ops.conv1d(x.to(device), layer, in_slope=0.1, cond=cond.to(device))
    _close(out, ref, what="gate")


@pytest.mark.parametrize("B,cin,cout,K,u,T", [(1, 512, 256, 16, 8, 40), (2, 256, 128, 12, 6, 37),
                                             (2, 128, 64, 4, 2, 301), (1, 64, 32, 4, 2, 1000)])
@pytest.mark.parametrize("wdt", [ops.WDT_F32, ops.WDT_F32S])
def test_conv_transpose_polyphase(device, B, cin, cout, K, u, T, wdt):
    g = torch.Generator().manual_seed(K + cin)
    x = torch.randn(B, cin, T, generator=g)
    w = torch.randn(cin, cout, K, generator=g) / (cin * 2) ** 0.5
    b = torch.randn(cout, generator=g) * 0.1
    pad = (K - u) // 2
    ref = F.conv_transpose1d(F.leaky_relu(x, 0.1), w, b, stride=u, padding=pad)
    with ops.pack_lowp(wdt):
        layer = ops.pack_conv_transpose(w.to(device), b.to(device), u, pad)
    out = ops.conv1d(x.to(device), layer, in_slope=0.1)
    _close(out, ref, what="convT")


@pytest.mark.parametrize("C,k,dil,T", [(256, 3, 1, 1024), (128, 7, 3, 999), (256, 11, 5, 640),
                                       (512, 5, 1, 200)])
def test_conv1d_split_f32_matches_exact_f32_error(device, C, k, dil, T):
    """Split fp32 (VITS_WDT_F32S: three exact bf16 terms, six bf16 MFMAs)
    against an fp64 convolution: its rms / max error must stay at the level
    of the exact-fp32 kernel's (v_mfma_f32_32x32x2_f32) - within 1.5x - on
    the decoder's shapes.  Measured on MI355X: split 2.9e-7..8.4e-7 rms vs
    exact 3.4e-7..9.5e-7 (tools/split_accuracy.py)."""
    g = torch.Generator().manual_seed(C + k)
    x = torch.randn(2, C, T, generator=g, dtype=torch.float64)
    w = torch.randn(C, C, k, generator=g, dtype=torch.float64) / (C * k) ** 0.5
    ref = F.conv1d(x, w, padding=(k - 1) * dil // 2, dilation=dil)
    rms = ref.pow(2).mean().sqrt().item()
    errs = {}
    for wdt in (ops.WDT_F32, ops.WDT_F32S):
        with ops.pack_lowp(wdt):
            layer = ops.pack_conv(w.float().to(device), None, dilation=dil)
        assert layer.wdtype == (ops.WDT_F32P if wdt == ops.WDT_F32S and ops.SPLIT_W else wdt)
        out = ops.conv1d(x.float().to(device), layer).double().cpu()
        e = out - ref
        errs[wdt] = (e.pow(2).mean().sqrt().item() / rms, e.abs().max().item() / rms)
    assert errs[ops.WDT_F32S][0] <= 1.5 * errs[ops.WDT_F32][0], errs
    assert errs[ops.WDT_F32S][1] <= 1.5 * errs[ops.WDT_F32][1], errs


@pytest.mark.parametrize("kind,cin,cout,k,dil,T", [
    ("store", 256, 256, 11, 5, 4000), ("store", 128, 256, 3, 1, 1001), ("gate", 128, 128, 7, 3, 2400),
    ("gate", 256, 512, 5, 1, 500), ("store", 96, 256, 1, 1, 130), ("up", 512, 256, 16, 8, 60),
    ("up", 256, 128, 12, 6, 403), ("store", 192, 512, 7, 1, 77), ("gate", 256, 256, 11, 1, 333)])
def test_conv1d_presplit_weights_bitwise_equal_f32s(device, monkeypatch, kind, cin, cout, k, dil,
                                                     T):
    """VITS_WDT_F32P (weights split once on the host into bf16 planes, A
    fragments from global memory, X-only LDS) runs the same six MFMAs in the
    same order as VITS_WDT_F32S (weights split per fragment in registers):
    the outputs must be bitwise identical - over both staging paths (T % 4
    == 0: 16-byte blocks; otherwise element-wise), gate / store /
    upsample epilogues, residual and cond inputs, and every tile the
    dispatcher picks (incl. the small-grid 64x128 fallback)."""
    g = torch.Generator().manual_seed(cin + k + T)
    B = 2
    x = torch.randn(B, cin, T, generator=g).to(device)
    bias = torch.randn(cout, generator=g).to(device)
    outs = {}
    for split_w in (False, True):
        monkeypatch.setattr(ops, "SPLIT_W", split_w)
        with ops.pack_lowp(ops.WDT_F32S):
            if kind == "up":
                w = torch.randn(cin, cout, k, generator=torch.Generator().manual_seed(1)) * 0.05
                layer = ops.pack_conv_transpose(w.to(device), torch.zeros(cout, device=device),
                                                dil, (k - dil) // 2)
            else:
                w = torch.randn(cout, cin, k, generator=torch.Generator().manual_seed(1)) * 0.05
                layer = ops.pack_conv(w.to(device), bias, dilation=dil, gate=kind == "gate")
        assert layer.wdtype == (ops.WDT_F32P if split_w else ops.WDT_F32S)
        if kind == "gate":
            cond = torch.randn(B, cout, generator=torch.Generator().manual_seed(2)).to(device)
            outs[split_w] = ops.conv1d(x, layer, in_slope=0.1, cond=cond)
        elif kind == "store":
            res = torch.randn(B, cout, T, generator=torch.Generator().manual_seed(3)).to(device)
            outs[split_w] = ops.conv1d(x, layer, in_slope=0.1, residual=res)
        else:
            outs[split_w] = ops.conv1d(x, layer, in_slope=0.1)
    torch.cuda.synchronize()
    assert torch.isfinite(outs[True]).all()
    assert torch.equal(outs[True], outs[False])


@pytest.mark.parametrize("wdt", [ops.WDT_F32, ops.WDT_F32S])
def test_conv1d_nonfinite_inputs_stay_nonfinite(device, wdt):
    """A non-finite activation (the reference's fp32 conv: +-inf or NaN in
    every output column its receptive field reaches) stays non-finite in
    exactly those columns on both fp32 paths.  Split fp32 may turn an inf
    into NaN there (x - hi = inf - inf, engine.FP32_MODE note); finite
    outputs are unaffected."""
    g = torch.Generator().manual_seed(11)
    C, k, T = 128, 7, 300
    x = torch.randn(2, C, T, generator=g)
    x[0, 5, 100] = float("inf")
    x[1, 3, 50] = float("-inf")
    x[1, 9, 200] = float("nan")
    w = torch.randn(C, C, k, generator=g) / (C * k) ** 0.5
    ref = F.conv1d(x, w, padding=(k - 1) // 2)
    with ops.pack_lowp(wdt):
        layer = ops.pack_conv(w.to(device), None)
    out = ops.conv1d(x.to(device), layer).cpu()
    fin = torch.isfinite(ref)
    assert not fin.all()
    assert torch.equal(torch.isfinite(out), fin)
    _close(out[fin], ref[fin], what="finite part")


def test_conv1d_masked_split_accumulate(device):
    B, H, T = 3, 64, 150
    g = torch.Generator().manual_seed(3)
    a = torch.randn(B, H, T, generator=g)
    w = torch.randn(2 * H, H, 1, generator=g) / H ** 0.5
    b = torch.randn(2 * H, generator=g) * 0.1
    x = torch.randn(B, H, T, generator=g)
    acc0 = torch.randn(B, H, T, generator=g)
    lengths = torch.tensor([150, 97, 1], dtype=torch.int32)
    mask = (torch.arange(T)[None] < lengths[:, None]).float().unsqueeze(1)
    rs = F.conv1d(a, w, b)
    ref_x = (x + rs[:, :H]) * mask
    ref_o = acc0 + rs[:, H:]
    dev = device
    layer = ops.pack_conv(w.to(dev), b.to(dev))
    xd, od, ad = x.to(dev).clone(), acc0.to(dev).clone(), a.to(dev)
    o0 = ops.make_out(xd, res=xd)
    o1 = ops.make_out(od, accumulate=True)
    d = ops.make_desc(layer, ad, o0, out1=o1, split=H, lengths=lengths.to(dev))
    ops.conv1d_launch(d, B, ad.device)
    _close(xd, ref_x, what="residual half")
    # out1 is not masked by the kernel: the reference masks output once at the end
    o1ref = ref_o.clone()
    o1ref[mask.expand_as(o1ref) == 0] = 0
    got = od.cpu()
    got[mask.expand_as(got) == 0] = 0
    _close(got, o1ref, what="skip half")


def test_linear_rows(device):
    g = torch.Generator().manual_seed(5)
    x = torch.randn(5, 1024, generator=g)
    w = torch.randn(3000, 1024, generator=g) * 0.03
    b = torch.randn(3000, generator=g)
    out = ops.linear_rows(x.to(device), w.to(device), b.to(device))
    _close(out, F.linear(x, w, b), what="linear")


def test_expand_prior(device):
    g = torch.Generator().manual_seed(9)
    B, Cc, Tx = 2, 192, 37
    dur = torch.randint(1, 6, (B, 1, Tx), generator=g).float()
    Ty = int(dur.sum(-1).max())
    cum = torch.cumsum(dur, -1)
    t = torch.arange(Ty).float()
    path = (t[None, :, None] < cum[:, 0, None, :]).float()
    path = path - F.pad(path, (1, 0))[:, :, :-1]
    attn = path  # [B, Ty, Tx]
    m = torch.randn(B, Cc, Tx, generator=g)
    s = torch.rand(B, Cc, Tx, generator=g) + 0.5
    n = torch.randn(B, Cc, Ty, generator=g)
    ref = torch.matmul(attn, m.transpose(1, 2)).transpose(1, 2) + n * torch.matmul(attn, s.transpose(1, 2)).transpose(1, 2)
    out = ops.expand_prior(attn.to(device), m.to(device), s.to(device), n.to(device))
    _close(out, ref, tol=1e-6, what="expand")


@pytest.mark.parametrize("T,dt", [(1234, torch.float32), (1236, torch.float32),
                                  (9216, torch.float32), (9216, torch.bfloat16),
                                  (4000, torch.float16), (1230, torch.bfloat16)])
def test_conv_post_tanh(device, T, dt):
    """The Generator tail: element-wise staging (T % 4 != 0) and the 4-step
    block form (T % 4 == 0), fp32 and 16-bit last-stage activations."""
    g = torch.Generator().manual_seed(11)
    x = (torch.randn(2, 32, T, generator=g)).to(dt)
    w = torch.randn(1, 32, 7, generator=g) * 0.2
    ref = torch.tanh(F.conv1d(F.leaky_relu(x.float()), w, None, padding=3))
    out = ops.conv_post_tanh(x.to(device), w.to(device))
    _close(out, ref, what="conv_post")


@pytest.mark.parametrize("B,Tt,Ts", [(4, 60, 13), (3, 500, 100), (2, 1000, 384), (1, 7, 7),
                                     (2, 300, 65), (5, 33, 17), (3, 64, 40), (3, 65, 64),
                                     (1, 1, 1), (64, 500, 100)])
def test_maximum_path_bitexact(device, B, Tt, Ts):
    """vits_maximum_path vs the C oracle (core.pyx restated), bit-exact:
    ragged lengths, 32-row decision-word block edges (33, 64, 65 rows), the
    global-workspace decision words (1000 x 384) and the benchmark shape."""
    from oracle import mas as mas_oracle

    rng = np.random.default_rng(Tt * 7 + Ts)
    nc = rng.standard_normal((B, Tt, Ts)).astype(np.float32) * 3
    t_t = rng.integers(max(1, Tt // 2), Tt + 1, size=B).astype(np.int32)
    t_t[0] = Tt
    t_s = np.minimum(rng.integers(1, Ts + 1, size=B), t_t).astype(np.int32)
    t_s[0] = min(Ts, Tt)
    mask = np.zeros((B, Tt, Ts), np.float32)
    for b in range(B):
        mask[b, :t_t[b], :t_s[b]] = 1
    ref = mas_oracle.maximum_path(nc, mask)
    out = ops.maximum_path(torch.from_numpy(nc).to(device), torch.from_numpy(mask).to(device))
    assert out.dtype == torch.float32
    assert np.array_equal(out.cpu().numpy().astype(np.int32), ref)


def test_maximum_path_ties_and_dtype(device):
    from oracle import mas as mas_oracle

    # integer-valued scores create many exact ties: the strict '<' rule decides
    rng = np.random.default_rng(1)
    nc = rng.integers(-2, 3, size=(3, 40, 12)).astype(np.float32)
    mask = np.ones_like(nc)
    ref = mas_oracle.maximum_path(nc, mask)
    out = ops.maximum_path(torch.from_numpy(nc).to(device).half(), torch.from_numpy(mask).to(device))
    assert out.dtype == torch.float16
    assert np.array_equal(out.float().cpu().numpy().astype(np.int32), ref)


@pytest.mark.parametrize("n_fft,hop", [(128, 32), (256, 64), (512, 128), (1024, 256), (2048, 512)])
def test_stft_mag_fwd_bwd(device, n_fft, hop):
    g = torch.Generator().manual_seed(n_fft)
    x = (torch.randn(3, 9216, generator=g) * 0.3).clamp(-1, 1)
    win = torch.hann_window(n_fft)
    xr = x.clone().requires_grad_(True)
    spec = torch.stft(xr, n_fft, hop, n_fft, win, center=True, pad_mode="reflect", return_complex=True)
    ref = torch.sqrt(spec.real ** 2 + spec.imag ** 2 + 1e-7)
    gm = torch.randn(ref.shape, generator=g)
    (ref * gm).sum().backward()
    xd = x.to(device).requires_grad_(True)
    out = ops.stft_mag(xd, win.to(device), n_fft, hop, n_fft)
    _close(out, ref, tol=2e-5, what="stft mag")
    (out * gm.to(device)).sum().backward()
    _close(xd.grad, xr.grad, tol=2e-5, what="stft grad")


def test_stft_spectrogram_args(device):
    # mel_processing.spectrogram_torch: pad (n_fft-hop)/2 reflect, win 768 centred in 1024
    g = torch.Generator().manual_seed(2)
    y = (torch.randn(2, 19200, generator=g) * 0.3).clamp(-1, 1)
    n_fft, hop, win = 1024, 192, 768
    p = (n_fft - hop) // 2
    yp = F.pad(y.unsqueeze(1), (p, p), mode="reflect").squeeze(1)
    spec = torch.stft(yp, n_fft, hop, win, torch.hann_window(win), center=False, return_complex=True)
    ref = torch.sqrt(spec.real ** 2 + spec.imag ** 2 + 1e-6)
    out = ops.stft_mag(y.to(device), torch.hann_window(win).to(device), n_fft, hop, win, pad=p, eps=1e-6)
    _close(out, ref, tol=2e-5, what="spectrogram")


def test_layer_norm_channels(device):
    g = torch.Generator().manual_seed(4)
    x = torch.randn(3, 256, 77, generator=g)
    r = torch.randn(3, 256, 77, generator=g)
    gamma = torch.randn(256, generator=g)
    beta = torch.randn(256, generator=g)
    ref = F.layer_norm((x + r).transpose(1, -1), (256,), gamma, beta, 1e-5).transpose(1, -1)
    out = ops.layer_norm_channels(x.to(device), gamma.to(device), beta.to(device), residual=r.to(device))
    _close(out, ref, tol=1e-5, what="LN")


@pytest.mark.parametrize("T,lens", [(100, [100]), (77, [77, 50, 3]), (500, [500, 321])])
def test_attention(device, T, lens):
    g = torch.Generator().manual_seed(T)
    B, H, D = len(lens), 2, 128
    q = torch.randn(B, H * D, T, generator=g)
    k = torch.randn(B, H * D, T, generator=g)
    v = torch.randn(B, H * D, T, generator=g)
    lengths = torch.tensor(lens, dtype=torch.int32)
    mask = (torch.arange(T)[None] < lengths[:, None]).float()
    am = (mask.unsqueeze(2) * mask.unsqueeze(1)).unsqueeze(1)
    qh = q.view(B, H, D, T).transpose(2, 3)
    kh = k.view(B, H, D, T).transpose(2, 3)
    vh = v.view(B, H, D, T).transpose(2, 3)
    sc = torch.matmul(qh / D ** 0.5, kh.transpose(-2, -1)).masked_fill(am == 0, -1e4)
    ref = torch.matmul(F.softmax(sc, -1), vh).transpose(2, 3).reshape(B, H * D, T)
    out = ops.attention(q.to(device), k.to(device), v.to(device), H, lengths=lengths.to(device))
    _close(out, ref, tol=2e-5, what="attention")


@pytest.mark.gpu
@pytest.mark.parametrize("D", [16, 32, 48, 64, 96])
def test_attention_head_dims(device, D):
    g = torch.Generator().manual_seed(D)
    B, H, T = 2, 2, 37
    q, k, v = (torch.randn(B, H * D, T, generator=g) for _ in range(3))
    lengths = torch.tensor([T, 20], dtype=torch.int32)
    mask = (torch.arange(T)[None] < lengths[:, None]).float()
    am = (mask.unsqueeze(2) * mask.unsqueeze(1)).unsqueeze(1)
    qh, kh, vh = (t.view(B, H, D, T).transpose(2, 3) for t in (q, k, v))
    sc = torch.matmul(qh / D ** 0.5, kh.transpose(-2, -1)).masked_fill(am == 0, -1e4)
    ref = torch.matmul(F.softmax(sc, -1), vh).transpose(2, 3).reshape(B, H * D, T)
    out = ops.attention(q.to(device), k.to(device), v.to(device), H, lengths=lengths.to(device))
    _close(out, ref, tol=2e-5, what=f"attention D={D}")


def test_attention_fused_qkv_strides(device):
    """q|k|v as channel slices of one [B, 3C, T] projection buffer (the
    engine's layout): batch stride 3*C*T for inputs, C*T for the output."""
    from vits_amd import engine

    g = torch.Generator().manual_seed(12)
    B, H, D, T = 3, 2, 128, 45
    qkv = torch.randn(B, 3 * H * D, T, generator=g)
    q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
    qh = q.reshape(B, H, D, T).transpose(2, 3)
    kh = k.reshape(B, H, D, T).transpose(2, 3)
    vh = v.reshape(B, H, D, T).transpose(2, 3)
    ref = torch.matmul(F.softmax(torch.matmul(qh / D ** 0.5, kh.transpose(-2, -1)), -1), vh)
    ref = ref.transpose(2, 3).reshape(B, H * D, T)
    out = torch.empty(B, H * D, T, device=device)
    engine._attention_into(qkv.to(device), H * D, H, None, out)
    _close(out, ref, tol=2e-5, what="fused-qkv attention")


@pytest.mark.parametrize("B,C,Tt,Ts", [(3, 192, 500, 100), (2, 5, 37, 13), (1, 16, 1, 1), (2, 192, 129, 33)])
def test_neg_cent(device, B, C, Tt, Ts):
    """vits_neg_cent vs the models.py:483-489 formula in float64 (the HIP
    kernel accumulates in fp32 in a different order: tol 2e-6 of max|nc|)."""
    from oracle.vits_oracle import neg_cent as nc_ref

    g = torch.Generator().manual_seed(B * 1000 + Tt)
    z = torch.randn(B, C, Tt, generator=g)
    m = torch.randn(B, C, Ts, generator=g)
    lg = torch.randn(B, C, Ts, generator=g) * 0.5
    ref = nc_ref(z.double(), m.double(), lg.double())
    out = ops.neg_cent(z.to(device), m.to(device), lg.to(device))
    assert out.shape == (B, Tt, Ts) and out.dtype == torch.float32
    err = (out.cpu().double() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 2e-6, err


# --------------------------------------------------------------------------
# bf16-MFMA conv variant (C5 / bf16 models): exact semantics are
# conv(bf16(leaky_relu(x)), bf16(w)) accumulated in fp32, so it is compared
# with that reference computed in float64 (tolerance 2e-5 of max|y|: fp32
# accumulation order only), and with the fp32 conv loosely (bf16 rounding).
# --------------------------------------------------------------------------

def _bf(t, dt=torch.bfloat16):
    return t.to(dt).double()


_LOWP = {torch.bfloat16: 1, torch.float16: 2}


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("B,cin,cout,k,dil,T,gate", [
    (2, 256, 256, 3, 1, 300, True), (1, 128, 128, 11, 5, 777, True), (2, 64, 128, 7, 1, 500, False),
    (3, 16, 32, 11, 1, 1000, False), (2, 32, 32, 3, 5, 2000, True), (1, 192, 512, 7, 1, 101, False),
    (2, 513, 256, 1, 1, 64, False), (1, 24, 40, 5, 2, 90, False),
])
def test_conv1d_bf16(device, B, cin, cout, k, dil, T, gate, dt):
    g = torch.Generator().manual_seed(B * 100 + cin + k)
    x = torch.randn(B, cin, T, generator=g)
    w = torch.randn(cout, cin, k, generator=g) / (cin * k) ** 0.5
    b = torch.randn(cout, generator=g) * 0.1
    pad = (k * dil - dil) // 2
    xa = F.leaky_relu(x, 0.1)
    yq = F.conv1d(_bf(xa, dt), _bf(w, dt), b.double(), padding=pad, dilation=dil)
    cond = torch.randn(B, cout, generator=g) if gate else None
    res = None if gate else torch.randn(B, cout, T, generator=g)
    if gate:
        ya, yb = yq.chunk(2, 1)
        sa, sb = cond.double().chunk(2, 1)
        ref = torch.tanh(ya + sa.unsqueeze(-1)) * torch.sigmoid(yb + sb.unsqueeze(-1))
    else:
        ref = yq + res.double()
    with ops.pack_lowp(_LOWP[dt]):
        layer = ops.pack_conv(w.to(device), b.to(device), dilation=dil, gate=gate)
    assert layer.wdtype == _LOWP[dt] and layer.w.dtype == dt
    out = ops.conv1d(x.to(device), layer, in_slope=0.1,
                     cond=None if cond is None else cond.to(device),
                     residual=None if res is None else res.to(device))
    _close(out, ref, tol=2e-5, what="bf16 conv vs bf16-rounded fp64")


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_conv_transpose_bf16(device, dt):
    g = torch.Generator().manual_seed(5)
    B, cin, cout, K, u, T = 2, 256, 128, 12, 6, 57
    x = torch.randn(B, cin, T, generator=g)
    w = torch.randn(cin, cout, K, generator=g) / (cin * 2) ** 0.5
    b = torch.randn(cout, generator=g) * 0.1
    pad = (K - u) // 2
    ref = F.conv_transpose1d(_bf(F.leaky_relu(x, 0.1), dt), _bf(w, dt), b.double(), stride=u,
                             padding=pad)
    with ops.pack_lowp(_LOWP[dt]):
        layer = ops.pack_conv_transpose(w.to(device), b.to(device), u, pad)
    out = ops.conv1d(x.to(device), layer, in_slope=0.1)
    _close(out, ref, tol=2e-5, what="bf16 convT")


def test_stft_mag_multi_matches_single(device):
    """The one-launch multi-job STFT (MR-STFT loss) equals the per-job kernel:
    magnitudes bit for bit (same block code), input gradients to fp32
    rounding (autograd sums the three per-resolution gradients of a signal
    in its own order)."""
    g = torch.Generator().manual_seed(3)
    xs = [torch.randn(3, 9216, generator=g).to(device).requires_grad_(True) for _ in range(2)]
    res = [(128, 32, 128), (512, 128, 512), (2048, 512, 2048)]
    specs = [(torch.hann_window(w).to(device), n, h, w, None, 1e-7) for n, h, w in res]
    mags = ops.stft_mag_multi([xs[0]] * 3 + [xs[1]] * 3, specs + specs)
    loss = sum((m * (i + 1)).sum() for i, m in enumerate(mags))
    gm = torch.autograd.grad(loss, xs)
    xs1 = [x.detach().clone().requires_grad_(True) for x in xs]
    ref = [ops.stft_mag(xs1[0], w, n, h, wl, eps=e) for (w, n, h, wl, _, e) in specs] + \
          [ops.stft_mag(xs1[1], w, n, h, wl, eps=e) for (w, n, h, wl, _, e) in specs]
    loss1 = sum((m * (i + 1)).sum() for i, m in enumerate(ref))
    g1 = torch.autograd.grad(loss1, xs1)
    for a, b in zip(mags, ref):
        assert torch.equal(a, b)
    for a, b in zip(gm, g1):
        _close(a, b, tol=1e-6, what="multi-STFT grad")


def test_stft_mag_multi_target_not_differentiable(device):
    """Magnitudes of a signal without grad come back without a grad_fn (the
    MR-STFT target), so a discriminator backward through them never reaches
    the transform's backward."""
    g = torch.Generator().manual_seed(4)
    x = torch.randn(2, 4096, generator=g).to(device).requires_grad_(True)
    y = torch.randn(2, 4096, generator=g).to(device)
    spec = (torch.hann_window(256).to(device), 256, 64, 256, None, 1e-7)
    mx, my = ops.stft_mag_multi([x, y], [spec, spec])
    assert mx.requires_grad and not my.requires_grad and my.grad_fn is None


def _resblock_pair_ref(x, w1, b1, cond, w2, b2, k, dil):
    """modules.py:251-259 for one (c1, c2, cs) pair, fp64 on CPU."""
    x, w1, b1, w2, b2 = (t.double().cpu() for t in (x, w1, b1, w2, b2))
    xt = F.conv1d(F.leaky_relu(x, 0.1), w1, b1, dilation=dil, padding=(k - 1) * dil // 2)
    xa, xb = torch.chunk(xt, 2, dim=1)
    sa, sb = torch.chunk(cond.double().cpu(), 2, dim=1)
    xt = torch.tanh(xa + sa.unsqueeze(-1)) * torch.sigmoid(xb + sb.unsqueeze(-1))
    return F.conv1d(xt, w2, b2, padding=(k - 1) // 2) + x


@pytest.mark.parametrize("C,k,dil,T", [
    (32, 3, 1, 12), (32, 11, 5, 300), (64, 7, 3, 2052), (64, 3, 5, 48), (32, 7, 1, 9216),
    (64, 11, 1, 500),
])
def test_resblock_pair_fused(device, C, k, dil, T):
    """csrc/resblock.hip (c1 -> gate -> c2 -> residual in one kernel, the
    32/64-channel Generator stages) against the pair in fp64 on CPU: tiles
    shorter than the sequence, sequence ends inside a tile (c2's zero
    padding of the gated signal), the three-branch grouped launch and the
    branch-mean epilogue (accumulate, post_div).  Tolerance 1e-4 of the
    output magnitude (fp32 MFMA; fast exp-based tanh / sigmoid ~1e-7)."""
    g = torch.Generator().manual_seed(C + k + dil + T)
    B = 2
    packs, refs, xs = [], [], []
    for j in range(3):
        x = torch.randn(B, C, T, generator=g) * 0.5
        w1 = torch.randn(C, C, k, generator=g) / (C * k) ** 0.5
        b1 = torch.randn(C, generator=g) * 0.1
        w2 = torch.randn(C, C // 2, k, generator=g) / (C * k / 2) ** 0.5
        b2 = torch.randn(C, generator=g) * 0.1
        cond = torch.randn(B, C, generator=g) * 0.3
        c1 = ops.pack_conv(w1.to(device), b1.to(device), dilation=dil, gate=True)
        c2 = ops.pack_conv(w2.to(device), b2.to(device))
        assert k > ops.RESBLOCK_PAIR_MAX_K or ops.resblock_pair_supported(c1, c2, T)
        packs.append((c1, c2, cond.to(device)))
        refs.append(_resblock_pair_ref(x, w1, b1, cond, w2, b2, k, dil))
        xs.append(x.to(device))
    ys = [torch.full((B, C, T), float("nan"), device=device) for _ in range(3)]
    ops.resblock_pair_launch(tuple(
        ops.resblock_pair_desc(c1, c2, xs[j], ys[j], cond=cd) for j, (c1, c2, cd) in enumerate(packs)),
        B, device)
    torch.cuda.synchronize()
    for j in range(3):
        _close(ys[j], refs[j], what=f"pair {j}")
    # branch mean into one buffer: y = (r0 + r1 + r2) / 3
    acc = torch.empty(B, C, T, device=device)
    for j, (c1, c2, cd) in enumerate(packs):
        ops.resblock_pair_launch(ops.resblock_pair_desc(
            c1, c2, xs[j], acc, cond=cd, accumulate=j > 0, post_div=3.0 if j == 2 else 1.0),
            B, device)
    torch.cuda.synchronize()
    _close(acc, (refs[0] + refs[1] + refs[2]) / 3, what="mean")


@pytest.mark.parametrize("C,k,dil,T", [
    (32, 3, 1, 12), (32, 11, 5, 300), (64, 7, 3, 2052), (64, 3, 5, 48), (32, 7, 1, 9216),
    (64, 11, 5, 1000), (64, 11, 1, 500), (128, 3, 1, 500), (128, 11, 5, 1000), (128, 7, 3, 124),
    (256, 3, 1, 132), (256, 11, 5, 1000), (256, 7, 3, 300),
])
@pytest.mark.parametrize("wdt", [ops.WDT_BF16, ops.WDT_F16])
def test_resblock_pair16_fused(device, C, k, dil, T, wdt):
    """csrc/resblock16.hip (the pair of a 16-bit model: 16-bit x / y and
    weight images, fp32 accumulation, the gated tensor rounded to 16 bits in
    LDS as the two-conv path rounds it in HBM) against the pair in fp64 on
    the same 16-bit-rounded inputs and weights: tiles shorter than the
    sequence, ends inside a tile, the three-branch grouped launch and the
    branch-mean epilogue.  256 channels: csrc/resblock_f32p.hip's 16-bit
    mode (no one-launch branch mean there).  Tolerance: 2 roundings of the
    operand type (bf16 2e-2, fp16 3e-3 of the output magnitude)."""
    dt = {ops.WDT_BF16: torch.bfloat16, ops.WDT_F16: torch.float16}[wdt]
    tol = 2e-2 if wdt == ops.WDT_BF16 else 3e-3
    g = torch.Generator().manual_seed(C + k + dil + T + wdt)
    B = 2
    packs, refs, xs = [], [], []
    for j in range(3):
        x = (torch.randn(B, C, T, generator=g) * 0.5).to(dt)
        w1 = (torch.randn(C, C, k, generator=g) / (C * k) ** 0.5).to(dt).float()
        b1 = torch.randn(C, generator=g) * 0.1
        w2 = (torch.randn(C, C // 2, k, generator=g) / (C * k / 2) ** 0.5).to(dt).float()
        b2 = torch.randn(C, generator=g) * 0.1
        cond = torch.randn(B, C, generator=g) * 0.3
        with ops.pack_lowp(wdt):
            c1 = ops.pack_conv(w1.to(device), b1.to(device), dilation=dil, gate=True)
            c2 = ops.pack_conv(w2.to(device), b2.to(device))
        xd = x.to(device)
        assert ops.resblock_pair16_supported(c1, c2, xd)
        packs.append((c1, c2, cond.to(device)))
        refs.append(_resblock_pair_ref(x.float(), w1, b1, cond, w2, b2, k, dil))
        xs.append(xd)
    ys = [torch.full((B, C, T), float("nan"), device=device, dtype=dt) for _ in range(3)]
    ops.resblock_pair16_launch(tuple(
        ops.resblock_pair16_desc(c1, c2, xs[j], ys[j], cond=cd)
        for j, (c1, c2, cd) in enumerate(packs)), B, device, wdt)
    torch.cuda.synchronize()
    for j in range(3):
        _close(ys[j], refs[j], tol=tol, what=f"pair {j}")
    acc = torch.empty(B, C, T, device=device, dtype=dt)
    for j, (c1, c2, cd) in enumerate(packs):
        ops.resblock_pair16_launch(ops.resblock_pair16_desc(
            c1, c2, xs[j], acc, cond=cd, accumulate=j > 0, post_div=3.0 if j == 2 else 1.0),
            B, device, wdt)
    torch.cuda.synchronize()
    _close(acc, (refs[0] + refs[1] + refs[2]) / 3, tol=2 * tol, what="mean")
    if C == 256:
        return
    # the branch mean as ONE launch (vits_resblock_pair16_mean_forward)
    mean = torch.full((B, C, T), float("nan"), device=device, dtype=dt)
    ops.resblock_pair16_launch(tuple(
        ops.resblock_pair16_desc(c1, c2, xs[j], mean, cond=cd)
        for j, (c1, c2, cd) in enumerate(packs)), B, device, wdt, mean=True)
    torch.cuda.synchronize()
    _close(mean, (refs[0] + refs[1] + refs[2]) / 3, tol=tol, what="mean launch")


@pytest.mark.parametrize("C,k,dil,T", [
    (64, 3, 1, 12), (64, 11, 5, 1000), (64, 7, 3, 2052), (128, 3, 5, 48), (128, 11, 5, 1000),
    (128, 7, 1, 500), (256, 11, 3, 300), (256, 3, 1, 132), (32, 3, 1, 2000), (32, 11, 5, 600),
])
def test_resblock_pair_f32p_fused(device, monkeypatch, C, k, dil, T):
    """csrc/resblock_f32p.hip (the split-fp32 pair of the 64/128/256-channel
    stages) equals the two-conv path it replaces BIT FOR BIT - c1 with the
    gate epilogue into an fp32 gated tensor, c2 with the residual epilogue:
    the same split planes, k-step order, products and epilogue expressions -
    for the three-branch grouped launch, the branch-mean epilogue
    (accumulate, post_div) and utterance lengths (the gated tensor and the
    output zero past them); and matches the pair in fp64 to 2e-6 of the
    output magnitude (fp32 arithmetic)."""
    g = torch.Generator().manual_seed(C + k + dil + T)
    B = 2
    packs, refs, xs = [], [], []
    # (the kernel takes every stage and k; the engine's rule picks where)
    monkeypatch.setattr(ops, "F32P_PAIR_MAX_K", {32: 15, 64: 15, 128: 15, 256: 15})
    for j in range(3):
        x = torch.randn(B, C, T, generator=g) * 0.5
        w1 = torch.randn(C, C, k, generator=g) / (C * k) ** 0.5
        b1 = torch.randn(C, generator=g) * 0.1
        w2 = torch.randn(C, C // 2, k, generator=g) / (C * k / 2) ** 0.5
        b2 = torch.randn(C, generator=g) * 0.1
        cond = torch.randn(B, C, generator=g) * 0.3
        c1 = ops.to_lowp(ops.pack_conv(w1.to(device), b1.to(device), dilation=dil, gate=True),
                         ops.WDT_F32S, min_rows=0)
        c2 = ops.to_lowp(ops.pack_conv(w2.to(device), b2.to(device)), ops.WDT_F32S, min_rows=0)
        assert c1.wdtype == c2.wdtype == ops.WDT_F32P
        xd = x.to(device)
        assert ops.resblock_pair_f32p_supported(c1, c2, xd)
        packs.append((c1, c2, cond.to(device)))
        refs.append(_resblock_pair_ref(x, w1, b1, cond, w2, b2, k, dil))
        xs.append(xd)

    def two_conv(j, y, lengths=None, **kw):
        c1, c2, cd = packs[j]
        gbuf = torch.full((B, C // 2, T), float("nan"), device=device)
        ops.conv1d_launch_seq([
            ops.make_desc(c1, xs[j], ops.make_out(gbuf), in_slope=0.1, cond=cd, lengths=lengths),
            ops.make_desc(c2, gbuf, ops.make_out(y, res=xs[j], **kw), lengths=lengths)], B, device)

    def fused(js, ys, lengths=None, **kw):
        ops.resblock_pair_launch(tuple(
            ops.resblock_pair_desc(packs[j][0], packs[j][1], xs[j], y, cond=packs[j][2],
                                   lengths=lengths, **kw) for j, y in zip(js, ys)),
            B, device, ops.WDT_F32P)

    ys = [torch.full((B, C, T), float("nan"), device=device) for _ in range(3)]
    fused(range(3), ys)
    for j in range(3):
        y2 = torch.full((B, C, T), float("nan"), device=device)
        two_conv(j, y2)
        torch.cuda.synchronize()
        d = (ys[j] - y2).abs().max().item()
        assert torch.equal(ys[j], y2), f"pair {j}: fused != two-conv, max diff {d:.3e}"
        _close(ys[j], refs[j], tol=2e-6, what=f"pair {j} vs fp64")
    # branch mean: accumulate in branch order, the last divides
    acc, acc2 = torch.empty(B, C, T, device=device), torch.empty(B, C, T, device=device)
    for j in range(3):
        kw = dict(accumulate=j > 0, post_div=3.0 if j == 2 else 1.0)
        fused([j], [acc], **kw)
        two_conv(j, acc2, **kw)
    torch.cuda.synchronize()
    assert torch.equal(acc, acc2), "mean"
    _close(acc, (refs[0] + refs[1] + refs[2]) / 3, tol=2e-6, what="mean vs fp64")
    # utterance lengths (bucketed inference): zero past them, bitwise again
    lens = torch.tensor([T, max(1, T - 37)], dtype=torch.int32, device=device)
    yl = [torch.zeros(B, C, T, device=device) for _ in range(3)]
    fused(range(3), yl, lengths=lens)
    for j in range(3):
        y2 = torch.zeros(B, C, T, device=device)
        two_conv(j, y2, lengths=lens)
        torch.cuda.synchronize()
        assert torch.equal(yl[j], y2), f"pair {j} with lengths"


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_generator16_fused_pairs_match_two_conv_path(device, monkeypatch, dt):
    """A 16-bit model's Generator with resblock16 pairs on its 32/64-channel
    stages against its two-conv path (ops.FUSED_PAIRS16 = False): the same
    rounding points (16-bit gated tensor, one rounding of each output), only
    the fp32 accumulation order differs - 1e-2 (bf16) / 2e-3 (fp16) of the
    waveform magnitude."""
    from common import base_model

    m = base_model(device).to(dt)
    g = torch.Generator().manual_seed(5)
    z = (torch.randn(2, 192, 40, generator=g) * 0.7).to(device).to(dt)
    gg = (torch.randn(2, 1024, generator=g) * 0.5).to(device).to(dt)
    tol = 1e-2 if dt == torch.bfloat16 else 2e-3
    with torch.no_grad():
        monkeypatch.setattr(ops, "FUSED_PAIRS16", True)
        m.dec.__dict__.pop("_vits_amd_plan", None)
        a = m.dec(z, gg)
        monkeypatch.setattr(ops, "FUSED_PAIRS16", False)
        b = m.dec(z, gg)
    _close(a, b, tol=tol, what="fused16 vs two-conv")


def test_generator_fused_pairs_match_two_conv_path(device, monkeypatch):
    """The Generator with fused pairs on its 32/64-channel stages equals the
    two-conv path (engine._FUSED_PAIRS = False) to fp32 rounding."""
    from common import base_model
    from vits_amd import engine

    m = base_model(device)
    g = torch.Generator().manual_seed(3)
    z = (torch.randn(2, 192, 40, generator=g) * 0.7).to(device)
    gg = (torch.randn(2, 1024, generator=g) * 0.5).to(device)
    with torch.no_grad():
        monkeypatch.setattr(engine, "_FUSED_PAIRS", True)
        a = m.dec(z, gg)
        monkeypatch.setattr(engine, "_FUSED_PAIRS", False)
        b = m.dec(z, gg)
    _close(a, b, what="fused vs two-conv")
