"""Host-side packing of the split-fp32 conv (VITS_WDT_F32S): the fp32
16-channel slab image, the row threshold and the tile rule (CPU only)."""
import subprocess
import sys

import torch

from vits_amd import ops


def test_f32s_slab_image_layout(monkeypatch):
    monkeypatch.setattr(ops, "SPLIT_W", False)
    g = torch.Generator().manual_seed(0)
    w = torch.randn(256, 40, 7, generator=g)
    with ops.pack_lowp(ops.WDT_F32S):
        layer = ops.pack_conv(w, None, dilation=3)
    assert layer.wdtype == ops.WDT_F32S and layer.w.dtype == torch.float32
    assert layer.kc == 16 and layer.cin_pad == 48 and layer.m_pad == 256
    # image [cin_pad/16][k][2][m_pad][8]: element (s, j, h, m, i) = W[m][16s + 8h + i][j]
    img = layer.w
    assert tuple(img.shape) == (3, 7, 2, 256, 8)
    for (m, c, j) in [(0, 0, 0), (255, 39, 6), (17, 23, 4), (100, 8, 1)]:
        s, h, i = c // 16, (c % 16) // 8, c % 8
        assert img[s, j, h, m, i].item() == w[m, c, j].item()
    # channel padding is zero
    assert img[2, :, 1].abs().sum().item() == 0.0
    assert layer.tile == ops.TILE_64x128


def test_f32s_row_threshold_and_tiles(monkeypatch):
    monkeypatch.setattr(ops, "SPLIT_W", False)
    w = torch.randn(64, 64, 3)
    with ops.pack_lowp(ops.WDT_F32S):
        small = ops.pack_conv(w, None)
        k3 = ops.pack_conv(torch.randn(256, 256, 3), None)
        k11 = ops.pack_conv(torch.randn(128, 128, 11), None, dilation=5)
        up = ops.pack_conv_transpose(torch.randn(256, 128, 12), None, 6, 3)
    assert small.wdtype == ops.WDT_F32  # < F32S_MIN_ROWS rows: exact fp32
    assert k3.wdtype == ops.WDT_F32S and k3.tile == ops.TILE_128x128
    assert k11.wdtype == ops.WDT_F32S and k11.tile == ops.TILE_64x256
    assert up.wdtype == ops.WDT_F32S and up.tile == ops.TILE_64x128


def test_fp32_mode_env():
    code = ("from vits_amd import engine, ops; "
            "print(engine.FP32_MODE, engine.FP32_WDTYPE == ops.WDT_F32)")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                         env={"VITS_FP32_MODE": "exact", "PATH": "/usr/bin:/bin"}, check=True)
    assert out.stdout.split()[-2:] == ["exact", "True"]
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                         env={"PATH": "/usr/bin:/bin"}, check=True)
    assert out.stdout.split()[-2:] == ["split", "False"]


def test_f32p_presplit_plane_image():
    """VITS_WDT_F32P (the default split-fp32 packing): the slab image split
    on the host into bf16 planes [cin_pad/16][k][2][3][m_pad][8], hi + mid +
    lo == the fp32 weight bit for bit, 128x128 tiles on >= 128 rows."""
    g = torch.Generator().manual_seed(0)
    w = torch.randn(256, 40, 7, generator=g) * torch.logspace(-6, 3, 40).view(1, 40, 1)
    with ops.pack_lowp(ops.WDT_F32S):
        layer = ops.pack_conv(w, None, dilation=3)
    assert ops.SPLIT_W and layer.wdtype == ops.WDT_F32P and layer.w.dtype == torch.bfloat16
    assert layer.kc == 16 and layer.cin_pad == 48 and layer.m_pad == 256
    img = layer.w
    assert tuple(img.shape) == (3, 7, 2, 3, 256, 8)
    rec = img[:, :, :, 0].float() + img[:, :, :, 1].float() + img[:, :, :, 2].float()
    for (m, c, j) in [(0, 0, 0), (255, 39, 6), (17, 23, 4), (100, 8, 1)]:
        s, h, i = c // 16, (c % 16) // 8, c % 8
        assert rec[s, j, h, m, i].item() == w[m, c, j].item()
        hi = img[s, j, h, 0, m, i].float().item()
        assert hi == torch.tensor(w[m, c, j].item()).view(torch.int32).bitwise_and(
            -65536).view(torch.float32).item()
    assert img[2, :, 1].abs().sum().item() == 0.0
    assert layer.tile == ops.TILE_128x128
