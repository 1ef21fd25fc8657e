"""The C-ABI library loads on a GPU-less host and exports every entry point
include/vits_amd.h declares (no compute calls here)."""
import ctypes
import os
import re

from common import HERE

ROOT = os.path.dirname(HERE)


def _declared():
    with open(os.path.join(ROOT, "include", "vits_amd.h")) as f:
        src = f.read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(vits_[a-z_0-9]+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_header_declares_entry_points():
    names = _declared()
    assert "vits_conv1d_forward" in names and "vits_maximum_path" in names
    assert len(names) >= 15


def test_library_exports_every_declared_symbol():
    from vits_amd import _lib

    lib = _lib.load()
    raw = ctypes.CDLL(_lib.lib_path())
    missing = [n for n in _declared() if not hasattr(raw, n)]
    assert not missing, missing
    # the Python binding covers every declared symbol too
    assert sorted(_lib.EXPORTED_SYMBOLS) == _declared()
    assert lib.vits_amd_version().startswith(b"vits_amd")


def test_struct_layout_matches_header():
    """ctypes struct sizes equal the C sizeof (checked by compiling a probe)."""
    import subprocess
    import tempfile

    from vits_amd._lib import (WNORM_MAX, SNORM_MAX, ConvDesc, ConvOut, GateBwdJob, Pack16Layer,
                               ResblockPairDesc, SnormLayer, StftJob, WnormLayer)

    probe = r'''
#include <stdio.h>
#include <stddef.h>
#include "vits_amd.h"
int main(){printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %d %d %zu %zu %zu %zu %zu %zu %zu\n", sizeof(vits_conv1d_desc),
 sizeof(vits_conv_out), offsetof(vits_conv1d_desc, out0), offsetof(vits_conv1d_desc, lengths),
 offsetof(vits_conv1d_desc, wdtype), sizeof(vits_stft_job), offsetof(vits_stft_job, eps),
 sizeof(vits_resblock_pair_desc), offsetof(vits_resblock_pair_desc, w2),
 offsetof(vits_resblock_pair_desc, post_div), sizeof(vits_wnorm_layer),
 sizeof(vits_snorm_layer), offsetof(vits_snorm_layer, eps), VITS_WNORM_MAX, VITS_SNORM_MAX,
 sizeof(vits_pack16_layer), offsetof(vits_pack16_layer, img_t), offsetof(vits_pack16_layer, cin_pad_t),
 offsetof(vits_conv1d_desc, gmask_slope), offsetof(vits_conv1d_desc, len_skip),
 sizeof(vits_gate_bwd_job), offsetof(vits_gate_bwd_job, half_channels));
 return 0;}
'''
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "p.c")
        exe = os.path.join(d, "p")
        with open(src, "w") as f:
            f.write(probe)
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), src, "-o", exe], check=True)
        out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout.split()
    assert int(out[0]) == ctypes.sizeof(ConvDesc)
    assert int(out[1]) == ctypes.sizeof(ConvOut)
    assert int(out[2]) == ConvDesc.out0.offset
    assert int(out[3]) == ConvDesc.lengths.offset
    assert int(out[4]) == ConvDesc.wdtype.offset
    assert int(out[5]) == ctypes.sizeof(StftJob)
    assert int(out[6]) == StftJob.eps.offset
    assert int(out[7]) == ctypes.sizeof(ResblockPairDesc)
    assert int(out[8]) == ResblockPairDesc.w2.offset
    assert int(out[9]) == ResblockPairDesc.post_div.offset
    assert int(out[10]) == ctypes.sizeof(WnormLayer)
    assert int(out[11]) == ctypes.sizeof(SnormLayer)
    assert int(out[12]) == SnormLayer.eps.offset
    assert int(out[13]) == WNORM_MAX and int(out[14]) == SNORM_MAX
    assert int(out[15]) == ctypes.sizeof(Pack16Layer)
    assert int(out[16]) == Pack16Layer.img_t.offset
    assert int(out[17]) == Pack16Layer.cin_pad_t.offset
    assert int(out[18]) == ConvDesc.gmask_slope.offset
    assert int(out[19]) == ConvDesc.len_skip.offset
    assert int(out[20]) == ctypes.sizeof(GateBwdJob)
    assert int(out[21]) == GateBwdJob.half_channels.offset


def test_dispatch_counters_host_side():
    """vits_dispatch_count / _reset are plain host functions (no GPU): one
    counter per VITS_CNT_* family of the header, reset to zero, -1 outside."""
    from vits_amd import _lib

    with open(os.path.join(ROOT, "include", "vits_amd.h")) as f:
        n = int(re.search(r"#define VITS_CNT_N (\d+)", f.read()).group(1))
    assert len(_lib.CNT_NAMES) == n
    _lib.dispatch_counts_reset()
    assert set(_lib.dispatch_counts().values()) == {0}
    lib = _lib.load()
    assert lib.vits_dispatch_count(-1) == -1 and lib.vits_dispatch_count(n) == -1
