"""ctypes binding of libvits_amd.so (the C-ABI declared in include/vits_amd.h).

The library is built in-tree by ``__graft_entry__.build()`` (Makefile in
``vits_amd/csrc``) into ``vits_amd/lib/libvits_amd.so``.  There is no
fallback: if the library is missing or fails to load, every op raises.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libvits_amd.so")
# A/B experiments (tools/ab_conv.sh) point this at an alternative build
_LIB_PATH = os.environ.get("VITS_AMD_LIB", _LIB_PATH)
_lock = threading.Lock()
_lib = None

VITS_OK = 0
VITS_E_ARG = -1
VITS_E_SHAPE = -2
VITS_E_UNSUP = -3

EPI_STORE, EPI_GATE, EPI_UPSAMPLE = 0, 1, 2
ACT_NONE, ACT_RELU, ACT_TANH, ACT_EXP = 0, 1, 2, 3
TILE_128x128, TILE_64x256, TILE_32x256, TILE_64x128 = 0, 1, 2, 3
WDT_F32, WDT_BF16, WDT_F16, WDT_F32S, WDT_F32P = 0, 1, 2, 3, 4
TILE_ROWS = {TILE_128x128: 128, TILE_64x256: 64, TILE_32x256: 32, TILE_64x128: 64}
DT_F32, DT_F16, DT_BF16, DT_I32 = 0, 1, 2, 3


class ConvOut(C.Structure):
    _fields_ = [
        ("y", C.c_void_p),
        ("y_bstride", C.c_int64),
        ("y_cstride", C.c_int32),
        ("act", C.c_int32),
        ("res", C.c_void_p),
        ("res_bstride", C.c_int64),
        ("res_cstride", C.c_int32),
        ("res_scale", C.c_float),
        ("accumulate", C.c_int32),
        ("post_div", C.c_float),
    ]


class ConvDesc(C.Structure):
    _fields_ = [
        ("x", C.c_void_p),
        ("x_bstride", C.c_int64),
        ("x_cstride", C.c_int32),
        ("x_tstride", C.c_int32),
        ("cin", C.c_int32),
        ("tin", C.c_int32),
        ("in_slope", C.c_float),
        ("w", C.c_void_p),
        ("m", C.c_int32),
        ("m_pad", C.c_int32),
        ("cin_pad", C.c_int32),
        ("kc", C.c_int32),
        ("k", C.c_int32),
        ("dil", C.c_int32),
        ("pad_left", C.c_int32),
        ("n_out", C.c_int32),
        ("tile", C.c_int32),
        ("epi", C.c_int32),
        ("bias", C.c_void_p),
        ("cond", C.c_void_p),
        ("cond_bstride", C.c_int64),
        ("split", C.c_int32),
        ("up_u", C.c_int32),
        ("up_pad", C.c_int32),
        ("t_out", C.c_int32),
        ("lengths", C.c_void_p),
        ("out0", ConvOut),
        ("out1", ConvOut),
        ("wdtype", C.c_int32),
        ("gmask", C.c_void_p),
        ("gmask_bstride", C.c_int64),
        ("gmask_cstride", C.c_int32),
        ("gmask_slope", C.c_float),
        ("io16", C.c_int32),
        ("len_skip", C.c_int32),
    ]


class ResblockPairDesc(C.Structure):
    """include/vits_amd.h vits_resblock_pair_desc."""
    _fields_ = [
        ("x", C.c_void_p),
        ("x_bstride", C.c_int64),
        ("x_cstride", C.c_int32),
        ("t_len", C.c_int32),
        ("channels", C.c_int32),
        ("in_slope", C.c_float),
        ("w1", C.c_void_p),
        ("m_pad1", C.c_int32),
        ("cin_pad1", C.c_int32),
        ("kc1", C.c_int32),
        ("k", C.c_int32),
        ("dil", C.c_int32),
        ("kc2", C.c_int32),
        ("b1", C.c_void_p),
        ("cond", C.c_void_p),
        ("cond_bstride", C.c_int64),
        ("w2", C.c_void_p),
        ("m_pad2", C.c_int32),
        ("cin_pad2", C.c_int32),
        ("b2", C.c_void_p),
        ("y", C.c_void_p),
        ("y_bstride", C.c_int64),
        ("y_cstride", C.c_int32),
        ("accumulate", C.c_int32),
        ("post_div", C.c_float),
        ("len_skip", C.c_int32),
        ("lengths", C.c_void_p),
    ]


class StftJob(C.Structure):
    _fields_ = [
        ("x", C.c_void_p),
        ("window", C.c_void_p),
        ("grad_mag", C.c_void_p),
        ("mag", C.c_void_p),
        ("re", C.c_void_p),
        ("im", C.c_void_p),
        ("grad_x", C.c_void_p),
        ("batch", C.c_int32),
        ("length", C.c_int32),
        ("n_fft", C.c_int32),
        ("hop", C.c_int32),
        ("win", C.c_int32),
        ("pad", C.c_int32),
        ("eps", C.c_float),
        ("layout", C.c_int32),
    ]


class ConvWgradDesc(C.Structure):
    _fields_ = [
        ("dy", C.c_void_p),
        ("dy_bstride", C.c_int64),
        ("dy_cstride", C.c_int32),
        ("cout", C.c_int32),
        ("x", C.c_void_p),
        ("x_bstride", C.c_int64),
        ("x_cstride", C.c_int32),
        ("cin", C.c_int32),
        ("tin", C.c_int32),
        ("n_out", C.c_int32),
        ("k", C.c_int32),
        ("dil", C.c_int32),
        ("pad_left", C.c_int32),
        ("in_slope", C.c_float),
        ("dw_t", C.c_void_p),
        ("dbias", C.c_void_p),
        ("wdtype", C.c_int32),
        ("reserved", C.c_int32),
        ("io16", C.c_int32),
        ("reserved2", C.c_int32),
    ]


class GateBwdJob(C.Structure):
    """vits_gate_bwd_job (one job of vits_gate_backward_io16_multi)."""
    _fields_ = [
        ("dy", C.c_void_p),
        ("dy_bstride", C.c_int64),
        ("dy_cstride", C.c_int64),
        ("x", C.c_void_p),
        ("x_bstride", C.c_int64),
        ("x_cstride", C.c_int64),
        ("g", C.c_void_p),
        ("g_bstride", C.c_int64),
        ("dx", C.c_void_p),
        ("dx_bstride", C.c_int64),
        ("dx_cstride", C.c_int64),
        ("dg", C.c_void_p),
        ("dg_bstride", C.c_int64),
        ("half_channels", C.c_int32),
        ("reserved", C.c_int32),
    ]


RADAM_MAX = 96


class RadamTensor(C.Structure):
    _fields_ = [
        ("param", C.c_void_p),
        ("grad", C.c_void_p),
        ("exp_avg", C.c_void_p),
        ("exp_avg_sq", C.c_void_p),
        ("numel", C.c_int64),
    ]


WNORM_MAX = 56
SNORM_MAX = 48


class Pack16Layer(C.Structure):
    _fields_ = [
        ("w", C.c_void_p),
        ("cout", C.c_int32),
        ("cin", C.c_int32),
        ("k", C.c_int32),
        ("img", C.c_void_p),
        ("m_pad", C.c_int32),
        ("cin_pad", C.c_int32),
        ("img_t", C.c_void_p),
        ("m_pad_t", C.c_int32),
        ("cin_pad_t", C.c_int32),
        ("gate", C.c_int32),
    ]


class WnormLayer(C.Structure):
    _fields_ = [
        ("v", C.c_void_p),
        ("g", C.c_void_p),
        ("w", C.c_void_p),
        ("dw", C.c_void_p),
        ("dv", C.c_void_p),
        ("dg", C.c_void_p),
        ("rows", C.c_int32),
        ("cols", C.c_int32),
    ]


class SnormLayer(C.Structure):
    _fields_ = [
        ("w", C.c_void_p),
        ("u", C.c_void_p),
        ("v", C.c_void_p),
        ("w_sn", C.c_void_p),
        ("dw_sn", C.c_void_p),
        ("dw", C.c_void_p),
        ("saved", C.c_void_p),
        ("rows", C.c_int32),
        ("cols", C.c_int32),
        ("eps", C.c_float),
        ("cl_channels", C.c_int32),
    ]


_SIGS = {
    "vits_conv1d_forward": (C.c_int, [C.POINTER(ConvDesc), C.c_int, C.c_void_p]),
    "vits_conv1d_forward_seq": (C.c_int, [C.POINTER(ConvDesc), C.c_int, C.c_int, C.c_void_p]),
    "vits_conv1d_forward_groups": (
        C.c_int, [C.POINTER(ConvDesc), C.POINTER(C.c_int32), C.c_int, C.c_int, C.c_void_p]),
    "vits_linear_forward": (
        C.c_int,
        [C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_int, C.c_int,
         C.c_int, C.c_void_p],
    ),
    "vits_expand_prior": (
        C.c_int,
        [C.c_void_p] * 5 + [C.c_int] * 5 + [C.c_float, C.c_void_p],
    ),
    "vits_expand_durations": (
        C.c_int,
        [C.c_void_p, C.c_int64, C.c_void_p, C.c_int, C.c_float, C.c_int, C.c_void_p, C.c_void_p,
         C.c_int64, C.c_int32, C.c_void_p, C.c_int, C.c_void_p, C.c_int64, C.c_float, C.c_void_p,
         C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p],
    ),
    "vits_conv_post_tanh": (
        C.c_int,
        [C.c_void_p, C.c_int64, C.c_int32, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int,
         C.c_int, C.c_void_p],
    ),
    "vits_conv_post_tanh_lowp": (
        C.c_int,
        [C.c_void_p, C.c_int64, C.c_int32, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int,
         C.c_int, C.c_int, C.c_void_p],
    ),
    "vits_maximum_path": (
        C.c_int,
        [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int,
         C.c_void_p, C.c_int64, C.c_void_p],
    ),
    "vits_maximum_path_lengths": (
        C.c_int,
        [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int,
         C.c_void_p, C.c_int64, C.c_void_p],
    ),
    "vits_maximum_path_workspace": (C.c_int64, [C.c_int, C.c_int, C.c_int]),
    "vits_stft_mag_forward_multi": (C.c_int, [C.POINTER(StftJob), C.c_int, C.c_void_p]),
    "vits_stft_mag_backward_multi": (
        C.c_int, [C.POINTER(StftJob), C.c_int, C.c_void_p, C.c_int64, C.c_void_p]),
    "vits_stft_workspace_multi": (C.c_int64, [C.POINTER(StftJob), C.c_int]),
    "vits_neg_cent": (
        C.c_int,
        [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int,
         C.c_void_p],
    ),
    "vits_stft_mag_forward": (
        C.c_int,
        [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_float,
         C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p],
    ),
    "vits_stft_mag_backward": (
        C.c_int,
        [C.c_void_p] * 5
        + [C.c_int] * 6
        + [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p],
    ),
    "vits_stft_workspace": (C.c_int64, [C.c_int] * 5),
    "vits_layer_norm_channels": (
        C.c_int,
        [C.c_void_p] * 5 + [C.c_int] * 3
        + [C.c_float, C.c_void_p, C.c_void_p, C.c_int64, C.c_float, C.c_void_p, C.c_void_p,
           C.c_void_p],
    ),
    "vits_attention_forward": (
        C.c_int,
        [C.c_void_p] * 4 + [C.c_int] * 4 + [C.c_int64, C.c_int64, C.c_void_p, C.c_void_p],
    ),
    "vits_conv1d_pack16": (
        C.c_int,
        [C.c_void_p] + [C.c_int] * 4 + [C.c_void_p] + [C.c_int] * 3
        + [C.c_void_p, C.c_int64, C.c_void_p],
    ),
    "vits_conv1d_pack16_pair": (
        C.c_int,
        [C.c_void_p] + [C.c_int] * 3 + [C.c_void_p] + [C.c_int] * 2 + [C.c_void_p]
        + [C.c_int] * 3 + [C.c_void_p],
    ),
    "vits_conv1d_pack16_pairs": (C.c_int, [C.POINTER(Pack16Layer), C.c_int, C.c_int,
                                           C.c_void_p]),
    "vits_conv1d_wgrad": (C.c_int, [C.POINTER(ConvWgradDesc), C.c_int, C.c_void_p]),
    "vits_conv1d_wgrad_workspace": (C.c_int64, [C.POINTER(ConvWgradDesc), C.c_int]),
    "vits_conv1d_wgrad_split": (C.c_int, [C.POINTER(ConvWgradDesc), C.c_int, C.c_void_p,
                                          C.c_int64, C.c_void_p]),
    "vits_gate_forward": (
        C.c_int,
        [C.c_void_p, C.c_int64, C.c_int32, C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_int32,
         C.c_int, C.c_int, C.c_int, C.c_void_p],
    ),
    "vits_gate_backward": (
        C.c_int,
        [C.c_void_p, C.c_int64, C.c_int32, C.c_void_p, C.c_int64, C.c_int32, C.c_void_p, C.c_int64,
         C.c_void_p, C.c_int64, C.c_int32, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p],
    ),
    "vits_resblock_pair_forward": (
        C.c_int, [C.POINTER(ResblockPairDesc), C.c_int, C.c_int, C.c_void_p]),
    "vits_resblock_pair_f32p_forward": (
        C.c_int, [C.POINTER(ResblockPairDesc), C.c_int, C.c_int, C.c_void_p]),
    "vits_resblock_pair_kc": (
        C.c_int, [C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "vits_resblock_pair16_forward": (
        C.c_int, [C.POINTER(ResblockPairDesc), C.c_int, C.c_int, C.c_int, C.c_void_p]),
    "vits_resblock_pair16_mean_forward": (
        C.c_int, [C.POINTER(ResblockPairDesc), C.c_int, C.c_int, C.c_int, C.c_void_p]),
    "vits_gate_forward_io16": (
        C.c_int,
        [C.c_void_p, C.c_int64, C.c_int32, C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_int32,
         C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p],
    ),
    "vits_gate_backward_io16": (
        C.c_int,
        [C.c_void_p, C.c_int64, C.c_int32, C.c_void_p, C.c_int64, C.c_int32, C.c_void_p, C.c_int64,
         C.c_void_p, C.c_int64, C.c_int32, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int,
         C.c_void_p],
    ),
    "vits_gate_backward_io16_multi": (
        C.c_int, [C.POINTER(GateBwdJob), C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p]),
    "vits_radam_step": (
        C.c_int,
        [C.POINTER(RadamTensor), C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_double,
         C.c_void_p] + [C.c_double] * 4 + [C.c_void_p],
    ),
    "vits_weight_norm_forward": (
        C.c_int, [C.POINTER(WnormLayer), C.c_int, C.c_void_p, C.c_void_p]),
    "vits_weight_norm_backward": (
        C.c_int, [C.POINTER(WnormLayer), C.c_int, C.c_void_p, C.c_void_p]),
    "vits_spectral_norm_supported": (C.c_int, [C.c_int, C.c_int]),
    "vits_spectral_norm_forward": (
        C.c_int, [C.POINTER(SnormLayer), C.c_int, C.c_int, C.c_int, C.c_void_p]),
    "vits_spectral_norm_workspace": (C.c_int64, [C.POINTER(SnormLayer), C.c_int]),
    "vits_spectral_norm_backward": (
        C.c_int, [C.POINTER(SnormLayer), C.c_int, C.c_int, C.c_void_p, C.c_int64, C.c_void_p]),
    "vits_wn_update_forward": (
        C.c_int, [C.c_void_p] * 7 + [C.c_int] * 4 + [C.c_void_p]),
    "vits_wn_update_backward": (
        C.c_int, [C.c_void_p] * 6 + [C.c_int] * 4 + [C.c_void_p]),
    "vits_mask_cast_forward": (C.c_int, [C.c_void_p] * 4 + [C.c_int] * 4 + [C.c_void_p]),
    "vits_mask_cast_backward": (C.c_int, [C.c_void_p] * 4 + [C.c_int] * 4 + [C.c_void_p]),
    "vits_wn_final_forward": (C.c_int, [C.c_void_p] * 4 + [C.c_int] * 4 + [C.c_void_p]),
    "vits_wn_final_backward": (C.c_int, [C.c_void_p] * 4 + [C.c_int] * 4 + [C.c_void_p]),
    "vits_coupling_forward": (C.c_int, [C.c_void_p] * 4 + [C.c_int] * 6 + [C.c_void_p]),
    "vits_coupling_backward": (C.c_int, [C.c_void_p] * 4 + [C.c_int] * 6 + [C.c_void_p]),
    "vits_stftd_join_to_cl_forward": (
        C.c_int, [C.c_void_p] * 2 + [C.c_int] * 6 + [C.c_float, C.c_int, C.c_void_p]),
    "vits_stftd_join_to_cl_backward": (
        C.c_int, [C.c_void_p] * 3 + [C.c_int] * 6 + [C.c_float, C.c_int, C.c_void_p]),
    "vits_bias_lrelu_forward": (
        C.c_int, [C.c_void_p] * 3 + [C.c_int64, C.c_int, C.c_float, C.c_int, C.c_void_p]),
    "vits_bias_lrelu_workspace": (C.c_int, [C.c_int64, C.c_int]),
    "vits_bias_lrelu_backward": (
        C.c_int, [C.c_void_p] * 5 + [C.c_int, C.c_int64, C.c_int, C.c_float, C.c_int,
                                     C.c_void_p]),
    "vits_amd_version": (C.c_char_p, []),
    "vits_amd_device_arch": (C.c_int, [C.c_char_p, C.c_int]),
    "vits_dispatch_count": (C.c_int64, [C.c_int]),
    "vits_dispatch_count_reset": (None, []),
}

EXPORTED_SYMBOLS = tuple(_SIGS.keys())


class VitsAmdError(RuntimeError):
    pass


# vits_dispatch_count families (include/vits_amd.h VITS_CNT_*)
CNT_NAMES = ("conv_f32", "conv_split", "conv_16", "wgrad_f32", "wgrad_16", "gate_f32",
             "gate_16", "resblock", "pack")


def dispatch_counts() -> dict:
    """{family: kernel launches since the last reset} of the library."""
    lib = load()
    return {n: int(lib.vits_dispatch_count(i)) for i, n in enumerate(CNT_NAMES)}


def dispatch_counts_reset() -> None:
    load().vits_dispatch_count_reset()


def lib_path() -> str:
    return _LIB_PATH


def load():
    """Load (once) and return the ctypes library; raises if unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(_LIB_PATH):
            raise VitsAmdError(
                f"libvits_amd.so not found at {_LIB_PATH}; run __graft_entry__.build() "
                "(make -C vits_amd/csrc). There is no CPU fallback."
            )
        lib = C.CDLL(_LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def check(rc: int, what: str):
    if rc != VITS_OK:
        kind = {VITS_E_ARG: "bad argument", VITS_E_SHAPE: "shape mismatch",
                VITS_E_UNSUP: "unsupported configuration"}.get(rc, f"HIP error {rc}")
        raise VitsAmdError(f"{what}: {kind} (rc={rc})")
