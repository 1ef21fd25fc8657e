"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of oracle/mas_oracle.c plus a
brute-force enumerator used to pin it (no reference fixture exists for the
external monotonic_align package)."""
from __future__ import annotations

import ctypes as C
import itertools
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "build", "libmas_oracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        lib = C.CDLL(_SO)
        lib.mas_oracle_maximum_path.restype = None
        lib.mas_oracle_maximum_path.argtypes = [C.c_void_p] * 4 + [C.c_int] * 3
        lib.mas_oracle_maximum_path_mt.restype = None
        lib.mas_oracle_maximum_path_mt.argtypes = [C.c_void_p] * 4 + [C.c_int] * 4
        _lib = lib
    return _lib


def maximum_path_lengths(neg_cent: np.ndarray, t_t: np.ndarray, t_s: np.ndarray) -> np.ndarray:
    """neg_cent [B, T_t, T_s] -> int32 path, DP on a float32 copy."""
    vals = np.ascontiguousarray(neg_cent, dtype=np.float32).copy()
    B, Tt, Ts = vals.shape
    path = np.zeros((B, Tt, Ts), dtype=np.int32)
    tt = np.ascontiguousarray(t_t, dtype=np.int32)
    ts = np.ascontiguousarray(t_s, dtype=np.int32)
    _load().mas_oracle_maximum_path(path.ctypes.data, vals.ctypes.data, tt.ctypes.data,
                                    ts.ctypes.data, B, Tt, Ts)
    return path


def maximum_path_lengths_mt(neg_cent: np.ndarray, t_t: np.ndarray, t_s: np.ndarray,
                            threads: int) -> np.ndarray:
    """maximum_path_lengths with the batch over `threads` OpenMP threads."""
    vals = np.ascontiguousarray(neg_cent, dtype=np.float32).copy()
    B, Tt, Ts = vals.shape
    path = np.empty((B, Tt, Ts), dtype=np.int32)
    tt = np.ascontiguousarray(t_t, dtype=np.int32)
    ts = np.ascontiguousarray(t_s, dtype=np.int32)
    _load().mas_oracle_maximum_path_mt(path.ctypes.data, vals.ctypes.data, tt.ctypes.data,
                                       ts.ctypes.data, B, Tt, Ts, int(threads))
    return path


def maximum_path(neg_cent: np.ndarray, mask: np.ndarray) -> np.ndarray:
    """Same contract as monotonic_align.maximum_path on numpy inputs."""
    mask = np.asarray(mask)
    t_t = mask.sum(1)[:, 0].astype(np.int32)
    t_s = mask.sum(2)[:, 0].astype(np.int32)
    return maximum_path_lengths(neg_cent, t_t, t_s)


def brute_force(value: np.ndarray, t_y: int, t_x: int):
    """All monotone surjective alignments of t_y frames onto t_x tokens
    (token index non-decreasing by steps of 0/1, starting at 0, ending at
    t_x-1).  Returns (best score in float64, list of argmax paths)."""
    best, paths = -np.inf, []
    # choose the t_x - 1 frames (in 1..t_y-1) where the token index advances
    for cuts in itertools.combinations(range(1, t_y), t_x - 1):
        idx = np.zeros(t_y, dtype=np.int64)
        for c in cuts:
            idx[c:] += 1
        s = float(np.sum(value[np.arange(t_y), idx].astype(np.float64)))
        if s > best + 1e-12:
            best, paths = s, [idx]
        elif abs(s - best) <= 1e-12:
            paths.append(idx)
    return best, paths
