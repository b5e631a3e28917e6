"""Seeded synthetic inputs (tests and bench.py only; not part of the codec).

``logs`` — tlwire-like log events (eazy_test.go:1273-1282
framing); ``f32`` — N(0, sigma) float32 gradient-like buckets (config C4).
"""

from __future__ import annotations

import ctypes as C
import os

import numpy as np

_SO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libeazy_synth.so")
_L = None


def _lib():
    global _L
    if _L is None:
        _L = C.CDLL(_SO)
        _L.ez_synth_logs.argtypes = [C.c_uint64, C.c_void_p, C.c_uint64]
        _L.ez_synth_f32.argtypes = [C.c_uint64, C.c_float, C.c_void_p, C.c_uint64]
    return _L


def logs(seed: int, n: int) -> np.ndarray:
    out = np.empty(n, np.uint8)
    _lib().ez_synth_logs(seed, out.ctypes.data, n)
    return out


def f32(seed: int, count: int, sigma: float = 1e-3) -> np.ndarray:
    out = np.empty(count, np.float32)
    _lib().ez_synth_f32(seed, sigma, out.ctypes.data, count)
    return out


def batch_offsets(count: int, size: int) -> np.ndarray:
    return np.arange(count + 1, dtype=np.int64) * size
