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


def global_logs(seed: int, first: int, last: int, size: int, chunk: int = 65536) -> np.ndarray:
    """Streams [first, last) of a global batch of `size`-byte log streams whose
    chunk k (streams k*chunk .. (k+1)*chunk-1) is logs(seed + k, chunk*size):
    every rank of a sharded run generates exactly its own streams, and the
    bytes do not depend on the number of ranks."""
    out = np.empty((last - first) * size, np.uint8)
    at = 0
    for k in range(first // chunk, (last + chunk - 1) // chunk):
        c = logs(seed + k, chunk * size)
        a, b = max(first, k * chunk) - k * chunk, min(last, (k + 1) * chunk) - k * chunk
        out[at : at + (b - a) * size] = c[a * size : b * size]
        at += (b - a) * size
    return out
