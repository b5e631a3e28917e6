"""The drop-in boundary: libeazy_amd.so loads (without a GPU too) and exports
every entry point include/eazy.h declares; compute entry points fail loudly
without a device (no CPU fallback).  CPU only."""

import ctypes
import os
import subprocess

import pytest

import eazy_amd as ez

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_header_symbols():
    lib = ez._lib()
    names = ez.exported_symbols()
    assert len(names) >= 30
    for n in names:
        assert hasattr(lib, n), n
    out = subprocess.run(["nm", "-D", "--defined-only", ez.LIB_PATH], capture_output=True, text=True).stdout
    for n in names:
        assert f" T {n}\n" in out, n


def test_header_is_plain_c():
    # the header must compile as C99 with no HIP/torch types
    src = os.path.join(ROOT, "include", "eazy.h")
    r = subprocess.run(["gcc", "-std=c99", "-fsyntax-only", "-Wall", "-Werror", "-x", "c", src], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_compress_bound():
    for n in (0, 1, 100, 4096, 1 << 20):
        assert ez.compress_bound(n) == n + (n >> 2) + 32


def test_no_cpu_fallback():
    if ez.device_count() > 0:
        pytest.skip("GPU present")
    with pytest.raises(ez.DeviceError):
        ez.Writer(None, 1 << 20, 1024)
    with pytest.raises(ez.DeviceError):
        ez.Reader(b=b"")
    lib = ez._lib()
    assert lib.ez_compress_batch(1 << 20, 1024, 0, None, None) == ez.EDEVICE
    assert lib.ez_decompress_batch(0, None, None, None) == ez.EDEVICE
    import numpy as np

    with pytest.raises(ez.DeviceError):
        ez.compress_batch_multi(b"abcdefgh" * 8, np.array([0, 64]), devices=[0, 0])
    with pytest.raises(ez.DeviceError):
        ez.decompress_batch_multi(b"\x80\x10\x14\x01a", np.array([0, 5]), np.array([0, 16]))


def test_writer_size_panics():
    # Writer.init writer.go:161-169 -> EZ_EINVAL, checked before any device use
    h = ctypes.c_void_p()
    for bs, hs in ((31, 16), (1 << 32, 16), (1024, 3)):
        assert ez._lib().ez_writer_new(bs, hs, 0, ctypes.byref(h)) == ez.EINVAL
