"""ctypes binding of the C oracle (oracle/eazy_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, always as the checker / CPU baseline, never as
the measured or shipped path.
"""

from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None

OK, EOF, ESHORTBUF, EUNEXPECTEDEOF, EOVERFLOW, EBADMAGIC, ENOMAGIC = 0, 1, 2, 3, 4, 5, 6
EBLOCKLIMIT, EUNSUPMETA, EUNSUPVER, EBREAK, EMISSEDMETA, EINVAL, ESINK = 7, 8, 9, 10, 11, 12, 13

_i64 = C.c_int64
_u8p = C.POINTER(C.c_uint8)
_i64p = C.POINTER(C.c_int64)


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _SO


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = C.CDLL(_SO)
        L.or_writer_new.restype = C.c_void_p
        L.or_writer_new.argtypes = [_i64, _i64]
        L.or_writer_free.argtypes = [C.c_void_p]
        L.or_writer_set_append_magic.argtypes = [C.c_void_p, C.c_int]
        L.or_writer_set_version.argtypes = [C.c_void_p, C.c_int]
        L.or_writer_set_flush_threshold.argtypes = [C.c_void_p, _i64]
        L.or_writer_set_sink_fault.argtypes = [C.c_void_p, _i64]
        L.or_writer_write.argtypes = [C.c_void_p, C.c_char_p, _i64, _i64p]
        L.or_writer_write_header.argtypes = [C.c_void_p]
        L.or_writer_write_break.argtypes = [C.c_void_p]
        L.or_writer_flush.argtypes = [C.c_void_p]
        L.or_writer_reset.argtypes = [C.c_void_p]
        L.or_writer_reset_size.argtypes = [C.c_void_p, _i64, _i64]
        L.or_writer_sink.restype = C.c_void_p
        L.or_writer_sink.argtypes = [C.c_void_p, _i64p]
        L.or_writer_sink_clear.argtypes = [C.c_void_p]
        L.or_writer_pos.restype = _i64
        L.or_writer_pos.argtypes = [C.c_void_p]
        L.or_writer_set_pos.argtypes = [C.c_void_p, _i64]
        L.or_reader_new_bytes.restype = C.c_void_p
        L.or_reader_new_bytes.argtypes = [C.c_char_p, _i64]
        L.or_reader_new.restype = C.c_void_p
        L.or_reader_new.argtypes = [C.c_int, _i64]
        L.or_reader_free.argtypes = [C.c_void_p]
        L.or_reader_src_append.argtypes = [C.c_void_p, C.c_char_p, _i64]
        L.or_reader_set.argtypes = [C.c_void_p, _i64, _i64, C.c_int, C.c_int]
        L.or_reader_read.argtypes = [C.c_void_p, C.c_void_p, _i64, _i64p]
        L.or_reader_reset_bytes.argtypes = [C.c_void_p, C.c_char_p, _i64]
        L.or_reader_reset.argtypes = [C.c_void_p, C.c_int, _i64]
        L.or_reader_detail.restype = _i64
        L.or_reader_detail.argtypes = [C.c_void_p]
        L.or_compress.argtypes = [_i64, _i64, C.c_int, C.c_int, C.c_char_p, _i64p, C.c_int, C.c_void_p, _i64, _i64p]
        L.or_decompress.argtypes = [C.c_char_p, _i64, _i64, C.c_void_p, _i64, _i64p, _i64p]
        L.or_batch_grain.restype = _i64
        L.or_batch_grain.argtypes = [_i64, C.c_int]
        L.or_compress_batch.argtypes = [_i64, _i64, C.c_void_p, C.c_void_p, _i64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        L.or_decompress_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, _i64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        for name in ("or_enc_tag", "or_enc_offset", "or_enc_meta"):
            getattr(L, name).argtypes = [_u8p, C.POINTER(C.c_size_t), _i64, _i64]
        L.or_dec_tag.argtypes = [C.c_char_p, _i64, _i64, C.POINTER(C.c_int), _i64p, _i64p]
        L.or_dec_offset.argtypes = [C.c_char_p, _i64, _i64, _i64, _i64p, _i64p]
        L.or_dec_meta.argtypes = [C.c_char_p, _i64, _i64, _i64p, _i64p, _i64p]
        _lib = L
    return _lib


class Panic(Exception):
    pass


def _enc(fn, a, b):
    buf = (C.c_uint8 * 32)()
    n = C.c_size_t(0)
    e = getattr(lib(), fn)(buf, C.byref(n), a, b)
    if e == EINVAL:
        raise Panic(fn)
    return C.string_at(buf, n.value)


def enc_tag(tag, l):
    return _enc("or_enc_tag", tag, l)


def enc_offset(off, l):
    return _enc("or_enc_offset", off, l)


def enc_meta(meta, l):
    return _enc("or_enc_meta", meta, l)


def dec_tag(b: bytes, st: int = 0):
    t, l, i = C.c_int(), _i64(), _i64()
    e = lib().or_dec_tag(b, len(b), st, C.byref(t), C.byref(l), C.byref(i))
    return t.value, l.value, i.value, e


def dec_offset(b: bytes, st: int, l: int):
    off, i = _i64(), _i64()
    e = lib().or_dec_offset(b, len(b), st, l, C.byref(off), C.byref(i))
    return off.value, i.value, e


def dec_meta(b: bytes, st: int):
    m, l, i = _i64(), _i64(), _i64()
    e = lib().or_dec_meta(b, len(b), st, C.byref(m), C.byref(l), C.byref(i))
    return m.value, l.value, i.value, e


class Writer:
    """eazy.Writer over the C oracle; the sink is an in-memory Buf."""

    def __init__(self, block, htable):
        self._w = lib().or_writer_new(block, htable)
        if not self._w:
            raise Panic("NewWriter")

    def __del__(self):
        if getattr(self, "_w", None):
            lib().or_writer_free(self._w)
            self._w = None

    append_magic = property(None, lambda s, v: lib().or_writer_set_append_magic(s._w, int(v)))
    ver = property(None, lambda s, v: lib().or_writer_set_version(s._w, int(v)))
    flush_threshold = property(None, lambda s, v: lib().or_writer_set_flush_threshold(s._w, int(v)))

    def sink_fault(self, accept):
        lib().or_writer_set_sink_fault(self._w, accept)

    def write(self, p: bytes):
        done = _i64()
        e = lib().or_writer_write(self._w, bytes(p), len(p), C.byref(done))
        if e == EINVAL:
            raise Panic("Write")
        return done.value, e

    def write_header(self):
        return lib().or_writer_write_header(self._w)

    def write_break(self):
        return lib().or_writer_write_break(self._w)

    def flush(self):
        return lib().or_writer_flush(self._w)

    def reset(self):
        lib().or_writer_reset(self._w)

    def reset_size(self, block, htable):
        if lib().or_writer_reset_size(self._w, block, htable) == EINVAL:
            raise Panic("ResetSize")

    @property
    def sink(self) -> bytes:
        n = _i64()
        p = lib().or_writer_sink(self._w, C.byref(n))
        return C.string_at(p, n.value) if n.value else b""

    def sink_clear(self):
        lib().or_writer_sink_clear(self._w)

    @property
    def pos(self):
        return lib().or_writer_pos(self._w)

    def set_pos(self, pos: int) -> None:  # testing hook
        lib().or_writer_set_pos(self._w, pos)


class Reader:
    """eazy.Reader over the C oracle.  Reader(b=...) is NewReaderBytes;
    Reader(src=...) is NewReader over an in-memory io.Reader."""

    def __init__(self, b: bytes | None = None, src: bytes | None = None, eof_with_data=True, chunk=0):
        if src is None:
            self._r = lib().or_reader_new_bytes(bytes(b or b""), len(b or b""))
        else:
            self._r = lib().or_reader_new(int(eof_with_data), chunk)
            self.append(src)

    def __del__(self):
        if getattr(self, "_r", None):
            lib().or_reader_free(self._r)
            self._r = None

    def append(self, b: bytes):
        lib().or_reader_src_append(self._r, bytes(b), len(b))

    def set(self, block_size_limit, buffer_size, require_magic=False, skip_unsupported_meta=False):
        lib().or_reader_set(self._r, block_size_limit, buffer_size, int(require_magic), int(skip_unsupported_meta))

    def read(self, n: int):
        buf = (C.c_uint8 * max(n, 1))()
        got = _i64()
        e = lib().or_reader_read(self._r, buf, n, C.byref(got))
        return C.string_at(buf, got.value), e

    def reset_bytes(self, b: bytes):
        lib().or_reader_reset_bytes(self._r, bytes(b), len(b))

    def reset(self, src: bytes = b"", eof_with_data=True, chunk=0):
        lib().or_reader_reset(self._r, int(eof_with_data), chunk)
        self.append(src)


def compress(block, htable, writes, append_magic=True, ver=0) -> bytes:
    data = b"".join(bytes(w) for w in writes)
    lens = (_i64 * max(len(writes), 1))(*[len(w) for w in writes])
    cap = len(data) + len(data) // 4 + 64 * (len(writes) + 1)
    out = (C.c_uint8 * cap)()
    n = _i64()
    e = lib().or_compress(block, htable, int(append_magic), ver, data, lens, len(writes), out, cap, C.byref(n))
    if e:
        raise RuntimeError(f"or_compress: {e}")
    return C.string_at(out, n.value)


def decompress(b: bytes, buf_size: int = 1 << 16, cap: int | None = None):
    cap = cap if cap is not None else max(1 << 20, 64 * len(b))
    out = (C.c_uint8 * cap)()
    n, nb = _i64(), _i64()
    e = lib().or_decompress(bytes(b), len(b), buf_size, out, cap, C.byref(n), C.byref(nb))
    return C.string_at(out, n.value), e, nb.value


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def batch_grain(count: int, nthreads: int) -> int:
    """Streams per task of the threaded batch runners."""
    return int(lib().or_batch_grain(count, nthreads))


def compress_batch(block, htable, data: np.ndarray, offs: np.ndarray, slot_offs: np.ndarray, nthreads: int):
    count = len(offs) - 1
    slots = np.zeros(int(slot_offs[-1]), np.uint8)
    sizes = np.zeros(count, np.int64)
    e = lib().or_compress_batch(block, htable, _ptr(data), _ptr(offs), count, _ptr(slots), _ptr(slot_offs), _ptr(sizes), nthreads)
    if e:
        raise RuntimeError(f"or_compress_batch: {e}")
    return slots, sizes


def decompress_batch(comp: np.ndarray, comp_offs: np.ndarray, comp_sizes: np.ndarray, out_offs: np.ndarray, nthreads: int):
    count = len(comp_sizes)
    out = np.zeros(int(out_offs[-1]), np.uint8)
    sizes = np.zeros(count, np.int64)
    e = lib().or_decompress_batch(_ptr(comp), _ptr(comp_offs), _ptr(comp_sizes), count, _ptr(out), _ptr(out_offs), _ptr(sizes), nthreads)
    if e:
        raise RuntimeError(f"or_decompress_batch: {e}")
    return out, sizes
