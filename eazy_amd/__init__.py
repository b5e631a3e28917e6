"""eazy_amd — MI355X-native eazy codec: Python binding of include/eazy.h.

The shipped path is libeazy_amd.so (gfx950 HIP kernels behind a C-ABI).
This module is a thin ctypes layer over it:

* ``Writer`` / ``Reader`` mirror the reference's streaming types
  (writer.go:17-46, reader.go:17-40) with the same field names, flush policy
  and error values; their compression / decompression runs on the GPU.
* ``compress_batch`` / ``pack`` / ``decompress_batch`` drive the batched,
  device-resident kernels (K1/K3/K2) on torch CUDA tensors.
* ``Encoder`` / ``Decoder`` expose the token codec (writer.go:537-621,
  reader.go:346-514).

There is no CPU fallback: importing works without a GPU (for the build and
symbol checks), but every compute call raises ``DeviceError`` when the HIP
runtime has no MI355X.
"""

from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("EZ_LIB") or os.path.join(_HERE, "libeazy_amd.so")  # EZ_LIB: experiment builds

# ---- constants (writer.go:49-122) ----
B, KiB, MiB, GiB = 1, 1 << 10, 1 << 20, 1 << 30
Literal, Copy, Meta, Padding = 0x00, 0x80, 0x80, 0x00
TagMask, TagLenMask = 0x80, 0x7F
Len1, Len2, Len4, LenAlt = 124, 125, 126, 127
Off1, Off2, Off4, OffAlt = 252, 253, 254, 255
OffLong = OffAlt
MetaMagic, MetaVer, MetaReset, MetaBreak = 0x00, 0x08, 0x10, 0x18
MetaTagMask, MetaLenMask, MetaLenWide, MetaLen0 = 0xF8, 0x07, 6, 7
Magic = b"\x80\x02eazy"
Version = 0

# ---- status codes (include/eazy.h) ----
OK, EOF, ESHORTBUF, EUNEXPECTEDEOF, EOVERFLOW, EBADMAGIC, ENOMAGIC = 0, 1, 2, 3, 4, 5, 6
EBLOCKLIMIT, EUNSUPMETA, EUNSUPVER, EBREAK, EMISSEDMETA, EINVAL = 7, 8, 9, 10, 11, 12
ESINK, ENOSPC, EDEVICE, ESTUCK = 13, 14, 15, 16
F_NO_MAGIC = 0x1


class EazyError(Exception):
    code = -1

    def __init__(self, code: int, detail: int = 0):
        self.code = code
        self.detail = detail
        super().__init__(f"{_strerror(code)}" + (f": {detail:#x}" if detail else ""))


class DeviceError(EazyError):
    """No usable MI355X (or a HIP runtime error) — there is no CPU fallback."""


class Panic(EazyError):
    """Where the reference panics (bad sizes, too big length/offset, bad meta); str() is
    the reference's panic value when known (writer.go:163, 167, 309, 562, 596)."""

    def __init__(self, code: int = 12, detail: int = 0, message: str | None = None):
        super().__init__(code, detail)
        if message is not None:
            self.args = (message,)


def _size_panic(block: int, htable: int) -> None:
    """Writer.init writer.go:161-169: the reference's panic for invalid sizes."""
    p = _lib().ez_writer_size_panic(block, htable)
    if p:
        raise Panic(12, message=_lib().ez_panic_message(p).decode())


def _strerror(code: int) -> str:
    try:
        return _lib().ez_strerror(code).decode()
    except OSError:
        return f"code {code}"


_L = None


def _lib():
    global _L
    if _L is not None:
        return _L
    if not os.path.exists(LIB_PATH):
        raise OSError(f"{LIB_PATH} missing: run __graft_entry__.build() (make -C eazy_amd)")
    L = C.CDLL(LIB_PATH)
    sz, i64, u8p, vp = C.c_size_t, C.c_int64, C.POINTER(C.c_uint8), C.c_void_p
    L.ez_strerror.restype = C.c_char_p
    L.ez_strerror.argtypes = [C.c_int]
    L.ez_compress_bound.restype = sz
    L.ez_compress_bound.argtypes = [sz]
    for f in ("ez_encode_tag", "ez_encode_offset", "ez_encode_meta"):
        getattr(L, f).argtypes = [u8p, sz, C.POINTER(sz), i64, i64]
    L.ez_encode_tag.argtypes = [u8p, sz, C.POINTER(sz), C.c_int, i64]
    L.ez_decode_tag.argtypes = [C.c_char_p, sz, sz, C.POINTER(C.c_int), C.POINTER(i64), C.POINTER(sz)]
    L.ez_decode_offset.argtypes = [C.c_char_p, sz, sz, i64, C.POINTER(i64), C.POINTER(sz)]
    L.ez_decode_meta.argtypes = [C.c_char_p, sz, sz, C.POINTER(i64), C.POINTER(i64), C.POINTER(sz)]
    L.ez_writer_new.argtypes = [i64, i64, C.c_int, C.POINTER(vp)]
    L.ez_writer_free.argtypes = [vp]
    L.ez_writer_set_append_magic.argtypes = [vp, C.c_int]
    L.ez_writer_set_version.argtypes = [vp, C.c_int]
    L.ez_writer_write.argtypes = [vp, C.c_char_p, sz, vp, sz, C.POINTER(sz)]
    L.ez_writer_write_batch.argtypes = [vp, C.c_char_p, vp, sz, vp, sz, vp]
    L.ez_writer_header.argtypes = [vp, vp, sz, C.POINTER(sz)]
    L.ez_writer_break.argtypes = [vp, vp, sz, C.POINTER(sz)]
    L.ez_writer_reset.argtypes = [vp]
    L.ez_writer_reset_size.argtypes = [vp, i64, i64]
    L.ez_writer_is_reset.argtypes = [vp]
    L.ez_writer_last_panic.argtypes = [vp]
    L.ez_reader_set_whole.argtypes = [vp, C.c_int]
    L.ez_reader_whole_decoded.argtypes = [vp]
    L.ez_writer_size_panic.argtypes = [i64, i64]
    L.ez_panic_message.restype = C.c_char_p
    L.ez_panic_message.argtypes = [C.c_int]
    L.ez_reader_new.argtypes = [C.c_int, C.POINTER(vp)]
    L.ez_reader_free.argtypes = [vp]
    L.ez_reader_configure.argtypes = [vp, i64, C.c_int, C.c_int]
    L.ez_reader_reset.argtypes = [vp]
    L.ez_reader_pending.argtypes = [vp]
    L.ez_reader_read.argtypes = [vp, vp, sz, sz, i64, vp, sz, C.POINTER(sz), C.POINTER(sz), C.POINTER(i64)]
    L.ez_compress_batch.argtypes = [i64, i64, C.c_int, vp, vp]
    L.ez_pack_workspace.restype = sz
    L.ez_pack_workspace.argtypes = [C.c_uint64]
    L.ez_pack_batch.argtypes = [vp, vp, vp, C.c_uint64, vp, vp, vp, vp]
    L.ez_decompress_workspace.restype = sz
    L.ez_decompress_workspace.argtypes = [C.c_uint64]
    L.ez_decompress_batch.argtypes = [i64, vp, vp, vp]
    _L = L
    return L


def exported_symbols() -> list[str]:
    """Names declared in include/eazy.h that the library must export."""
    import re

    hdr = open(os.path.join(_HERE, "..", "include", "eazy.h")).read()
    return sorted(set(re.findall(r"\b(ez_[a-z_0-9]+)\s*\(", hdr)))


def device_count() -> int:
    return _lib().ez_device_count()


def compress_kernel(block: int, htable: int, max_len: int, count: int) -> str:
    """The K1 kernel a batch of `count` fresh streams of <= max_len bytes runs
    on the current device ('s' K1s: parse + token writer, 'x' K1x's data-parallel rounds
    then the general kernel, 'w' general wave per stream)."""
    L = _lib()
    L.ez_compress_kernel.argtypes = [C.c_int64, C.c_int64, C.c_uint64, C.c_uint64]
    v = L.ez_compress_kernel(block, htable, max_len, count)
    if v < 0:
        _check(-v)
    return chr(v)


def select_compress_kernel(kind: str = "") -> None:
    """Force the K1 kernel of later batch calls ('s' K1s, 'S' K1s with the u32
    exchange table, 'w' general alone, 'x' K1x's rounds for any fresh single-Write batch,
    'l' K1L (the lean parse with the window's ring semantics) alone;
    '' = automatic).  Tests and A/B measurement only."""
    _check(_lib().ez_select_compress_kernel(ord(kind) if kind else 0))


def select_decompress_kernel(kind: str = "") -> None:
    """Force the first K2 kernel of later batch decodes ('r' ring, 't' token-parallel wave per
    stream, 'w' wave per stream; '' = automatic).  Tests and A/B measurement only."""
    _check(_lib().ez_select_decompress_kernel(ord(kind) if kind else 0))


def decompress_kernel_last() -> str:
    """The first K2 kernel the last batch decode of this process ran ('r', 't', 'w'; 'e' the
    exact decoder alone; '' none yet)."""
    v = _lib().ez_decompress_kernel_last()
    return chr(v) if v else ""


def k1c_stats(enable: bool) -> dict:
    """K1c's verdict counts so far (streams proven; fallen back to K1L for a chunk error or
    re-visit, no common copy end, a changed judgement, the record slot; path segments), then
    counting on (cleared) or off.  While on, each K1c batch waits for its verdicts.  Tests only."""
    out = (C.c_uint64 * 6)()
    _check(_lib().ez_compress_k1c_stats(1 if enable else 0, out))
    return dict(zip(("proven", "chunk", "sync", "judge", "cap", "segments"), (int(v) for v in out)))


def release_cached(device: int = -1) -> None:
    """ez_release_cached: free the device scratch kept between batch calls (device < 0: all)."""
    _check(_lib().ez_release_cached(device))


def multi_last_shards() -> list:
    """ez_multi_last_shards: [(device, t0_ms, t1_ms)] of the last multi-device batch call's shards."""
    L = _lib()
    L.ez_multi_last_shards.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
    n = L.ez_multi_last_shards(None, None, None, 0)
    dev = (C.c_int * max(n, 1))()
    t0 = (C.c_double * max(n, 1))()
    t1 = (C.c_double * max(n, 1))()
    n = L.ez_multi_last_shards(dev, t0, t1, n)
    return [(dev[k], t0[k], t1[k]) for k in range(n)]


def _check(code: int, detail: int = 0) -> None:
    if code == OK:
        return
    if code == EDEVICE:
        raise DeviceError(code)
    if code == EINVAL:
        raise Panic(code)
    raise EazyError(code, detail)


def compress_bound(n: int) -> int:
    return _lib().ez_compress_bound(n)


# ---------------------------------------------------------------- token codec


class Encoder:
    """Low-level encoder (writer.go:10-15, 537-621)."""

    def __init__(self, ver: int = 0):
        self.Ver = ver

    @staticmethod
    def _enc(fn, *args) -> bytes:
        buf = (C.c_uint8 * 32)()
        n = C.c_size_t(0)
        _check(getattr(_lib(), fn)(buf, 32, C.byref(n), *args))
        return C.string_at(buf, n.value)

    def tag(self, b: bytes, tag: int, l: int) -> bytes:
        return bytes(b) + self._enc("ez_encode_tag", tag, l)

    def offset(self, b: bytes, off: int, l: int) -> bytes:
        return bytes(b) + self._enc("ez_encode_offset", off, l)

    def meta(self, b: bytes, meta: int, l: int) -> bytes:
        return bytes(b) + self._enc("ez_encode_meta", meta, l)


class Decoder:
    """Low-level decoder (reader.go:10-15, 346-514): returns Go's results, err as code."""

    def __init__(self, ver: int = 0):
        self.Ver = ver

    def tag(self, b: bytes, st: int):
        t, l, i = C.c_int(), C.c_int64(), C.c_size_t()
        e = _lib().ez_decode_tag(bytes(b), len(b), st, C.byref(t), C.byref(l), C.byref(i))
        return t.value, l.value, i.value, e

    def offset(self, b: bytes, st: int, l: int):
        off, i = C.c_int64(), C.c_size_t()
        e = _lib().ez_decode_offset(bytes(b), len(b), st, l, C.byref(off), C.byref(i))
        return off.value, i.value, e

    def meta(self, b: bytes, st: int):
        m, l, i = C.c_int64(), C.c_int64(), C.c_size_t()
        e = _lib().ez_decode_meta(bytes(b), len(b), st, C.byref(m), C.byref(l), C.byref(i))
        return m.value, l.value, i.value, e


# ---------------------------------------------------------------- Writer


class Writer:
    """eazy.Writer (writer.go:17-46): NewWriter(wr, block, htable).

    ``wr`` is an io.Writer-like object whose ``write(bytes)`` returns the
    number of bytes taken (or raises).  One Write -> one wr.write (with
    FlushThreshold 0), header on the first Write, a failed or short sink
    write resets the stream (writer.go:387-401).
    """

    def __init__(self, wr, block: int, htable: int, device: int = 0):
        _size_panic(block, htable)
        h = C.c_void_p()
        _check(_lib().ez_writer_new(block, htable, device, C.byref(h)))
        self._h = h
        self.Writer = wr
        self._append_magic = True
        self.FlushThreshold = 0
        self._ver = 0
        self._b = bytearray()
        self._written = 0
        self._resets = 0

    def __del__(self):
        if getattr(self, "_h", None):
            _lib().ez_writer_free(self._h)
            self._h = None

    @property
    def AppendMagic(self) -> bool:
        return self._append_magic

    @AppendMagic.setter
    def AppendMagic(self, on: bool) -> None:
        self._append_magic = bool(on)
        _lib().ez_writer_set_append_magic(self._h, int(bool(on)))

    @property
    def Ver(self) -> int:  # w.e.Ver
        return self._ver

    @Ver.setter
    def Ver(self, v: int) -> None:
        self._ver = int(v)
        _lib().ez_writer_set_version(self._h, int(v))

    def _call(self, fn, *args, cap: int) -> bytes:
        buf = (C.c_uint8 * max(cap, 1))()
        n = C.c_size_t()
        _check(fn(self._h, *args, buf, cap, C.byref(n)))
        return C.string_at(buf, n.value)

    def Write(self, p: bytes) -> int:  # writer.go:206-337
        p = bytes(p)
        try:
            b = self._call(_lib().ez_writer_write, p, len(p), cap=compress_bound(len(p)))
        except EazyError as e:
            raise self._failed(e) from None
        self._b += b
        self._write()
        return len(p)

    def _failed(self, e: EazyError) -> EazyError:
        """A failed Write: when the device history had taken it, the handle restarted its stream
        (it is reset now) and the mirror forgets w.b and written too; a failure found before
        anything reached the device (ENOSPC, bad Write ends, no device) leaves both as they
        were.  An EZ_EINVAL with a reference panic behind it carries that panic's value."""
        if _lib().ez_writer_is_reset(self._h):
            self._resets += 1
            self._b = bytearray()
            self._written = 0
        if isinstance(e, Panic):
            p = _lib().ez_writer_last_panic(self._h)
            if p != 0:  # EZ_PANIC_NONE: an invalid argument, not a reference panic
                return Panic(EINVAL, message=_lib().ez_panic_message(p).decode())
        return e

    def WriteBatch(self, ps) -> int:
        """Several Writes in one device call (no reference counterpart; a throughput form of
        Write for small Writes): the sink sees exactly what ``for p in ps: Write(p)`` gives it
        — the same calls with the same bytes, FlushThreshold applied after each Write, the
        first error raised — because the handle returns where each Write's bytes end and the
        flushes are replayed per Write.  When a short sink write restarts the stream
        (writer.go:391-393) the remaining Writes go through Write on the new stream.
        Returns the bytes of all Writes."""
        ps = [bytes(p) for p in ps]
        k = len(ps)
        if k == 0:
            return 0
        ends = (C.c_uint64 * k)()
        at = 0
        for j, p in enumerate(ps):
            at += len(p)
            ends[j] = at
        cap = sum(compress_bound(len(p)) for p in ps)
        buf = (C.c_uint8 * max(cap, 1))()
        oe = (C.c_uint64 * k)()
        try:
            _check(_lib().ez_writer_write_batch(self._h, b"".join(ps), ends, k, buf, cap, oe))
        except EazyError as e:
            raise self._failed(e) from None
        out = C.string_at(buf, oe[k - 1])
        prev, gen = 0, self._resets
        for j in range(k):
            self._b += out[prev : oe[j]]
            prev = oe[j]
            self._write()
            if self._resets != gen:  # the stream restarted: the rest on the new stream
                for p in ps[j + 1 :]:
                    self.Write(p)
                break
        return at

    def WriteHeader(self) -> None:  # writer.go:342-350
        if not _lib().ez_writer_is_reset(self._h):
            return
        self._b += self._call(_lib().ez_writer_header, cap=32)
        self._write()

    def WriteBreak(self) -> None:  # writer.go:358-366
        self._b += self._call(_lib().ez_writer_break, cap=32)
        self._write()

    def Flush(self) -> None:  # writer.go:371-377
        if self._b:
            self._flush()

    def Reset(self, wr) -> None:  # writer.go:149-152
        self.Writer = wr
        self._reset()

    def ResetSize(self, wr, block: int, htable: int) -> None:  # writer.go:155-159
        self.Writer = wr
        _size_panic(block, htable)
        _check(_lib().ez_writer_reset_size(self._h, block, htable))
        self._b = bytearray()
        self._written = 0

    def _reset(self) -> None:  # writer.go:187-200
        self._resets += 1
        _check(_lib().ez_writer_reset(self._h))
        self._b = bytearray()
        self._written = 0

    def _write(self) -> None:  # writer.go:379-385
        if self.FlushThreshold < 0 or len(self._b) < self.FlushThreshold:
            return
        self._flush()

    def _flush(self) -> None:  # writer.go:387-401
        try:
            n = self.Writer.write(bytes(self._b))
            err = None
        except Exception as e:  # noqa: BLE001 - any sink error resets the stream
            n, err = getattr(e, "n", 0), e
        n = len(self._b) if n is None else n
        self._written += n
        if err is not None or n != len(self._b):
            self._reset()
        if err is not None:
            raise err
        self._b = bytearray()


def NewWriter(wr, block: int, htable: int, device: int = 0) -> Writer:
    return Writer(wr, block, htable, device)


# ---------------------------------------------------------------- Reader


class Reader:
    """eazy.Reader (reader.go:17-40).  NewReader(r) / NewReaderBytes(b).

    ``Read(n)`` returns ``(data, err)`` with err one of the status codes
    (OK, EOF, EBREAK, ...), exactly the (n, err) pair of Go's Read.
    ``r`` is either an object with ``read_go(k) -> (bytes, err_code)`` (Go
    io.Reader semantics, e.g. data together with EOF) or a Python file-like
    whose ``read(k)`` returns b"" at EOF.
    """

    def __init__(self, r=None, b: bytes | None = None, device: int = 0):
        h = C.c_void_p()
        _check(_lib().ez_reader_new(device, C.byref(h)))
        self._h = h
        _lib().ez_reader_set_whole(h, 0 if r is not None else 1)  # a whole buffer: decoded at once
        self.Reader = r
        self._b = bytearray(b or b"")
        self._bcap = len(self._b)  # cap(r.b)
        self._i = 0
        self._boff = 0
        self.BlockSizeLimit = 16 * MiB if r is not None else 0
        self.BufferSize = 64 * 1024 if r is not None else 0
        self.RequireMagic = False
        self.SkipUnsupportedMeta = False
        self.detail = 0

    def __del__(self):
        if getattr(self, "_h", None):
            _lib().ez_reader_free(self._h)
            self._h = None

    def Reset(self, rd) -> None:  # reader.go:96-99
        self.ResetBytes(b"")
        self.Reader = rd
        _lib().ez_reader_set_whole(self._h, 0)

    def ResetBytes(self, b: bytes) -> None:  # reader.go:102-113
        self.Reader = None
        self._b = bytearray(b)
        self._bcap = len(self._b)
        self._i = 0
        self._boff = 0
        _lib().ez_reader_reset(self._h)
        _lib().ez_reader_set_whole(self._h, 1)

    @property
    def whole_decoded(self) -> bool:
        """True while the Reads are served from the whole-stream decode (ez_reader_whole_decoded)."""
        return bool(_lib().ez_reader_whole_decoded(self._h))

    @property
    def ahead_count(self) -> int:
        """Read-aheads this NewReader(io.Reader) handle has made (ez_reader_ahead_count)."""
        L = _lib()
        L.ez_reader_ahead_count.restype = C.c_int64
        L.ez_reader_ahead_count.argtypes = [C.c_void_p]
        return int(L.ez_reader_ahead_count(self._h))

    def Read(self, n: int):  # reader.go:116-141
        L = _lib()
        cfg = (self.BlockSizeLimit, int(self.RequireMagic), int(self.SkipUnsupportedMeta))
        if cfg != getattr(self, "_cfg", None):  # (the handle keeps it: one C call per change, not per Read)
            L.ez_reader_configure(self._h, *cfg)
            self._cfg = cfg
        p = C.create_string_buffer(max(n, 1))  # (bytes(p[:got]) of a c_uint8 array builds a list: 10x slower)
        got, err = 0, OK
        while got < n and err == OK:
            nb = len(self._b)
            bb = (C.c_uint8 * max(nb, 1)).from_buffer(self._b if nb else bytearray(1))  # no copy of r.b
            m, i, det = C.c_size_t(), C.c_size_t(), C.c_int64()
            err = L.ez_reader_read(self._h, bb, nb, self._i, self._boff,
                                   C.byref(p, got), n - got, C.byref(m), C.byref(i), C.byref(det))
            del bb  # release the export: more() resizes r.b
            if err == EDEVICE:
                raise DeviceError(err)
            got += m.value
            self._i = i.value
            self.detail = det.value
            if got == n:
                break
            if err != ESHORTBUF:
                continue
            err = self._more()
            if err == EOF and (L.ez_reader_pending(self._h) or self._i < len(self._b)):
                err = EUNEXPECTEDEOF
        return C.string_at(p, got), err

    def _more(self) -> int:  # reader.go:516-543
        if self.Reader is None:
            return EOF
        del self._b[: self._i]
        self._boff += self._i
        self._i = 0
        end = len(self._b)
        if end == 0:  # r.b = make([]byte, r.BufferSize)
            self._bcap = self.BufferSize
        else:  # r.b = append(r.b, make([]byte, 1024)...): the same array unless it has no room
            self._bcap = _go_append_cap(self._bcap, end + 1024)
        room = self._bcap - end  # r.Reader.Read(r.b[end:cap(r.b)])
        if hasattr(self.Reader, "read_go"):
            data, err = self.Reader.read_go(room)
        else:
            data = self.Reader.read(room)
            err = EOF if not data else OK
        self._b += data
        if data and err == EOF:
            err = OK
        return err


# Go's size classes (runtime/sizeclasses.go) and growslice for a byte slice (runtime/slice.go, Go 1.20,
# the reference's go.mod): the capacity append(r.b, make([]byte, 1024)...) leaves in more()
# (reader.go:529), which decides how much the next io.Reader.Read is offered.
_GO_CLASSES = (8, 16, 24, 32, 48, 64, 80, 96, 112, 128, 144, 160, 176, 192, 208, 224, 240, 256, 288, 320, 352, 384, 416,
               448, 480, 512, 576, 640, 704, 768, 896, 1024, 1152, 1280, 1408, 1536, 1792, 2048, 2304, 2688, 3072, 3200,
               3456, 4096, 4864, 5376, 6144, 6528, 6784, 6912, 8192, 9472, 9728, 10240, 10880, 12288, 13568, 14336,
               16384, 18432, 19072, 20480, 21760, 24576, 27264, 28672, 32768)


def _go_append_cap(old_cap: int, new_len: int) -> int:
    """cap(append(s, ...)) for a []byte of capacity old_cap grown to new_len elements."""
    if new_len <= old_cap:
        return old_cap
    newcap = old_cap
    if new_len > 2 * old_cap:
        newcap = new_len
    elif old_cap < 256:
        newcap = 2 * old_cap
    else:
        while 0 < newcap < new_len:
            newcap += (newcap + 3 * 256) // 4
        if newcap <= 0:
            newcap = new_len
    if newcap < 32768:  # roundupsize: the smallest size class, else whole 8 KiB pages
        return next(c for c in _GO_CLASSES if c >= newcap) if newcap > 0 else 0
    return (newcap + 8191) & ~8191


def NewReader(r, device: int = 0) -> Reader:
    return Reader(r=r, device=device)


def NewReaderBytes(b: bytes, device: int = 0) -> Reader:
    return Reader(b=b, device=device)


# ---------------------------------------------------------------- batches


class _Batch(C.Structure):
    _fields_ = [
        ("in_", C.c_void_p),
        ("in_off", C.c_void_p),
        ("out", C.c_void_p),
        ("out_off", C.c_void_p),
        ("out_size", C.c_void_p),
        ("status", C.c_void_p),
        ("count", C.c_uint64),
        ("max_len", C.c_uint64),
        ("in_bytes", C.c_uint64),   # decompress hints (ABI 2): the batch's input / output extents
        ("out_bytes", C.c_uint64),
    ]


def _stream_ptr(stream) -> int:
    import torch

    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


def _need_cuda(*ts) -> None:
    for t in ts:
        if not t.is_cuda:
            raise DeviceError(EDEVICE)


@dataclass
class CompressedBatch:
    slots: "object"       # uint8 CUDA tensor
    slot_off: "object"    # int64 CUDA tensor, count+1
    sizes: "object"       # int64 CUDA tensor, count
    status: "object"      # int32 CUDA tensor, count


def slot_offsets(in_off, extra: int = 0):
    """Slot offsets with capacity ez_compress_bound(n) per stream (device)."""
    import torch

    n = in_off[1:] - in_off[:-1]
    cap = n + (n >> 2) + 32 + extra
    cap = (cap + 15) & ~15
    return torch.cat([torch.zeros(1, dtype=torch.int64, device=in_off.device), torch.cumsum(cap, 0)])


def compress_batch(data, in_off, block: int = MiB, htable: int = 1024, max_len: int | None = None,
                   append_magic: bool = True, slot_off=None, out: CompressedBatch | None = None,
                   stream=None) -> CompressedBatch:
    """K1: compress independent streams data[in_off[s]:in_off[s+1]] (CUDA tensors)."""
    import torch

    _need_cuda(data, in_off)
    count = in_off.numel() - 1
    if out is None:
        if slot_off is None:
            slot_off = slot_offsets(in_off)
        total = int(slot_off[-1].item())
        out = CompressedBatch(
            torch.empty(total + 16, dtype=torch.uint8, device=data.device),
            slot_off,
            torch.empty(count, dtype=torch.int64, device=data.device),
            torch.empty(count, dtype=torch.int32, device=data.device),
        )
    if max_len is None:
        max_len = int((in_off[1:] - in_off[:-1]).max().item()) if count else 0
    b = _Batch(data.data_ptr(), in_off.data_ptr(), out.slots.data_ptr(), out.slot_off.data_ptr(),
               out.sizes.data_ptr(), out.status.data_ptr(), count, max_len)
    flags = 0 if append_magic else F_NO_MAGIC
    _check(_lib().ez_compress_batch(block, htable, flags, C.byref(b), _stream_ptr(stream)))
    return out


def _host_u8(b) -> "np.ndarray":
    import numpy as np

    if isinstance(b, np.ndarray):
        return np.ascontiguousarray(b, dtype=np.uint8).reshape(-1)
    return np.frombuffer(bytes(b), dtype=np.uint8)


def compress_batch_multi(data, in_off, block: int = MiB, htable: int = 1024, devices=None,
                         append_magic: bool = True):
    """Host-memory batch over several devices (ez_compress_batch_multi): stream s =
    data[in_off[s]:in_off[s+1]] (numpy uint8 / int64, or bytes) as one Write to a fresh
    NewWriter(block, htable), compressed in contiguous whole-stream shards, one per entry of
    `devices` (None: every visible device; repeats allowed).  Returns (packed bytes, packed
    offsets int64[count+1], statuses int32[count])."""
    import numpy as np

    d = _host_u8(data)
    off = np.ascontiguousarray(in_off, dtype=np.uint64)
    count = len(off) - 1
    n = off[1:].astype(np.int64) - off[:-1].astype(np.int64)
    cap = int(np.sum(n + (n >> 2) + 32)) + 16
    packed = np.empty(max(cap, 1), np.uint8)
    poff = np.zeros(count + 1, np.uint64)
    status = np.zeros(max(count, 1), np.int32)
    devs = None if devices is None else (C.c_int * len(devices))(*devices)
    L = _lib()
    L.ez_compress_batch_multi.argtypes = [C.c_int64, C.c_int64, C.c_int, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p,
                                          C.c_int, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p]
    _check(L.ez_compress_batch_multi(block, htable, 0 if append_magic else F_NO_MAGIC, d.ctypes.data, off.ctypes.data, count,
                                     devs, len(devices) if devices else 0, packed.ctypes.data, cap, poff.ctypes.data,
                                     status.ctypes.data))
    return packed[: int(poff[-1])], poff.astype(np.int64), status[:count]


def decompress_batch_multi(comp, comp_off, out_off, block_size_limit: int = 0, devices=None):
    """Host-memory decode over several devices (ez_decompress_batch_multi): stream s =
    comp[comp_off[s]:comp_off[s+1]] read to EOF into out[out_off[s]:out_off[s+1]].  Returns
    (out bytes, sizes int64[count], statuses int32[count])."""
    import numpy as np

    c = _host_u8(comp)
    coff = np.ascontiguousarray(comp_off, dtype=np.uint64)
    ooff = np.ascontiguousarray(out_off, dtype=np.uint64)
    count = len(coff) - 1
    out = np.zeros(max(int(ooff[-1]), 1), np.uint8)
    sizes = np.zeros(max(count, 1), np.uint64)
    status = np.zeros(max(count, 1), np.int32)
    devs = None if devices is None else (C.c_int * len(devices))(*devices)
    L = _lib()
    L.ez_decompress_batch_multi.argtypes = [C.c_int64, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_int, C.c_void_p,
                                            C.c_void_p, C.c_void_p, C.c_void_p]
    _check(L.ez_decompress_batch_multi(block_size_limit, c.ctypes.data, coff.ctypes.data, count, devs,
                                       len(devices) if devices else 0, out.ctypes.data, ooff.ctypes.data, sizes.ctypes.data,
                                       status.ctypes.data))
    return out[: int(ooff[-1])], sizes[:count].astype(np.int64), status[:count]


def compress_batch_writes(data, in_off, write_idx, write_end, block: int = MiB, htable: int = 1024,
                          append_magic: bool = True, stream=None) -> CompressedBatch:
    """K1 for multi-Write streams: stream s receives the Writes k = write_idx[s]
    .. write_idx[s+1]-1, Write k ending at data[write_end[k]] (CUDA int64 tensors).
    Its slot holds the bytes Go's sink receives over those Write calls."""
    import torch

    _need_cuda(data, in_off, write_idx, write_end)
    count = in_off.numel() - 1
    nw = write_idx[1:] - write_idx[:-1]
    n = in_off[1:] - in_off[:-1]
    cap = (n + (n >> 2) + 32 + 5 * nw + 15) & ~15  # ez_compress_bound + a trailing literal tag per Write
    slot_off = torch.cat([torch.zeros(1, dtype=torch.int64, device=data.device), torch.cumsum(cap, 0)])
    total = int(slot_off[-1].item())
    out = CompressedBatch(
        torch.empty(total + 16, dtype=torch.uint8, device=data.device),
        slot_off,
        torch.empty(count, dtype=torch.int64, device=data.device),
        torch.empty(count, dtype=torch.int32, device=data.device),
    )
    max_len = int((in_off[1:] - in_off[:-1]).max().item()) if count else 0
    max_writes = int(nw.max().item()) if count else 1
    b = _Batch(data.data_ptr(), in_off.data_ptr(), out.slots.data_ptr(), out.slot_off.data_ptr(),
               out.sizes.data_ptr(), out.status.data_ptr(), count, max_len)
    L = _lib()
    L.ez_compress_batch_writes.argtypes = [C.c_int64, C.c_int64, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64,
                                           C.c_void_p]
    flags = 0 if append_magic else F_NO_MAGIC
    _check(L.ez_compress_batch_writes(block, htable, flags, C.byref(b), write_idx.data_ptr(), write_end.data_ptr(),
                                      max(1, max_writes), _stream_ptr(stream)))
    return out


def pack(cb: CompressedBatch, packed=None, packed_off=None, workspace=None, stream=None):
    """K3: dense packing of the compressed slots -> (packed, packed_off)."""
    import torch

    count = cb.sizes.numel()
    dev = cb.slots.device
    if packed is None:
        packed = torch.empty(cb.slots.numel(), dtype=torch.uint8, device=dev)
    if packed_off is None:
        packed_off = torch.empty(count + 1, dtype=torch.int64, device=dev)
    if workspace is None:
        workspace = torch.empty(_lib().ez_pack_workspace(count), dtype=torch.uint8, device=dev)
    _check(_lib().ez_pack_batch(cb.slots.data_ptr(), cb.slot_off.data_ptr(), cb.sizes.data_ptr(), count,
                                packed.data_ptr(), packed_off.data_ptr(), workspace.data_ptr(), _stream_ptr(stream)))
    return packed, packed_off


def decompress_batch(comp, comp_off, out_off, block_size_limit: int = 0, out=None, sizes=None, status=None,
                     workspace=None, exact_only: bool = False, stream=None, max_len: int = 0,
                     in_bytes: int = 0, out_bytes: int = 0):
    """K2: decode complete streams comp[comp_off[s]:comp_off[s+1]] into
    out[out_off[s]:out_off[s+1]] -> (out, sizes, status).  exact_only skips
    the fast decoders (every stream on the exact decoder).  max_len (the largest
    slot), in_bytes = comp_off[-1] - comp_off[0] and out_bytes = out_off[-1] -
    out_off[0] are optional host hints: with them the call never waits for the
    stream to pick its decoder."""
    import torch

    _need_cuda(comp, comp_off, out_off)
    count = comp_off.numel() - 1
    dev = comp.device
    if out is None:
        out = torch.empty(int(out_off[-1].item()) + 16, dtype=torch.uint8, device=dev)
    if sizes is None:
        sizes = torch.empty(count, dtype=torch.int64, device=dev)
    if status is None:
        status = torch.empty(count, dtype=torch.int32, device=dev)
    if workspace is None and not exact_only:
        workspace = torch.empty(_lib().ez_decompress_workspace(count), dtype=torch.uint8, device=dev)
    b = _Batch(comp.data_ptr(), comp_off.data_ptr(), out.data_ptr(), out_off.data_ptr(), sizes.data_ptr(),
               status.data_ptr(), count, max_len, in_bytes, out_bytes)
    ws = None if exact_only else workspace.data_ptr()
    _check(_lib().ez_decompress_batch(block_size_limit, C.byref(b), ws, _stream_ptr(stream)))
    return out, sizes, status


# ---------------------------------------------------------------- Dumper (reader.go:43-54, 545-768)
from .dump import Dump, Dumper, NewDumper  # noqa: E402,F401
