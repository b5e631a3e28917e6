"""One interface over the three implementations the tests compare:
the C oracle (oracle/), the Python restatement (tests/pyoracle.py) and the
shipped GPU path (eazy_amd, libeazy_amd.so).

Writer: write(p) -> (n, err); write_header/write_break/flush() -> err;
reset(); reset_size(b, h); setters append_magic / ver / flush_threshold;
sink -> bytes written to the underlying io.Writer so far.
Reader: read(n) -> (bytes, err); set(limit, bufsize, require_magic, skip);
reset_bytes(b); reset(src); append(b) (more data at the io.Reader).
"""

from __future__ import annotations

import oracle as _orc
import pyoracle as _py


class COracle:
    name = "c-oracle"
    Panic = _orc.Panic

    @staticmethod
    def W(block, htable):
        return _orc.Writer(block, htable)

    @staticmethod
    def Rb(b):
        return _orc.Reader(b=b)

    @staticmethod
    def Rs(src, eof_with_data=True):
        return _orc.Reader(src=src, eof_with_data=eof_with_data)


class PyOracle:
    name = "py-oracle"
    Panic = _py.Panic

    @staticmethod
    def W(block, htable):
        return _py.Writer(block, htable)

    @staticmethod
    def Rb(b):
        return _py.Reader(b)

    @staticmethod
    def Rs(src, eof_with_data=True):
        return _py.Reader(src=src)


class _Buf:
    """eazy_test.go Buf: append-only io.Writer (optionally failing once)."""

    def __init__(self):
        self.data = bytearray()
        self.fail_accept = None

    def write(self, b):
        if self.fail_accept is not None:
            n = min(len(b), self.fail_accept)
            self.data += b[:n]
            self.fail_accept = None
            e = IOError("sink failed")
            e.n = n
            raise e
        self.data += b
        return len(b)


class _Src:
    """In-memory io.Reader with Go semantics (BufReader: EOF with the last bytes)."""

    def __init__(self, data, eof_with_data=True):
        self.data = bytearray(data)
        self.eof_with_data = eof_with_data

    def read_go(self, k):
        import eazy_amd as ez

        chunk = bytes(self.data[:k])
        del self.data[:k]
        if self.eof_with_data:
            return chunk, ez.EOF if not self.data else ez.OK
        return chunk, ez.EOF if (not chunk and k > 0) else ez.OK


class _GpuWriter:
    def __init__(self, block, htable):
        import eazy_amd as ez

        self._ez = ez
        self.buf = _Buf()
        self.w = ez.Writer(self.buf, block, htable)

    def _err(self, fn, *a):
        ez = self._ez
        try:
            r = fn(*a)
            return r, ez.OK
        except ez.Panic:
            raise
        except ez.EazyError as e:
            return 0, e.code
        except OSError:
            return 0, ez.ESINK

    def write(self, p):
        return self._err(self.w.Write, p)

    def write_header(self):
        return self._err(self.w.WriteHeader)[1]

    def write_break(self):
        return self._err(self.w.WriteBreak)[1]

    def flush(self):
        return self._err(self.w.Flush)[1]

    def reset(self):
        self.w.Reset(self.buf)

    def reset_size(self, block, htable):
        self.w.ResetSize(self.buf, block, htable)

    def sink_fault(self, accept):
        self.buf.fail_accept = accept

    def sink_clear(self):
        self.buf.data = bytearray()

    @property
    def sink(self):
        return bytes(self.buf.data)

    append_magic = property(None, lambda s, v: setattr(s.w, "AppendMagic", v))
    ver = property(None, lambda s, v: setattr(s.w, "Ver", v))
    flush_threshold = property(None, lambda s, v: setattr(s.w, "FlushThreshold", v))


class _GpuReader:
    def __init__(self, b=None, src=None, eof_with_data=True):
        import eazy_amd as ez

        if src is None:
            self.src = None
            self.r = ez.Reader(b=b or b"")
        else:
            self.src = _Src(src, eof_with_data)
            self.r = ez.Reader(r=self.src)

    def read(self, n):
        return self.r.Read(n)

    def set(self, block_size_limit, buffer_size, require_magic=False, skip_unsupported_meta=False):
        self.r.BlockSizeLimit = block_size_limit
        self.r.BufferSize = buffer_size
        self.r.RequireMagic = require_magic
        self.r.SkipUnsupportedMeta = skip_unsupported_meta

    def append(self, b):
        self.src.data += b

    def reset_bytes(self, b):
        self.r.ResetBytes(b)

    def reset(self, src=b""):
        self.src = _Src(src)
        self.r.Reset(self.src)


class Gpu:
    name = "gpu"

    @staticmethod
    def W(block, htable):
        return _GpuWriter(block, htable)

    @staticmethod
    def Rb(b):
        return _GpuReader(b=b)

    @staticmethod
    def Rs(src, eof_with_data=True):
        return _GpuReader(src=src, eof_with_data=eof_with_data)

    @property
    def Panic(self):
        import eazy_amd as ez

        return ez.Panic
