"""Dumper: the debug printer of a compressed stream (reader.go:43-54, 545-768).

Host side, like the reference's: it walks the tokens with ``Decoder`` (the
C-ABI token decoders of libeazy_amd.so, reader.go:346-514) and prints one line
per padding run, meta, literal and copy, in the reference's text format (Go
``fmt`` verbs restated below: ``%x`` widths, ``%q`` quoting, ``% x`` hex).

Parity: the token walk and the error values follow reader.go:602-710 and are
checked on the reference's KAT streams and fuzz corpora; the reference's own
tests only log dump text, so the text itself is pinned by nothing but this
restatement of the format (parity unpinned for the text).
"""

from __future__ import annotations

import unicodedata

from . import EOF, ESHORTBUF, EUNEXPECTEDEOF, OK, Copy, Decoder, Literal, Meta, MetaVer, OffLong, _strerror


def _rune(b: bytes, i: int):
    """utf8.DecodeRune: (rune, width); (0xFFFD, 1) for an invalid encoding."""
    c = b[i]
    if c < 0x80:
        return c, 1
    n = 2 if 0xC2 <= c <= 0xDF else 3 if 0xE0 <= c <= 0xEF else 4 if 0xF0 <= c <= 0xF4 else 0
    if n and i + n <= len(b):
        try:
            return ord(b[i : i + n].decode("utf-8")), n
        except UnicodeDecodeError:
            pass
    return 0xFFFD, 1


def _is_print(r: int) -> bool:
    """strconv.IsPrint: letters, marks, numbers, punctuation, symbols and U+0020."""
    return r == 0x20 or unicodedata.category(chr(r))[0] in "LMNPS"


def go_quote(b: bytes) -> str:
    """fmt's %q of a []byte (strconv.Quote of string(b))."""
    out = ['"']
    i = 0
    while i < len(b):
        r, w = _rune(b, i)
        if w == 1 and r == 0xFFFD:
            out.append("\\x%02x" % b[i])
            i += 1
            continue
        i += w
        if r in (0x22, 0x5C):
            out.append("\\" + chr(r))
        elif _is_print(r):
            out.append(chr(r))
        elif r in _ESC:
            out.append(_ESC[r])
        elif r < 0x20 or r == 0x7F:
            out.append("\\x%02x" % r)
        elif r < 0x10000:
            out.append("\\u%04x" % r)
        else:
            out.append("\\U%08x" % r)
    out.append('"')
    return "".join(out)


_ESC = {0x07: "\\a", 0x08: "\\b", 0x0C: "\\f", 0x0A: "\\n", 0x0D: "\\r", 0x09: "\\t", 0x0B: "\\v"}


class Dumper:
    """eazy.Dumper: ``Writer`` (an object with ``write(bytes)``, or None),
    ``Debug(ioff, iend, ooff, tag, l, off)`` (tag: ord of 'p', 'm', 'l', 'c', 'e'),
    ``GlobalOffset`` (< 0: no global offset column)."""

    def __init__(self, w=None):
        self.Writer = w
        self.Debug = None
        self.GlobalOffset = 0
        self._d = Decoder()
        self.pos = 0  # output position (r.pos)
        self.boff = 0  # input bytes consumed by earlier Writes (r.boff)
        self.b = bytearray()

    def _dbg(self, st, i, tag, l, off):
        if self.Debug is not None:
            self.Debug(self.boff + st, self.boff + i, self.pos, ord(tag), l, off)

    def Write(self, p: bytes):  # reader.go:602-710
        """Prints the whole tokens of p; returns (bytes consumed, error code)."""
        p = bytes(p)
        self.b = bytearray()
        i, err = 0, OK
        try:
            while i < len(p):
                if self.GlobalOffset >= 0:
                    self.b += b"%6x  " % (self.GlobalOffset + i)
                self.b += b"%4x  %6x  " % (i, self.pos)
                st = i
                while i < len(p) and p[i] == 0:
                    i += 1
                if i != st:
                    self.b += b"pad  %4x\n" % (i - st)
                    self._dbg(st, i, "p", i - st, 0)
                    continue
                tag, l, i2, e = self._d.tag(p, i)
                if e != OK:
                    i, err = st, e
                    return i, err
                i = i2
                if tag == Meta and l == 0:
                    meta, l, i, e = self._d.meta(p, i)
                    if e != OK:
                        err = e
                        return i, err
                    if i + l > len(p):
                        err = ESHORTBUF
                        return i, err
                    if meta == MetaVer and l == 1:
                        self._d.Ver = p[i]
                    arg = p[i : i + l]
                    self.b += ("meta %2x %x  %-8s  %s\n" % (meta >> 3, l, go_quote(arg), " ".join("%02x" % c for c in arg))).encode()
                    self._dbg(st, i, "m", l, meta)
                    i += l
                elif tag == Literal:
                    if i + l > len(p):
                        err = ESHORTBUF
                        return i, err
                    self.b += ("lit  %4x        %s\n" % (l, go_quote(p[i : i + l]))).encode()
                    self._dbg(st, i, "l", l, 0)
                    i += l
                    self.pos += l
                elif tag == Copy:
                    long = "  (long)" if i < len(p) and p[i] == OffLong else ""
                    off, i2, e = self._d.offset(p, i, l)
                    if e != OK:
                        i, err = st, e
                        return i, err
                    i = i2
                    self.b += ("copy %4x  off %4x%s\n" % (l, off, long)).encode()
                    self._dbg(st, i, "c", l, off)
                    self.pos += l
            return i, err
        finally:  # the deferred accounting and sink write (reader.go:605-620)
            self.boff += i
            if self.GlobalOffset >= 0:
                self.GlobalOffset += i
            if self.Writer is not None:
                self.Writer.write(bytes(self.b))

    def ReadFrom(self, r):  # reader.go:563-600
        """Dumps everything r yields (``read_go(k) -> (bytes, err)`` with Go io.Reader
        semantics, or ``read(k)`` returning b"" at the end); returns (bytes read, err)."""
        buf = bytearray(0x10000)
        keep, tot, err = 0, 0, OK
        while True:
            room = len(buf) - keep
            if hasattr(r, "read_go"):
                data, err = r.read_go(room)
            else:
                data = r.read(room)
                err = OK if data else EOF
            n = len(data)
            if n == 0:
                break
            tot += n
            buf[keep : keep + n] = data
            n += keep
            m, err = self.Write(bytes(buf[:n]))
            rest = bytes(buf[m:n])
            buf[: len(rest)] = rest
            keep = len(rest)
            if err not in (OK, ESHORTBUF):
                break
        if err == EOF:
            err = OK
        if keep != 0 and err == OK:
            err = EUNEXPECTEDEOF
        return tot, err

    def Close(self):  # reader.go:712-732
        if self.GlobalOffset >= 0:
            self.b += b"%6x  " % self.GlobalOffset
        self.b += b"%4x  " % 0
        self.b += b"%6x  " % self.pos
        if self.Debug is not None:
            self.Debug(self.boff, self.boff, self.pos, ord("e"), 0, 0)
        return OK


def NewDumper(w=None) -> Dumper:  # reader.go:557-561
    return Dumper(w)


def Dump(p: bytes) -> str:  # reader.go:545-555
    """The debug print of a compressed buffer, with the error that stopped it."""
    d = Dumper()
    _, err = d.Write(p)
    d.Close()
    if err != OK:
        d.b += b"\nerror: " + _strerror(err).encode()
    return d.b.decode()
