"""Independent pure-Python restatement of tlog-dev/eazy writer.go / reader.go.

TEST INFRASTRUCTURE ONLY.  Used in this container to cross-check the C oracle
(oracle/eazy_oracle.c) and to generate the committed golden fixtures under
tests/golden/.  Written separately from the C restatement so that the two
agree only if both follow the Go code.  Small inputs only (pure-Python loops).

Every function cites the reference lines it restates
(/root/reference/writer.go, /root/reference/reader.go).
"""

from __future__ import annotations

import struct

LITERAL, COPY, META = 0x00, 0x80, 0x80
LEN1, LEN2, LEN4, LEN_ALT = 124, 125, 126, 127
OFF1, OFF2, OFF4, OFF_ALT = 252, 253, 254, 255
OFF_LONG = OFF_ALT
META_MAGIC, META_VER, META_RESET, META_BREAK = 0 << 3, 1 << 3, 2 << 3, 3 << 3
META_TAG_MASK, META_LEN_MASK, META_LEN_WIDE, META_LEN0 = 0xF8, 0x07, 6, 7
MIN_COPY_CHUNK = 6
MAGIC = b"\x80\x02eazy"
MiB = 1 << 20

# error names (numerically identical to include/eazy.h EZ_*)
OK, EOF, ESHORTBUF, EUNEXPECTEDEOF, EOVERFLOW, EBADMAGIC, ENOMAGIC = 0, 1, 2, 3, 4, 5, 6
EBLOCKLIMIT, EUNSUPMETA, EUNSUPVER, EBREAK, EMISSEDMETA, EINVAL, ESINK = 7, 8, 9, 10, 11, 12, 13


class Panic(Exception):
    """A Go panic in the reference."""


# ---------------------------------------------------------------- Encoder


def enc_tag(b: bytearray, tag: int, l: int) -> None:
    """Encoder.Tag writer.go:537-563."""
    if l < LEN1:
        b.append(tag | l)
        return
    l -= LEN1
    if l < 0x100:
        b += bytes([tag | LEN1, l])
        return
    l -= 0x100
    if l < 0x10000:
        b += bytes([tag | LEN2]) + struct.pack("<H", l)
        return
    l -= 0x10000
    if l < 0x100000000 - 8:
        b += bytes([tag | LEN4]) + struct.pack("<I", l)
        return
    raise Panic("too big length")


def enc_offset(b: bytearray, off: int, l: int) -> None:
    """Encoder.Offset writer.go:565-597."""
    if off >= l:
        off -= l
    else:
        b.append(OFF_LONG)
    if off < OFF1:
        b.append(off)
        return
    off -= OFF1
    if off < 0x100:
        b += bytes([OFF1, off])
        return
    off -= 0x100
    if off < 0x10000:
        b += bytes([OFF2]) + struct.pack("<H", off)
        return
    off -= 0x10000
    if off < 0x100000000 - 8:
        b += bytes([OFF4]) + struct.pack("<I", off)
        return
    raise Panic("too big offset")


def enc_meta(b: bytearray, meta: int, l: int) -> None:
    """Encoder.Meta writer.go:599-621."""
    if meta & ~META_TAG_MASK:
        raise Panic(meta)
    if l == 0:
        b += bytes([META, meta | META_LEN0])
        return
    if l < META_LEN_WIDE and l & (l - 1) == 0:
        b += bytes([META, meta | (l.bit_length() - 1)])
        return
    if l < OFF1:
        b += bytes([META, meta | META_LEN_WIDE, l])
        return
    b += bytes([META, meta | META_LEN_WIDE])
    enc_offset(b, l, 0)


# ---------------------------------------------------------------- Decoder


def dec_tag(b: bytes, st: int):
    """Decoder.Tag reader.go:346-392 -> (tag, l, i, err)."""
    if st >= len(b):
        return 0, 0, st, ESHORTBUF
    i = st
    tag = b[i] & 0x80
    l = b[i] & 0x7F
    i += 1
    if l == LEN1:
        if i + 1 > len(b):
            return tag, l, st, ESHORTBUF
        l = LEN1 + b[i]
        i += 1
    elif l == LEN2:
        if i + 2 > len(b):
            return tag, l, st, ESHORTBUF
        l = LEN1 + 0x100 + (b[i] | b[i + 1] << 8)
        i += 2
    elif l == LEN4:
        if i + 4 > len(b):
            return tag, l, st, ESHORTBUF
        l = LEN1 + 0x100 + 0x10000 + struct.unpack_from("<I", b, i)[0]
        i += 4
    elif l == LEN_ALT:
        return tag, l, st, EOVERFLOW
    return tag, l, i, OK


def _basic_offset(b: bytes, st: int):
    """Decoder.basicOffset reader.go:422-472 -> (off, i, err)."""
    i = st
    if i == len(b):
        return 0, st, ESHORTBUF
    off = b[i]
    i += 1
    if off == OFF1:
        if i + 1 > len(b):
            return off, st, ESHORTBUF
        off = OFF1 + b[i]
        i += 1
    elif off == OFF2:
        if i + 2 > len(b):
            return off, st, ESHORTBUF
        off = OFF1 + 0x100 + (b[i] | b[i + 1] << 8)
        i += 2
    elif off == OFF4:
        if i + 4 > len(b):
            return off, st, ESHORTBUF
        off = OFF1 + 0x100 + 0x10000 + struct.unpack_from("<I", b, i)[0]
        i += 4
    elif off == OFF_ALT:
        return off, st, EOVERFLOW
    return off, i, OK


def dec_offset(b: bytes, st: int, l: int):
    """Decoder.Offset reader.go:394-420 -> (off, i, err)."""
    i = st
    if i == len(b):
        return 0, st, ESHORTBUF
    long_ = b[i] == OFF_LONG
    if long_:
        i += 1
    off, i, err = _basic_offset(b, i)
    if err:
        return off, st, err
    if not long_:
        off += l
    return off, i, OK


def dec_meta(b: bytes, st: int):
    """Decoder.Meta reader.go:474-514 -> (meta, l, i, err)."""
    i = st
    if i == len(b):
        return 0, 0, st, ESHORTBUF
    m = b[i]
    i += 1
    meta, l = m & META_TAG_MASK, m & META_LEN_MASK
    if l == META_LEN0:
        return meta, 0, i, OK
    if l < META_LEN_WIDE:
        return meta, 1 << l, i, OK
    if i == len(b):
        return meta, 0, st, ESHORTBUF
    l = b[i]
    i += 1
    if l < OFF1:
        return meta, l, i, OK
    l, j, err = _basic_offset(b, i - 1)
    if err:
        return meta, l, st, err
    return meta, l, j, OK


# ---------------------------------------------------------------- Writer


class Writer:
    """Writer writer.go:17-535 over an in-memory sink (eazy_test.go Buf)."""

    def __init__(self, block: int, htable: int):  # NewWriter writer.go:133-145
        self.append_magic = True
        self.flush_threshold = 0
        self.ver = 0
        self.b = bytearray()
        self.written = 0
        self._sink = bytearray()
        self.sink_writes = []
        self.fail_accept = None
        self.block = bytearray()
        self.ht = []
        self._init(block, htable)
        self.pos = 0

    def _init(self, bs: int, hs: int) -> None:  # writer.go:161-185
        if (bs - 1) & bs or bs < 32 or bs > 1 << 31:
            raise Panic("block size")
        if (hs - 1) & hs or hs < 4:
            raise Panic("hash table size")
        self.bs, self.mask = bs, bs - 1
        self.block = bytearray(bs)
        self.hsh = 32 - (hs - 1).bit_length()
        self.ht = [0] * hs

    def _reset(self) -> None:  # writer.go:187-200
        self.b = bytearray()
        self.pos = 0
        self.written = 0
        self.block = bytearray(self.bs)
        self.ht = [0] * len(self.ht)

    def reset(self) -> None:  # Reset writer.go:149-152
        self._reset()

    def reset_size(self, block: int, htable: int) -> None:  # writer.go:155-159
        self._init(block, htable)
        self._reset()

    def _isreset(self) -> bool:  # writer.go:403-405
        return self.written + len(self.b) == 0

    def _hash(self, p: bytes, i: int) -> int:  # writer.go:491-493
        return ((struct.unpack_from("<I", p, i)[0] * 0x1E35A7BD) & 0xFFFFFFFF) >> self.hsh

    def _header(self) -> None:  # writer.go:495-517
        if self.append_magic:
            self.b += MAGIC
        if self.ver != 0:
            self.b += bytes([META, META_VER, self.ver & 0xFF])
        self.b += bytes([META, META_RESET, (self.bs & -self.bs).bit_length() - 1])

    def _literal(self, d: bytes, st: int, end: int) -> None:  # writer.go:519-522
        enc_tag(self.b, LITERAL, end - st)
        self.b += d[st:end]

    def _copy(self, st: int, end: int) -> None:  # writer.go:524-527
        enc_tag(self.b, COPY, end - st)
        enc_offset(self.b, self.pos - st, end - st)

    def _copy_data(self, d: bytes, st: int, end: int) -> None:  # writer.go:529-535
        for k in range(st, end):
            self.block[self.pos & self.mask] = d[k]
            self.pos += 1

    def _write_zeros(self, p: bytes, done: int, i: int):  # writer.go:407-439
        iend = i
        while iend < len(p) and p[iend] == 0:
            iend += 1
        while i > done and p[i - 1] == 0:
            i -= 1
        if iend - i < MIN_COPY_CHUNK:
            return done, i + 1
        if done != i:
            self._literal(p, done, i)
            self._copy_data(p, done, i)
        enc_tag(self.b, COPY, iend - i)
        self.b += bytes([OFF_LONG, 0])
        self._copy_data(p, i, iend)
        return iend, iend

    def _write_runlen(self, p: bytes, done: int, st: int, i: int):  # writer.go:441-489
        if st + 8 < len(p) and p[st : st + 8] == bytes(8):
            return self._write_zeros(p, done, st)
        jf = 0
        while i + jf < len(p) and p[st + jf] == p[i + jf]:
            jf += 1
        jb = -1
        while st + jb >= 0 and i + jb >= done and p[st + jb] == p[i + jb]:
            jb -= 1
        jb += 1
        if jf - jb < MIN_COPY_CHUNK:
            return done, i + 1
        if i - st >= self.bs - 8:
            iend = done + i - st
            self._literal(p, done, iend)
            self._copy_data(p, done, iend)
            return iend, iend
        ist, iend = i + jb, i + jf
        self._literal(p, done, ist)
        self._copy_data(p, done, ist)
        enc_tag(self.b, COPY, iend - ist)
        enc_offset(self.b, i - st, iend - ist)
        self._copy_data(p, ist, iend)
        return iend, iend

    def write(self, p: bytes):  # Write writer.go:206-337 -> (n, err)
        p = bytes(p)
        if self._isreset():
            self._header()
        start = self.pos
        done = 0
        i = 0
        n = len(p)
        blk = self.block
        while i + 4 <= n:
            h = self._hash(p, i)
            pos = self.ht[h]
            self.ht[h] = (start + i) & 0xFFFFFFFF
            off = pos - self.pos
            if -off > self.bs:
                i += 1
                continue
            if off >= 0 and i > done + off:
                done, i = self._write_runlen(p, done, done + off, i)
                continue
            ist, st = i - 1, pos - 1
            while ist >= done and p[ist] == blk[st & self.mask]:
                ist -= 1
                st -= 1
            ist += 1
            st += 1
            iend, end = i, pos
            while iend < n and p[iend] == blk[end & self.mask]:
                iend += 1
                end += 1
            blit = self.pos - self.bs
            bend = blit + (iend - done)
            diff = bend - st
            if diff > 0:
                end -= diff
                iend -= diff
            diff = (end - self.bs) - blit
            if diff > 0:
                end -= diff
                iend -= diff
            if end - st < MIN_COPY_CHUNK:
                i += 1
                continue
            if done < ist:
                self._literal(p, done, ist)
                self._copy_data(p, done, ist)
            if self.pos - st > self.bs:
                raise Panic("too big offset")
            self._copy(st, end)
            self._copy_data(p, ist, iend)
            if i + 1 + 4 <= n:
                self.ht[self._hash(p, i + 1)] = (start + i + 1) & 0xFFFFFFFF
            i = iend
            done = iend
        if done < n:
            self._literal(p, done, n)
            self._copy_data(p, done, n)
            done = n
        err = self._write_out()
        if err:
            return 0, err
        return done, OK

    def write_header(self):  # writer.go:342-350
        if not self._isreset():
            return OK
        self._header()
        return self._write_out()

    def write_break(self):  # writer.go:358-366
        if self._isreset():
            self._header()
        self.b += bytes([META, META_BREAK | META_LEN0])
        return self._write_out()

    def flush(self):  # writer.go:371-377
        if not self.b:
            return OK
        return self._flush()

    def _write_out(self):  # writer.go:379-385
        if self.flush_threshold < 0 or len(self.b) < self.flush_threshold:
            return OK
        return self._flush()

    @property
    def sink(self) -> bytes:
        return bytes(self._sink)

    def sink_fault(self, accept: int) -> None:
        """The next sink Write takes `accept` bytes and fails."""
        self.fail_accept = accept

    def _flush(self):  # writer.go:387-401
        if self.fail_accept is not None:
            n = min(len(self.b), self.fail_accept)
            self.fail_accept = None
            self._sink += self.b[:n]
            self.written += n
            self._reset()
            return ESINK
        self._sink += self.b
        self.sink_writes.append(bytes(self.b))
        self.written += len(self.b)
        self.b = bytearray()
        return OK


def compress(block: int, htable: int, writes, append_magic=True, ver=0) -> bytes:
    w = Writer(block, htable)
    w.append_magic = append_magic
    w.ver = ver
    for p in writes:
        n, err = w.write(p)
        assert err == OK and n == len(p)
    return w.sink


# ---------------------------------------------------------------- Reader


class Reader:
    """Reader reader.go:17-543.  src is None (NewReaderBytes) or a list of
    chunks served by an io.Reader that returns io.EOF with its last bytes
    (eazy_test.go BufReader)."""

    def __init__(self, b: bytes = b"", src=None, block_size_limit=None, buffer_size=None):
        self.ver = 0
        self.block = bytearray()
        self.mask = 0
        self.pos = 0
        self.state = 0
        self.off = 0
        self.len = 0
        self.b = bytearray(b)
        self.i = 0
        self.boff = 0
        self.src = None if src is None else bytearray(src)
        if src is None:  # NewReaderBytes reader.go:89-93
            self.block_size_limit = 0 if block_size_limit is None else block_size_limit
            self.buffer_size = 0 if buffer_size is None else buffer_size
        else:  # NewReader reader.go:79-85
            self.block_size_limit = 16 * MiB if block_size_limit is None else block_size_limit
            self.buffer_size = 64 * 1024 if buffer_size is None else buffer_size
        self.require_magic = False
        self.skip_unsupported_meta = False

    def set(self, block_size_limit, buffer_size, require_magic=False, skip_unsupported_meta=False):
        self.block_size_limit = block_size_limit
        self.buffer_size = buffer_size
        self.require_magic = require_magic
        self.skip_unsupported_meta = skip_unsupported_meta

    def append(self, b: bytes) -> None:
        """More data arrives at the underlying io.Reader."""
        self.src += b

    def reset_bytes(self, b: bytes) -> None:  # ResetBytes reader.go:102-113
        self.src = None
        self.b = bytearray(b)
        self.block = bytearray()
        self.pos = 0
        self.i = 0
        self.boff = 0
        self.state = 0

    def reset(self, src: bytes = b"") -> None:  # Reset reader.go:96-99
        self.reset_bytes(b"")
        self.src = bytearray(src)

    def read(self, plen: int):  # Read reader.go:116-141 -> (bytes, err)
        p = bytearray(plen)
        n = 0
        err = OK
        while n < plen and err == OK:
            m, i, err = self._read(p, n, self.i)
            n += m
            self.i = i
            if n == plen:
                break
            if err != ESHORTBUF:
                continue
            err = self._more()
            if err == EOF and (self.state != 0 or self.i < len(self.b)):
                err = EUNEXPECTEDEOF
        return bytes(p[:n]), err

    def _read(self, p: bytearray, at: int, st: int):  # reader.go:143-216
        i = st
        while self.state == 0:
            i, err = self._read_tag(i)
            if err:
                return 0, i, err
        if len(self.block) == 0:
            return 0, st, EMISSEDMETA
        if self.state == ord("l") and i == len(self.b):
            return 0, i, ESHORTBUF
        plen = len(p) - at
        end = min(self.len, plen)
        if self.state == ord("l"):
            end = min(end, len(self.b) - i)
            p[at : at + end] = self.b[i : i + end]
            i += end
        elif self.off + self.len <= self.pos:
            s = self.off & self.mask
            end = min(end, len(self.block) - s)
            p[at : at + end] = self.block[s : s + end]
            self.off += end
        elif self.off == self.pos:
            p[at : at + end] = bytes(end)
        else:
            run = min(self.pos - self.off, plen)
            for j in range(run):
                p[at + j] = self.block[(self.off + j) & self.mask]
            j = run
            while j < end:
                k = min(j, end - j)
                p[at + j : at + j + k] = p[at : at + k]
                j += k
            self.off += end
        self.len -= end
        for k in range(end):
            self.block[self.pos & self.mask] = p[at + k]
            self.pos += 1
        if self.len == 0:
            self.state = 0
        return end, i, OK

    def _read_tag(self, st: int):  # reader.go:218-270
        i = st
        b = self.b
        while i < len(b) and b[i] == 0:
            i += 1
        st = i
        tag, l, i, err = dec_tag(b, st)
        if err:
            return st, err
        if self.boff == 0 and st == 0 and b[st] != META and self.require_magic:
            return st, ENOMAGIC
        if tag == META and l == 0:
            return self._continue_meta(i)
        if self.block_size_limit != 0 and l > self.block_size_limit:
            return st, EBLOCKLIMIT
        if tag == LITERAL:
            self.state = ord("l")
            self.off = 0
        else:
            off, i, err = dec_offset(b, i, l)
            if err:
                return st, err
            if off > len(self.block):
                return st, EOVERFLOW
            self.off = self.pos - off
            self.state = ord("c")
        self.len = l
        return i, OK

    def _continue_meta(self, st: int):  # reader.go:272-325
        i = st
        st -= 1
        b = self.b
        meta, l, i, err = dec_meta(b, i)
        if err:
            return i, err
        if self.boff == 0 and st == 0 and meta != META_MAGIC and self.require_magic:
            return st, ENOMAGIC
        if i + l > len(b):
            return st, ESHORTBUF
        tag_len = [4, 1, 1, 0]
        j = meta >> 3
        if j < len(tag_len) and l != tag_len[j]:
            return st, EUNSUPMETA
        if meta == META_MAGIC:
            if bytes(b[i : i + l]) != b"eazy":
                return st, EBADMAGIC
        elif meta == META_VER:
            self.ver = b[i]
            if self.ver > 0:
                return st, EUNSUPVER
        elif meta == META_RESET:
            bs = b[i]
            if bs > 32 or l != 1 or (self.block_size_limit != 0 and 1 << bs > self.block_size_limit):
                return st, EOVERFLOW
            self._reset(bs)
        elif meta == META_BREAK:
            return i + l, EBREAK
        else:
            if not self.skip_unsupported_meta:
                return st, EUNSUPMETA
        return i + l, OK

    def _reset(self, bs: int) -> None:  # reader.go:327-344
        self.block = bytearray(1 << bs)
        self.pos = 0
        self.mask = (1 << bs) - 1
        self.state = 0

    def _more(self):  # reader.go:516-543 (source returns EOF with its last bytes)
        if self.src is None:
            return EOF
        self.b = self.b[self.i :]
        self.boff += self.i
        self.i = 0
        room = self.buffer_size if len(self.b) == 0 else 1024
        chunk = self.src[:room]
        del self.src[:room]
        self.b += chunk
        err = EOF if not self.src else OK
        if len(chunk) != 0 and err == EOF:
            err = OK
        return err


def decompress(b: bytes, buf: int = 1 << 16):
    """NewReaderBytes(b) read until EOF (ErrBreak skipped) -> (bytes, err, breaks)."""
    r = Reader(b)
    out = bytearray()
    breaks = 0
    while True:
        got, err = r.read(buf)
        out += got
        if err == EBREAK:
            breaks += 1
            continue
        if err == EOF:
            return bytes(out), OK, breaks
        if err:
            return bytes(out), err, breaks
