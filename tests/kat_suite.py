"""The reference's own tests (eazy_test.go), restated over tests/impls.py.

Each function takes an implementation I (C oracle, Python oracle or GPU) and
asserts what the Go test asserts; exact-byte expectations are the Go tests'
known answers.  Go's math/rand seed-0 inputs cannot be reproduced without Go,
so the seeded round-trip tests use inputs of the same shape (numpy PCG64,
fixed seeds) — they are round-trip checks in the reference too.
"""

from __future__ import annotations

import numpy as np

MiB = 1 << 20
OK, EOF, ESHORTBUF, EUNEXPECTEDEOF, EOVERFLOW, EBADMAGIC, ENOMAGIC = 0, 1, 2, 3, 4, 5, 6
EBLOCKLIMIT, EUNSUPMETA, EUNSUPVER, EBREAK, EMISSEDMETA = 7, 8, 9, 10, 11
MAGIC = b"\x80\x02eazy"
Literal, Copy, Meta, OffLong, Len1, Len2 = 0x00, 0x80, 0x80, 0xFF, 124, 125
MetaMagic, MetaVer, MetaReset, MetaBreak, MetaLen0, MetaTagMask = 0x00, 0x08, 0x10, 0x18, 7, 0xF8


def _w(I, block, htable, magic=True, ver=0):
    w = I.W(block, htable)
    if not magic:
        w.append_magic = False
    if ver:
        w.ver = ver
    return w


def _wr(w, p):
    n, err = w.write(p)
    assert err == OK
    assert n == len(p)


def t_magic(I):  # TestMagic eazy_test.go:39-64
    w = I.W(MiB, 512)
    assert w.write_header() == OK
    buf = w.sink
    assert buf[: len(MAGIC)] == MAGIC
    assert buf == bytes.fromhex("800265617a79801014")
    assert w.write_header() == OK
    assert w.sink == buf
    _wr(w, b"\x00")
    assert w.sink == buf + b"\x01\x00"


def t_literal(I):  # TestLiteral eazy_test.go:66-104
    w = _w(I, 32, 16, magic=False)
    _wr(w, b"very_first_message")
    r = I.Rb(w.sink)
    assert r.read(10) == (b"very_first", OK)
    assert r.read(10) == (b"_message", EOF)


def t_copy(I):  # TestCopy eazy_test.go:106-183
    w = _w(I, 32, 16, magic=False)
    _wr(w, b"prefix_1234_suffix")
    st = len(w.sink)
    _wr(w, b"prefix_567_suffix")
    buf = w.sink
    # expected second Write: Copy|7,0x12-7; Literal|3 "567"; Copy|7,0x11-7 (:176-178)
    assert buf[st:] == bytes([Copy | 7, 0x12 - 7, Literal | 3]) + b"567" + bytes([Copy | 7, 0x11 - 7])
    assert buf == bytes([Meta, MetaReset, 5, 0x12]) + b"prefix_1234_suffix" + buf[st:]
    r = I.Rb(buf)
    assert r.read(10) == (b"prefix_123", OK)
    assert r.read(10) == (b"4_suffixpr", OK)
    assert r.read(30) == (b"efix_567_suffix", EOF)


def t_bug1(I):  # TestBug1 eazy_test.go:185-207 (bytes.Buffer source)
    r = I.Rs(bytes([Meta, MetaReset, 14]) + bytes([Literal | 3, 0x94, 0xA8, 0xFB, Copy | 9]), eof_with_data=False)
    got, err = r.read(1000)
    assert err == EUNEXPECTEDEOF
    assert got == bytes([0x94, 0xA8, 0xFB])
    r.append(bytes([0xFD, 0x03, 0x65]))  # offset
    got, err = r.read(1000)
    assert err == EOVERFLOW
    assert got == b""


def t_padding(I):  # TestPadding eazy_test.go:209-268
    B = 32
    w = I.W(B, B >> 1)
    _wr(w, b"prefix_1234_suffix")
    pad = bytes(B - len(w.sink) % B)
    head = w.sink
    _wr(w, b"prefix_567_suffix")
    buf = head + pad + w.sink[len(head) :]
    r = I.Rb(buf)
    assert r.read(10) == (b"prefix_123", OK)
    assert r.read(10) == (b"4_suffixpr", OK)
    assert r.read(30) == (b"efix_567_suffix", EOF)


def t_zero_region(I):  # TestZeroRegion eazy_test.go:270-280
    r = I.Rb(bytes([Meta, MetaReset, 2, Meta, MetaVer, 0, Copy | 10, OffLong, 0]))
    got, err = r.read(16)
    assert err == EOF
    assert got == bytes(10)


def t_reset(I):  # TestReset eazy_test.go:282-340 (one sink, split per Reset)
    w = I.W(1024, 32)
    parts = []
    cuts = [0]
    _wr(w, b"some_message")
    cuts.append(len(w.sink))
    w.reset()
    _wr(w, b"another_message")
    cuts.append(len(w.sink))
    w.reset_size(2048, 64)
    _wr(w, b"third_message")
    cuts.append(len(w.sink))
    w.reset_size(512, 16)
    _wr(w, b"fourth_message")
    cuts.append(len(w.sink))
    w.reset_size(1024, 32)
    _wr(w, b"fifth_message")
    cuts.append(len(w.sink))
    sink = w.sink
    parts = [sink[cuts[k] : cuts[k + 1]] for k in range(5)]
    msgs = [b"some_message", b"another_message", b"third_message", b"fourth_message", b"fifth_message"]
    r = I.Rs(parts[0])
    assert r.read(0x20) == (msgs[0], EOF)
    r.reset(parts[1])
    assert r.read(0x20) == (msgs[1], EOF)
    r.reset_bytes(parts[2])
    assert r.read(0x20) == (msgs[2], EOF)
    r.reset_bytes(parts[3])
    assert r.read(0x20) == (msgs[3], EOF)
    r.reset(parts[4])
    assert r.read(0x20) == (msgs[4], EOF)


def t_break(I):  # TestBreak eazy_test.go:342-415
    w = _w(I, 32, 16, magic=False)
    _wr(w, b"message1")
    assert w.write_break() == OK
    _wr(w, b"qwessage2")
    r = I.Rb(w.sink)
    assert r.read(20) == (b"message1", EBREAK)
    assert r.read(20) == (b"qwessage2", EOF)
    # a Break on a fresh stream
    w.reset()
    st = len(w.sink)
    assert w.write_break() == OK
    r.reset_bytes(w.sink[st:])
    assert r.read(20) == (b"", EBREAK)
    assert r.read(20) == (b"", EOF)
    # data, Break, end
    w.reset()
    st = len(w.sink)
    _wr(w, b"123")
    assert w.write_break() == OK
    r.reset_bytes(w.sink[st:])
    assert r.read(3) == (b"123", OK)
    assert r.read(20) == (b"", EBREAK)
    assert r.read(20) == (b"", EOF)


def t_require_magic(I):  # TestReaderRequireMagic eazy_test.go:417-431
    w = _w(I, 1024, 32, magic=False)
    _wr(w, b"\x00")
    r = I.Rs(w.sink)
    r.set(16 * MiB, 64 * 1024, require_magic=True)
    got, err = r.read(1)
    assert err == ENOMAGIC


def t_flush(I):  # TestFlush eazy_test.go:433-491
    w = _w(I, 1024, 32, magic=False)
    w.flush_threshold = -1
    assert w.write_header() == OK
    _wr(w, b"aaabbb")
    assert w.write_break() == OK
    _wr(w, b"ccc")
    assert len(w.sink) == 0
    assert w.flush() == OK
    assert len(w.sink) == 16
    assert w.write_break() == OK
    assert len(w.sink) == 16
    assert w.flush() == OK
    want = bytes([Meta, MetaReset, 10, Literal | 6]) + b"aaabbb" + bytes([Meta, MetaBreak | MetaLen0, Literal | 3])
    want += b"ccc" + bytes([Meta, MetaBreak | MetaLen0])
    assert w.sink == want
    r = I.Rs(w.sink)
    assert r.read(10) == (b"aaabbb", EBREAK)
    assert r.read(10) == (b"ccc", EBREAK)
    assert r.read(10) == (b"", EOF)


def t_flush_reset(I):  # TestFlushReset eazy_test.go:493-512
    w = _w(I, 1024, 32, magic=False)
    w.flush_threshold = -1
    _wr(w, b"123")
    assert len(w.sink) == 0
    w.reset()
    w.flush_threshold = 0
    _wr(w, b"456")
    assert w.sink == bytes([Meta, MetaReset, 10, Literal | 3]) + b"456"


def _intersection(I, msg2f):  # testIntersection eazy_test.go:539-579
    rng = np.random.default_rng(0)
    w = I.W(1024, 512)
    msg = (rng.integers(0, 0x78 - 0x20, 1024) + 0x20).astype(np.uint8).tobytes()
    _wr(w, msg)
    msg2 = msg2f(rng, msg)
    _wr(w, msg2)
    r = I.Rb(w.sink)
    got, err = r.read(len(msg) + len(msg2) + 10)
    assert err == EOF
    assert got == msg + msg2


def t_intersection_long(I):  # TestIntersectionLong eazy_test.go:514-526
    def f(rng, msg):
        head = (rng.integers(0, 0x78 - 0x20, 0x10) + 0x20).astype(np.uint8).tobytes()
        return head + msg[:0x10]

    _intersection(I, f)


def t_intersection_short(I):  # TestIntersectionShort eazy_test.go:528-537
    _intersection(I, lambda rng, msg: msg[len(msg) - 0x10 :] + msg[:0x10])


def t_runlen_decoder(I):  # TestRunlenDecoder eazy_test.go:581-597
    b = bytes([Meta, MetaReset, 4, Meta, MetaVer, 0, Literal | 1]) + b"a" + bytes([Copy | 5, OffLong, 1])
    b += bytes([Literal | 2]) + b"bc" + bytes([Copy | 5, OffLong, 2, Literal | 2]) + b"xx"
    r = I.Rs(b)
    assert r.read(1000) == (b"aaaaaabcbcbcbxx", EOF)


def t_runlen_encoder(I):  # TestRunlenEncoder eazy_test.go:599-670
    w = I.W(128, 16)
    _wr(w, b"\x00")
    off = len(w.sink)
    _wr(w, b"aaaaaaabcbcbcbcbxx")
    assert w.sink[off:] == bytes([Literal | 1]) + b"a" + bytes([Copy | 6, OffLong, 1, Literal | 2]) + b"bc" + bytes(
        [Copy | 7, OffLong, 2, Literal | 2]
    ) + b"xx"
    data = bytearray((b"0" * 32 * 130)[:0x1005])
    off = len(w.sink)
    _wr(w, bytes(data))
    enclen = 0x1005 - 1 - Len1 - 0x100
    assert w.sink[off:] == bytes([Literal | 1]) + b"0" + bytes([Copy | Len2, enclen & 0xFF, enclen >> 8, OffLong, 1])
    data[3:] = bytes(len(data) - 3)
    off = len(w.sink)
    _wr(w, bytes(data))
    enclen = 0x1005 - 3 - Len1 - 0x100
    assert w.sink[off:] == bytes([Literal | 3]) + b"000" + bytes([Copy | Len2, enclen & 0xFF, enclen >> 8, OffLong, 0])


def _giant(I, f):  # testGiantLiteral eazy_test.go:722-747
    rng = np.random.default_rng(0)
    w = I.W(1024, 512)
    msg = f(rng, 1024)
    _wr(w, msg)
    r = I.Rb(w.sink)
    got, err = r.read(len(msg))
    assert err == OK
    assert got == msg


def _rnd_msg(rng, n):
    return bytearray((rng.integers(0, 0x78 - 0x20, n) + 0x20).astype(np.uint8).tobytes())


def t_giant_literal(I):  # TestGiantLiteral eazy_test.go:672-720
    cp = b"0123456789abcdefgh"

    def no_copies(rng, bs):
        return bytes(_rnd_msg(rng, 2 * bs))

    def long_copy(rng, bs):
        m = _rnd_msg(rng, 2 * bs)
        m[: len(cp)] = cp
        m[len(m) - len(cp) :] = cp
        return bytes(m)

    def short_copy(rng, bs):
        m = bytearray(long_copy(rng, bs))
        m[len(m) - bs + 3 : len(m) - bs + 3 + len(cp)] = cp
        return bytes(m)

    for f in (no_copies, long_copy, short_copy):
        _giant(I, f)


def t_unsupported_version(I):  # TestUnsupportedVersion eazy_test.go:749-762
    w = _w(I, 1024, 32, ver=1)
    w.write(b"\x01\x02")
    r = I.Rb(w.sink)
    got, err = r.read(1)
    assert err == EUNSUPVER
    assert got == b""


def t_meta(I, enc_meta):  # TestMeta eazy_test.go:764-815 (enc_meta: Encoder.Meta)
    some = MetaTagMask
    w = _w(I, 1024, 32, magic=False)
    _wr(w, b"\x01")
    b = bytearray(w.sink)
    b += enc_meta(some, 0)
    b += enc_meta(some, 4) + bytes([1, 2, 3, 4])
    b += enc_meta(some, 128)
    blob = bytearray(128)
    blob[:10] = b"0123456789"
    blob[-10:] = b"9876543210"
    b += blob
    b += enc_meta(some, 256)
    blob = bytearray(256)
    blob[:6] = b"abcdef"
    blob[-10:-4] = b"fedcba"
    b += blob
    st = len(w.sink)
    _wr(w, b"\x02")
    b += w.sink[st:]
    r = I.Rb(bytes(b))
    r.set(0, 0, skip_unsupported_meta=True)
    assert r.read(3) == (b"\x01\x02", EOF)


def t_long_len_off(I):  # TestLongLenOff eazy_test.go:817-856
    rng = np.random.default_rng(0)
    w = I.W(1 << 18, 1 << 16)
    msg = _rnd_msg(rng, 1 << 17)
    _wr(w, bytes(msg))
    src = w.sink
    r = I.Rs(src)
    got, err = r.read(len(msg) + 1)
    assert err == EOF
    assert got == bytes(msg)
    msg[128:] = _rnd_msg(rng, len(msg) - 128)
    st = len(w.sink)
    _wr(w, bytes(msg))
    r.append(w.sink[st:])
    got, err = r.read(len(msg) + 1)
    assert err == EOF
    assert got == bytes(msg)


def t_fuzz_writer_seeds(I):  # FuzzWriter seeds eazy_test.go:1296-1312, body :1314-1361
    seeds = [
        (b"prefix_1234_suffix", b"prefix_567_suffix", b"suffix_prefix"),
        (b"aaaaaa", b"aaaaaaaaaaaa", b"aaaaaaaaaaaaaaaaaaaaaaaa"),
        (b"aaaaab", b"aaaaabaaaaaa", b"aaaaaaaaaaabaaaaaaaaaaaa"),
    ]
    for ps in seeds:
        w = I.W(512, 32)
        for p in ps:
            _wr(w, p)
        r = I.Rb(w.sink)
        out = bytearray()
        while True:
            got, err = r.read(16)
            out += got
            if err == EOF:
                break
            assert err == OK
        assert bytes(out) == b"".join(ps)


def t_sink_failure_resets(I):  # Writer.flush writer.go:387-401: a failed write restarts the stream
    w = I.W(1024, 32)
    _wr(w, b"first message, first message")
    good = len(w.sink)
    w.sink_fault(3)
    n, err = w.write(b"second message")
    assert err != OK and n == 0
    st = len(w.sink)  # 3 bytes of the failed write landed
    assert st == good + 3
    _wr(w, b"third message")
    assert w.sink[st : st + len(MAGIC)] == MAGIC  # a fresh stream with a header


ALL = [
    t_magic,
    t_literal,
    t_copy,
    t_bug1,
    t_padding,
    t_zero_region,
    t_reset,
    t_break,
    t_require_magic,
    t_flush,
    t_flush_reset,
    t_intersection_long,
    t_intersection_short,
    t_runlen_decoder,
    t_runlen_encoder,
    t_giant_literal,
    t_unsupported_version,
    t_long_len_off,
    t_fuzz_writer_seeds,
]
