"""Token codec (Encoder writer.go:537-621 / Decoder reader.go:346-514):
the reference's varint known answers and short-buffer behaviour
(TestReaderShortBuffer eazy_test.go:858-978, TestPrintLengthEncoding /
TestPrintOffsetEncoding :1406-1497), for the C oracle, the Python oracle and
the product's host codec (libeazy_amd.so ez_encode_* / ez_decode_*).  CPU only."""

import pytest

import oracle as orc
import pyoracle as py

Copy, Literal, OffLong = 0x80, 0x00, 0xFF
ESHORTBUF, EOVERFLOW = 2, 4


def _py_enc(fn):
    def f(a, b):
        buf = bytearray()
        fn(buf, a, b)
        return bytes(buf)

    return f


class _Prod:
    @staticmethod
    def enc_tag(t, l):
        import eazy_amd as ez

        return ez.Encoder().tag(b"", t, l)

    @staticmethod
    def enc_offset(o, l):
        import eazy_amd as ez

        return ez.Encoder().offset(b"", o, l)

    @staticmethod
    def enc_meta(m, l):
        import eazy_amd as ez

        return ez.Encoder().meta(b"", m, l)

    @staticmethod
    def dec_tag(b, st=0):
        import eazy_amd as ez

        return ez.Decoder().tag(b, st)

    @staticmethod
    def dec_offset(b, st, l):
        import eazy_amd as ez

        return ez.Decoder().offset(b, st, l)

    @staticmethod
    def dec_meta(b, st):
        import eazy_amd as ez

        return ez.Decoder().meta(b, st)


class _C:
    enc_tag, enc_offset, enc_meta = staticmethod(orc.enc_tag), staticmethod(orc.enc_offset), staticmethod(orc.enc_meta)
    dec_tag, dec_offset, dec_meta = staticmethod(orc.dec_tag), staticmethod(orc.dec_offset), staticmethod(orc.dec_meta)


class _Py:
    enc_tag = staticmethod(lambda t, l: _py_enc(py.enc_tag)(t, l))
    enc_offset = staticmethod(lambda o, l: _py_enc(py.enc_offset)(o, l))
    enc_meta = staticmethod(lambda m, l: _py_enc(py.enc_meta)(m, l))
    dec_tag = staticmethod(lambda b, st=0: py.dec_tag(b, st))
    dec_offset = staticmethod(py.dec_offset)
    dec_meta = staticmethod(py.dec_meta)


def _panics(f):
    try:
        f()
    except Exception as e:  # noqa: BLE001
        return "anic" in type(e).__name__
    return False


CODECS = [_C, _Py, _Prod]

# SURVEY.md §8c varint boundaries
LEN_KAT = {1: "01", 123: "7b", 124: "7c00", 255: "7c83", 379: "7cff", 380: "7d0000", 381: "7d0100", 65915: "7dffff",
           65916: "7e00000000"}
OFF_KAT = {1: "01", 251: "fb", 252: "fc00", 507: "fcff", 508: "fd0000", 513: "fd0500", 66043: "fdffff",
           66044: "fe00000000"}


@pytest.mark.parametrize("C", CODECS, ids=["c-oracle", "py-oracle", "product"])
def test_length_encoding(C):
    for l, h in LEN_KAT.items():
        assert C.enc_tag(Literal, l).hex() == h
        assert C.enc_tag(Copy, l)[0] == Copy | bytes.fromhex(h)[0]
    for b in (b"\x00", b"\x01", bytes([123]), bytes([124, 0]), bytes([124, 1]), bytes([124, 0xFF]), bytes([125, 0, 0]),
              bytes([125, 1, 0]), bytes([125, 0, 1])):
        t, l, i, e = C.dec_tag(b, 0)
        assert e == 0 and i == len(b)


@pytest.mark.parametrize("C", CODECS, ids=["c-oracle", "py-oracle", "product"])
def test_offset_encoding(C):
    for o, h in OFF_KAT.items():
        assert C.enc_offset(o, 0).hex() == h
    assert C.enc_offset(5, 10).hex() == "ff05"
    assert C.enc_offset(20, 10).hex() == "0a"
    for b in (b"\x00", b"\x01", bytes([251]), bytes([252, 0]), bytes([252, 1]), bytes([252, 0xFF]), bytes([253, 0, 0]),
              bytes([253, 1, 0]), bytes([253, 0, 1]), bytes([0xFD, 0x03, 0x65])):
        off, i, e = C.dec_offset(b, 0, 0)
        assert e == 0 and i == len(b)
    assert C.dec_offset(bytes([0xFD, 0x03, 0x65]), 0, 0)[0] == 26367  # TestBug1's offset


@pytest.mark.parametrize("C", CODECS, ids=["c-oracle", "py-oracle", "product"])
def test_short_buffer_tag(C):  # TestReaderShortBuffer/Tag :863-898
    for tlen in (20, 0x100, 0x200, 0x5000_0000):
        b = C.enc_tag(Copy, tlen)
        for k in range(len(b)):
            tag, _, j, e = C.dec_tag(b[:k], 0)
            assert e == ESHORTBUF and j == 0
            if k > 0:
                assert tag == Copy
        tag, l, j, e = C.dec_tag(b, 0)
        assert (tag, l, j, e) == (Copy, tlen, len(b), 0)
    assert _panics(lambda: C.enc_tag(Literal, 0x1_1000_0000))
    tag, _, j, e = C.dec_tag(bytes([Literal | 127]), 0)
    assert (e, j, tag) == (EOVERFLOW, 0, Literal)


@pytest.mark.parametrize("C", CODECS, ids=["c-oracle", "py-oracle", "product"])
def test_short_buffer_offset(C):  # TestReaderShortBuffer/Offset :900-948
    tlen = 10
    for toff in (20, 0x100, 0x200, 0x500, 0x5000_0000):
        for l in (tlen, toff + tlen):
            b = C.enc_offset(toff, l)
            for k in range(len(b)):
                _, j, e = C.dec_offset(b[:k], 0, l)
                assert e == ESHORTBUF and j == 0
            off, j, e = C.dec_offset(b, 0, l)
            assert (off, j, e) == (toff, len(b), 0)
    assert _panics(lambda: C.enc_offset(0x1_1000_0000, tlen))


@pytest.mark.parametrize("C", CODECS, ids=["c-oracle", "py-oracle", "product"])
def test_short_buffer_meta(C):  # TestReaderShortBuffer/Meta :950-977
    meta = 10 << 3
    for tlen in (0, 4, 0x80, 0x100, 0x200, 0x500, 0x5000_0000):
        b = C.enc_meta(meta, tlen)
        for k in range(1, len(b)):
            tag, _, j, e = C.dec_meta(b[:k], 1)
            assert e == ESHORTBUF and j == 1
            if k > 1:
                assert tag == meta
        tag, l, j, e = C.dec_meta(b, 1)
        assert (tag, l, j, e) == (meta, tlen, len(b), 0)
    assert _panics(lambda: C.enc_meta(1024, 4))  # TestMeta :814
