"""Dumper / Dump (reader.go:43-54, 545-768), host side (eazy_amd/dump.py).

The token walk and its errors are checked against the oracle's decoder on the
reference's KAT streams and FuzzReader corpus; the expected text of
test_dump_runlen_kat is derived by hand from the format verbs of
reader.go:622-700 (the reference's tests only log dumps: the text is parity
unpinned).  CPU only: the token decoders are host code of libeazy_amd.so."""

import os

import oracle as orc
from golden_data import h, load

EXPECT_RUNLEN = (
    '     0     0       0  meta  2 1  "\\x04"    04\n'
    '     3     3       0  meta  1 1  "\\x00"    00\n'
    '     6     6       0  lit     1        "a"\n'
    "     8     8       1  copy    5  off    1  (long)\n"
    '     b     b       6  lit     2        "bc"\n'
    "     e     e       8  copy    5  off    2  (long)\n"
    '    11    11       d  lit     2        "xx"\n'
    "    14     0       f  "
)


def test_dump_runlen_kat():
    """TestRunlenDecoder's stream (eazy_test.go:581-597)."""
    from eazy_amd.dump import Dump

    p = bytes.fromhex("80 10 04 80 08 00 01 61 85 ff 01 02 62 63 85 ff 02 02 78 78")
    assert Dump(p) == EXPECT_RUNLEN


def test_dump_errors():
    import eazy_amd as ez
    from eazy_amd.dump import Dump, Dumper

    # a truncated copy offset: the walk stops at the token's start with ErrShortBuffer
    p = bytes.fromhex("80 10 04 01 61 85")
    d = Dumper()
    d.GlobalOffset = -1
    i, err = d.Write(p)
    assert (i, err) == (5, ez.ESHORTBUF)
    assert Dump(p).endswith("\nerror: short buffer")
    # LenAlt is an overflow (reader.go:367-369)
    i, err = Dumper().Write(b"\x7f")
    assert (i, err) == (0, ez.EOVERFLOW)


def test_go_quote():
    from eazy_amd.dump import go_quote

    assert go_quote(b"some message") == '"some message"'
    assert go_quote(b'a"b\\c') == '"a\\"b\\\\c"'
    assert go_quote(b"\x00\x07\x08\x09\x0a\x0b\x0c\x0d\x1b\x7f") == '"\\x00\\a\\b\\t\\n\\v\\f\\r\\x1b\\x7f"'
    assert go_quote("héllo ☃".encode()) == '"héllo ☃"'
    assert go_quote(b"\xff\xc3") == '"\\xff\\xc3"'  # invalid UTF-8 bytes
    assert go_quote("​\U000e0001".encode()) == '"\\u200b\\U000e0001"'  # format characters


class _BufReader:
    """Go BufReader (eazy_test.go): the last bytes come with io.EOF."""

    def __init__(self, data, step=1 << 16):
        self.data = bytearray(data)
        self.step = step

    def read_go(self, k):
        import eazy_amd as ez

        n = min(k, self.step)
        chunk = bytes(self.data[:n])
        del self.data[:n]
        return chunk, ez.EOF if not self.data else ez.OK


def test_dumper_reference_test():
    """TestDumper (eazy_test.go:980-1010): two Writes with a break and three
    padding bytes between them, dumped through ReadFrom."""
    import eazy_amd as ez
    from eazy_amd.dump import NewDumper

    w1, w2 = b"some message", b"again some message"
    first = orc.compress(1024, 32, [w1])
    both = orc.compress(1024, 32, [w1, w2])
    stream = first + b"\x80\x1f" + bytes(3) + both[len(first):]

    class Sink:
        data = b""

        def write(self, b):
            Sink.data += b

    tags = []
    d = NewDumper(Sink())
    d.Debug = lambda ioff, iend, ooff, tag, l, off: tags.append((chr(tag), ioff, iend, ooff, l))
    n, err = d.ReadFrom(_BufReader(stream))
    assert (n, err) == (len(stream), ez.OK)
    assert d.Close() == ez.OK
    text = Sink.data.decode()
    assert 'lit     c        "some message"' in text
    assert "pad     3" in text
    assert 'meta  3 0  ""' in text  # the break
    assert [t[0] for t in tags][:3] == ["m", "m", "l"] and tags[-1][0] == "e"
    assert tags[-1][3] == len(w1) + len(w2)  # output position at the end
    # the steps tile the input
    steps = [t for t in tags if t[0] != "e"]
    at = 0
    for t in steps:
        assert t[1] == at
        at = t[2] + (t[4] if t[0] in "lm" else 0)
    assert at == len(stream)

    # Fed 7 bytes at a time, a meta tag whose next byte has not arrived is consumed
    # anyway: Decoder.Meta returns the position after the tag with ErrShortBuffer
    # (reader.go:476-477), which Dumper.Write returns as is (:660-663) and ReadFrom
    # drops the tag (:583-584).  The reference's behaviour, kept.
    Sink.data = b""
    d = NewDumper(Sink())
    assert d.ReadFrom(_BufReader(stream, step=7)) == (len(stream), ez.OK)
    assert 'lit     a        "\\fsome mess"' in Sink.data.decode()


def test_dumper_fuzz_reader_corpus():
    """FuzzReader's corpus (testdata/fuzz/FuzzReader): the walk never fails
    unexpectedly, and where the oracle's Reader decodes a stream to its end the
    Dumper walks all of it to the same output length."""
    import eazy_amd as ez
    from eazy_amd.dump import Dump, Dumper

    for e in load()["fuzz_reader"]:
        p = h(e["input"])
        for q in (p, bytes.fromhex("800801801014") + p):
            Dump(q)
            d = Dumper()
            i, err = d.Write(q)
            assert 0 <= i <= len(q)
            assert err in (ez.OK, ez.ESHORTBUF, ez.EOVERFLOW), e["name"]
        r = e["read4096"]
        if r["errs"] == [ez.EOF]:
            d = Dumper()
            i, err = d.Write(p)
            assert (i, err) == (len(p), ez.OK), e["name"]
            assert d.pos == len(h(r["out"])), e["name"]


def test_dumper_synthetic_streams():
    """Dumps of the committed synthetic-log streams account for every input byte
    and every output byte (the token walk matches the stream's decode)."""
    from eazy_amd.dump import Dumper

    for e in load()["synthetic_logs"][:4]:
        raw = h(e["input"])
        s = h(e["stream_1048576_1024"])
        d = Dumper()
        assert d.Write(s) == (len(s), 0)
        assert d.pos == len(raw)
        # through ReadFrom, in one read (a token split between reads is dropped from its
        # tag on, as in the reference: see test_dumper_reference_test)
        pieces = [s]

        class Src:
            def read(self, k, _p=pieces):
                return _p.pop(0) if _p else b""

        d2 = Dumper()
        assert d2.ReadFrom(Src()) == (len(s), 0)
        assert d2.pos == len(raw)


def test_dump_text_go_test_strings():
    """The expected texts go/eazy/eazy_test.go's TestDump carries (uncompiled here: no Go
    toolchain) are what the Python mirror prints for that stream, whole and cut."""
    import re

    from eazy_amd import dump

    c = orc.compress(32, 16, [b"prefix_1234_suffix", b"prefix_567_suffix"], append_magic=False)
    src = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "go", "eazy", "eazy_test.go")).read()
    body = src[src.index("func TestDump"):src.index("func TestHandlesFreedWithoutClose")]

    lit = r'"((?:[^"\\]|\\.)*)"'

    def go_string(var):
        start = body.index(var + " := ") + len(var) + 4
        end = body.index("\n\tif ", start)
        return "".join(p.encode().decode("unicode_escape") for p in re.findall(lit, body[start:end]))

    assert dump.Dump(c) == go_string("want")
    assert dump.Dump(c[:-3]) == go_string("cut")
