"""ez_compress_bound(n) = n + n/4 + 32 (include/eazy.h) is a safe output
capacity for one Writer.Write of n bytes.  CPU only.

Proof (writer.go:206-337, Encoder.Tag/Offset writer.go:537-597):
  * the tokens of one Write partition its n input bytes: literal lengths plus
    copy lengths sum to n (the decoder reproduces exactly n bytes);
  * a copy of length l >= 6 (minCopyChunk, writer.go:119) costs at most l
    bytes: tag 1 B for l < 124 and offset <= 5 B when off >= l (6 <= l), or
    OffLong + 1 B when off < l < 124 (3 <= l); tag <= 5 B + offset <= 6 B
    once l >= 124; a zero region is tag + `ff 00` (writeZeros, >= 8 bytes);
  * every literal token is followed by a copy except the last one, so there
    are at most n/6 + 1 literal tags (zero-length ones included),
    1 byte each, plus at most 4 extra bytes for each literal of length >= 124
    (<= n/124 of them);
  * the header is at most 9 bytes (writer.go:495-517).
Hence c <= n + n/6 + 1 + 4n/124 + 9 < n + n/4 + 32.  The tests check the
bound on the inputs that push the ratio hardest (random bytes = one long
literal; 1-byte literals between 6-byte far copies) and on the corpora."""

import random

import numpy as np
import pytest

import oracle as orc

MiB = 1 << 20


def bound(n):
    return n + n // 4 + 32


def test_bound_matches_library():
    import eazy_amd as ez

    for n in (0, 1, 5, 6, 123, 124, 4096, 65916, 1 << 20, (1 << 32) + 7):
        assert ez._lib().ez_compress_bound(n) == bound(n)


def _adversarial(n, rng):
    """1 literal byte, then a 6-byte match of a chunk placed far back."""
    base = bytearray(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
    chunks = [bytes(rng.integers(0, 256, 6, dtype=np.uint8)) for _ in range(64)]
    out = bytearray()
    for c in chunks:
        out += c + bytes([rng.integers(0, 256)])
    while len(out) < n:
        out += bytes([rng.integers(0, 256)]) + chunks[int(rng.integers(0, 64))]
    return bytes(out[:n]) if n <= len(out) else bytes(base)


@pytest.mark.parametrize("block,htable", [(MiB, 1024), (1024, 32), (64, 16)])
def test_bound_worst_shapes(block, htable):
    rng = np.random.default_rng(7)
    worst = 0.0
    for n in (0, 1, 7, 64, 1000, 4096, 70000):
        for kind in range(4):
            if kind == 0:
                p = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            elif kind == 1:
                p = _adversarial(n, rng)
            elif kind == 2:
                p = bytes(n)
            else:
                p = (b"ab" * n)[:n]
            c = orc.compress(block, htable, [p])
            assert len(c) <= bound(n), (n, kind, len(c))
            if n >= 1000:
                worst = max(worst, (len(c) - 9) / n)
    assert worst < 1.25


def test_bound_per_write_in_long_streams():
    """Each Write of a multi-Write stream stays within bound(len(Write))."""
    rng = random.Random(3)
    w = orc.Writer(1024, 32)
    for _ in range(200):
        n = rng.randrange(0, 3000)
        p = bytes(rng.randrange(0, 256) if rng.random() < 0.7 else 0x41 for _ in range(n))
        before = len(w.sink)
        w.write(p)
        assert len(w.sink) - before <= bound(n)


def test_bound_on_corpora():
    from golden_data import load

    g = load()
    for case in g["fuzz_writer"]:
        for wr in case["writes"]:
            p = bytes.fromhex(wr)
            assert len(orc.compress(MiB, 1024, [p])) <= bound(len(p))
