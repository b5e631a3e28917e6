"""NewReader(io.Reader) read-ahead (ez_reader_read with whole == 0, K2j continuing the stream): every
Read's (bytes, error) equals the C oracle's Reader over the same io.Reader (reader.go:116-141, 516-543),
on log streams, Breaks, truncation inside every token kind, a MetaReset mid-stream (handed over: Read by
Read), a corrupted byte, incompressible data (literals across refills), zero runs (long copies), many
small Writes, io.Readers of several piece sizes and Read sizes; the read-ahead count shows the device
path ran."""

import numpy as np
import pytest

import oracle as orc

pytestmark = pytest.mark.gpu

MiB = 1 << 20


class PieceSrc:
    """An io.Reader over bytes that returns at most `piece` bytes per Read, EOF with the last ones."""

    def __init__(self, b, piece):
        self.b, self.at, self.piece, self.asks = b, 0, piece, 0

    def read_go(self, k):
        import eazy_amd as ez

        self.asks += 1
        m = min(k, self.piece, len(self.b) - self.at)
        d = self.b[self.at : self.at + m]
        self.at += m
        return d, (ez.EOF if self.at == len(self.b) else ez.OK)


def _reads(r, sizes, limit=1 << 26):
    """Read with the given sizes (cycled) until an error other than ErrBreak; [(bytes, err)]."""
    out, k, total = [], 0, 0
    while total < limit:
        d, err = r.Read(sizes[k % len(sizes)]) if hasattr(r, "Read") else r.read(sizes[k % len(sizes)])
        out.append((bytes(d), err))
        total += len(d)
        k += 1
        if err not in (0, 10):
            break
    return out


def _check(comp, piece, sizes, want_ahead=True):
    import eazy_amd as ez

    ref = orc.Reader(src=comp, eof_with_data=True, chunk=piece)
    want = _reads(ref, sizes)
    src = PieceSrc(comp, piece)
    r = ez.NewReader(src)
    got = _reads(r, sizes)
    assert len(got) == len(want), (len(got), len(want), got[-1][1], want[-1][1])
    for k, (g, w) in enumerate(zip(got, want)):
        assert g[1] == w[1], f"Read {k}: error {g[1]} != {w[1]}"
        assert g[0] == w[0], f"Read {k}: {len(g[0])} bytes != {len(w[0])}"
    if want_ahead:
        assert r.ahead_count > 0, "the read-ahead did not run"
    return r


def _logs(seed, n):
    from eazy_amd import synth

    return synth.logs(seed, n).tobytes()


@pytest.mark.parametrize("piece", [64 << 10, 9000, 1 << 20])
def test_logs_stream(cuda, piece):
    p = _logs(71, 3 * MiB)
    comp = orc.compress(MiB, 1024, [p])
    r = _check(comp, piece, [4096])
    assert r.ahead_count >= 2


@pytest.mark.parametrize("sizes", [[16], [100_000], [4096, 1, 65536, 333]])
def test_read_sizes(cuda, sizes):
    comp = orc.compress(MiB, 1024, [_logs(72, MiB)])
    _check(comp, 64 << 10, sizes)


def test_breaks_and_small_writes(cuda):
    """Many small Writes with Breaks between some (WriteBreak, writer.go:358-366)."""
    p = _logs(73, 2 * MiB)
    w = orc.Writer(MiB, 1024)
    at, k = 0, 0
    rng = np.random.default_rng(5)
    while at < len(p):
        n = int(rng.integers(1, 3000))
        w.write(p[at : at + n])
        at += n
        k += 1
        if k % 97 == 0:
            w.write_break()
    comp = w.sink
    _check(comp, 64 << 10, [4096])
    _check(comp, 20000, [777, 4096])


def test_truncated_streams(cuda):
    """The stream cut at many points (inside tags, offsets, literal bodies, metas): the Reads up to the
    cut and the io.ErrUnexpectedEOF (or EOF) match."""
    comp = orc.compress(MiB, 1024, [_logs(74, 600_000)])
    rng = np.random.default_rng(6)
    cuts = sorted(set(int(x) for x in rng.integers(9000, len(comp), 24)))
    for c in cuts + [len(comp) - 1, len(comp) - 2, len(comp) - 3]:
        _check(comp[:c], 64 << 10, [4096], want_ahead=False)


def test_reset_mid_stream(cuda):
    """Two streams back to back (the second's MetaReset comes after output: K2j hands that buffer over,
    it is decoded Read by Read) and a third after them."""
    a = orc.compress(MiB, 1024, [_logs(75, 400_000)])
    b = orc.compress(1 << 16, 256, [_logs(76, 300_000)], append_magic=False)
    c = orc.compress(MiB, 1024, [_logs(77, 500_000)])
    _check(a + b + c, 64 << 10, [4096])


def test_corrupted_byte(cuda):
    comp = bytearray(orc.compress(MiB, 1024, [_logs(78, 800_000)]))
    rng = np.random.default_rng(7)
    for at in rng.integers(20, len(comp) - 20, 6):
        bad = bytearray(comp)
        bad[int(at)] ^= 0xFF
        _check(bytes(bad), 64 << 10, [4096], want_ahead=False)


def test_incompressible_and_zero_runs(cuda):
    """Random bytes (literals longer than a refill: the pending literal carried across read-aheads)
    and long zero runs (long copies: output many times the input)."""
    rng = np.random.default_rng(8)
    rnd = rng.integers(0, 256, 900_000, dtype=np.uint8).tobytes()
    _check(orc.compress(MiB, 1024, [rnd]), 64 << 10, [4096])
    z = bytearray(_logs(79, 300_000))
    for k in range(0, len(z), 50_000):
        z[k : k + 20_000] = bytes(20_000)
    mix = bytes(z) + bytes(3 * MiB) + rnd[:100_000]
    _check(orc.compress(MiB, 1024, [mix]), 64 << 10, [4096, 100_000])


def test_cpp_mirror_reader_ahead(cuda):
    """The C++ mirror's NewReader over the same handle path (eazy_test --reader-ahead)."""
    import os
    import subprocess

    exe = os.path.join(os.path.dirname(__file__), "cpp", "eazy_test")
    if not os.path.exists(exe):
        pytest.skip("tests/cpp/eazy_test not built")
    p = subprocess.run([exe, "--reader-ahead"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
