"""Pin the CPU oracle: the reference's own tests (eazy_test.go) against both
restatements (C oracle/, Python tests/pyoracle.py).  CPU only."""

import pytest

import impls
import kat_suite as K
import oracle as orc
import pyoracle as py

IMPLS = [impls.COracle, impls.PyOracle]


@pytest.mark.parametrize("I", IMPLS, ids=lambda i: i.name)
@pytest.mark.parametrize("t", K.ALL, ids=lambda f: f.__name__)
def test_reference_test(I, t):
    t(I)


@pytest.mark.parametrize("I", IMPLS, ids=lambda i: i.name)
def test_meta(I):
    if I is impls.COracle:
        K.t_meta(I, orc.enc_meta)
    else:

        def enc(meta, l):
            b = bytearray()
            py.enc_meta(b, meta, l)
            return bytes(b)

        K.t_meta(I, enc)


@pytest.mark.parametrize("I", IMPLS, ids=lambda i: i.name)
def test_sink_failure_resets(I):
    K.t_sink_failure_resets(I)


def test_writer_panics():
    # Writer.init writer.go:161-169
    for bs, hs in ((31, 16), (33, 16), (1 << 32, 16), (16, 16), (1024, 3), (1024, 6), (1024, 0)):
        with pytest.raises(orc.Panic):
            orc.Writer(bs, hs)
        with pytest.raises(py.Panic):
            py.Writer(bs, hs)


def test_oracle_uint32_position_wrap():
    """SURVEY A.9 on the oracle: a Writer at 2^32 - 10000 loses the matches whose table
    entries were written past 2^32 (uint32 values look ~4 GiB away: far skip), so the same
    Writes compress worse than from position 0; at 2^25 nothing changes."""
    from eazy_amd import synth

    d = synth.logs(71, 16 * 4096).tobytes()
    writes = [d[k * 4096 : (k + 1) * 4096] for k in range(16)]
    out = {}
    for p0 in (0, 1 << 25, (1 << 32) - 10000):
        w = orc.Writer(1 << 20, 1024)
        w.set_pos(p0)
        for p in writes:
            w.write(p)
        out[p0] = w.sink
    assert out[0] == out[1 << 25]
    assert len(out[(1 << 32) - 10000]) > 1.5 * len(out[0])


def test_oracle_batch_spreads_few_streams_over_threads():
    """The CPU baseline's batch runner: a batch of only 64 long streams must
    use every thread (work grains of count / (threads * 4) streams, not 64),
    and give the same bytes as one thread.  (The grain is asserted, not a
    wall-clock speedup: timings on a shared host are noise.)"""
    import os

    import numpy as np

    from eazy_amd import synth

    assert orc.batch_grain(64, 16) == 1 and orc.batch_grain(64, 8) == 2
    assert orc.batch_grain(65536, 16) == 64 and orc.batch_grain(10, 1) == 2 and orc.batch_grain(0, 4) == 1
    threads = min(8, os.cpu_count() or 1)
    count, size = 64, 64 << 10
    # every thread gets at least 4 tasks
    assert count // orc.batch_grain(count, threads) >= 4 * threads
    data = synth.logs(13, count * size)
    offs = (np.arange(count + 1) * size).astype(np.int64)
    slot = (np.arange(count + 1) * (size + size // 4 + 32)).astype(np.int64)
    res = {n: orc.compress_batch(1 << 20, 1024, data, offs, slot, n) for n in (1, threads)}
    assert np.array_equal(res[1][1], res[threads][1]) and np.array_equal(res[1][0], res[threads][0])
