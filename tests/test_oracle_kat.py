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
