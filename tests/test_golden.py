"""The C oracle against the committed golden fixtures (inputs from the
reference's testdata/fuzz corpora + seeded synthetic logs; expected outputs
from the independent Python restatement).  CPU only."""

import pytest

import oracle as orc
from golden_data import h, load


def test_fuzz_writer_corpus():
    for e in load()["fuzz_writer"]:
        writes = [h(x) for x in e["writes"]]
        for block, ht in ((512, 32), (1 << 20, 1024)):
            s = orc.compress(block, ht, writes)
            assert s.hex() == e[f"stream_{block}_{ht}"], e["name"]
            for w, want in zip(writes, e[f"single_{block}_{ht}"]):
                assert orc.compress(block, ht, [w]).hex() == want, e["name"]
            out, err, _ = orc.decompress(s, buf_size=16)  # io.CopyBuffer with a 16-byte buffer (:1340)
            assert err == 0 and out == b"".join(writes), e["name"]


def _read_all(r, buf, limit=1 << 16):
    out, errs = bytearray(), []
    while len(out) < limit:
        got, err = r.read(buf)
        out += got
        errs.append(err)
        if err not in (0, 10):
            break
    return {"out": bytes(out[:limit]).hex(), "errs": errs}


@pytest.mark.parametrize("buf", [16, 4096])
def test_fuzz_reader_corpus(buf):
    for e in load()["fuzz_reader"]:
        r = orc.Reader(src=h(e["input"]))
        assert _read_all(r, buf) == e[f"read{buf}"], e["name"]


def test_synthetic_logs():
    for e in load()["synthetic_logs"]:
        b = h(e["input"])
        for block, ht in ((1 << 20, 1024), (1 << 17, 1024), (1024, 32)):
            assert orc.compress(block, ht, [b]).hex() == e[f"stream_{block}_{ht}"]


def test_multi_write():
    m = load()["multi_write"]
    writes = [h(x) for x in m["writes"]]
    assert orc.compress(1 << 20, 1024, writes).hex() == m["stream_1048576_1024"]
    assert orc.compress(2048, 64, writes).hex() == m["stream_2048_64"]
