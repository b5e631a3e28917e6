"""The C++ restatement of eazy_test.go (tests/cpp/eazy_test.cpp) over the C++
host side (eazy_amd/cpp/eazy.hpp): host-only tests here, all of it on the GPU."""

import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CPP = os.path.join(HERE, "cpp")


def _build():
    p = subprocess.run(["make", "-s", "-C", CPP], capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-2000:]
    return os.path.join(CPP, "eazy_test")


def _run(*args):
    p = subprocess.run([_build(), *args], capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout[-4000:] + p.stderr[-2000:]
    return p.stdout


def test_cpp_host_only():
    out = _run("--cpu")
    assert "7/7 passed" in out


def test_cpp_dump_matches_python_dumper(tmp_path):
    """eazy::Dump (C++ mirror) prints what eazy_amd/dump.py prints, on the reference's KAT
    streams, both fuzz corpora and the synthetic streams of the golden file (host only)."""
    from golden_data import load

    from eazy_amd import dump

    g = load()
    streams = [bytes.fromhex(e["input"]) for e in g["fuzz_reader"]]
    for key in ("fuzz_writer", "synthetic_logs"):
        for e in g[key]:
            streams += [bytes.fromhex(v) for k, v in e.items() if k.startswith("stream_") and isinstance(v, str)]
    # cut streams end in an error line
    streams += [s[: len(s) // 2] for s in streams[-8:]]
    assert len(streams) > 20
    f = tmp_path / "streams.hex"
    f.write_text("\n".join(s.hex() for s in streams) + "\n")
    got = _run("--dump", str(f)).split("\n----\n")
    assert len(got) >= 2 * len(streams)

    class Chunks:  # reads of at most 7 bytes
        def __init__(self, b):
            self.b, self.at = b, 0

        def read(self, k):
            r = self.b[self.at : self.at + min(k, 7)]
            self.at += len(r)
            return r

    from eazy_amd import _strerror

    for k, s in enumerate(streams):
        assert got[2 * k] == dump.Dump(s), s.hex()[:80]
        sink = bytearray()

        class W:
            def write(self, b):
                sink.extend(b)

        tot, err = dump.NewDumper(W()).ReadFrom(Chunks(s))
        assert got[2 * k + 1] == f"{sink.decode()}|{tot}|{_strerror(err)}", s.hex()[:80]


@pytest.mark.gpu
def test_cpp_full(cuda):
    out = _run()
    assert "FAIL" not in out and "25/25 passed" in out
