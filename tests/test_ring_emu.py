"""The K2r decoder's per-lane code (eazy_amd/csrc/ez_decompress_ring.hip),
compiled for the host by tools/ring_emu.hip and run stream by stream on the
oracle's compressed streams: the decoded bytes must be the original input.
CPU only — it checks the kernel's logic (LDS ring indexing, mirror, whole-line
flushes, zero history) here; the GPU tests run the same code on the MI355X."""

import os
import subprocess

import numpy as np
import pytest

import oracle as orc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EMU = os.path.join(ROOT, "tools", "ring_emu")


@pytest.fixture(scope="module")
def emu():
    src = os.path.join(ROOT, "tools", "ring_emu.hip")
    deps = [src] + [os.path.join(ROOT, "eazy_amd", "csrc", f) for f in ("ez_decompress_ring.hip", "ez_k2_parse.h", "ez_bytes.h", "ez_format.h",
                                                                              "ez_internal.h")]
    if not os.path.exists(EMU) or os.path.getmtime(EMU) < max(os.path.getmtime(d) for d in deps):
        p = subprocess.run(["/opt/rocm/bin/hipcc", "-O1", "-std=c++17", "--offload-arch=gfx950", "-Wno-align-mismatch",
                            "-o", EMU, src], capture_output=True, text=True, timeout=600)
        assert p.returncode == 0, p.stderr[-2000:]
    return EMU


@pytest.fixture(params=[1, 0], ids=["header-window", "header-per-token"])
def hw(request):
    return request.param


def _run(emu, tmp_path, bufs, block=1 << 20, htable=1024, hw=1):
    comp = [orc.compress(block, htable, [b]) for b in bufs]
    offs = np.concatenate([[0], np.cumsum([len(c) for c in comp])]).astype(np.uint64)
    cap = max(16, max(len(b) for b in bufs))
    (tmp_path / "in").write_bytes(b"".join(comp))
    (tmp_path / "off").write_bytes(offs.tobytes())
    subprocess.run([emu, str(tmp_path / "in"), str(tmp_path / "off"), str(cap), str(tmp_path / "out"), str(tmp_path / "sz"), str(hw)],
                   check=True, timeout=600)
    out = (tmp_path / "out").read_bytes()
    sz = np.frombuffer((tmp_path / "sz").read_bytes(), np.uint64)
    at = 0
    for s, b in enumerate(bufs):
        assert sz[s] != np.uint64(~np.uint64(0)), f"stream {s} (len {len(b)}) handed over"
        assert out[at : at + int(sz[s])] == b, f"stream {s} (len {len(b)})"
        at += int(sz[s])


def test_logs(emu, tmp_path, hw):
    from eazy_amd import synth

    d = synth.logs(3, 256 * 4096).tobytes()
    _run(emu, tmp_path, [d[k * 4096 : (k + 1) * 4096] for k in range(256)], hw=hw)


def test_long_streams(emu, tmp_path, hw):
    """Streams much longer than the ring: far copies read the flushed output."""
    from eazy_amd import synth

    d = synth.logs(5, 4 << 20).tobytes()
    _run(emu, tmp_path, [d[: 1 << 20], d[1 << 20 : (1 << 20) + 100003], d[3 << 20 :]], hw=hw)


def test_edges_random_runs(emu, tmp_path, hw):
    from eazy_amd import synth

    rng = np.random.default_rng(11)
    d = synth.logs(9, 1 << 20).tobytes()
    bufs = [b"", b"a", b"abcd", b"aaaaaaaaaaaa", bytes(64), bytes(7), bytes(9), bytes(17), b"ab" * 40, bytes(1000), b"xyz" * 700]
    at = 0
    for n in rng.integers(0, 9000, 40):
        bufs.append(d[at : at + int(n)])
        at += int(n)
    for k in range(24):
        n = int(rng.integers(100, 20000))
        kind = k % 4
        if kind == 0:
            b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        elif kind == 1:
            b = rng.integers(0, 3, n, dtype=np.uint8).tobytes()
        elif kind == 2:
            b = (bytes(rng.integers(0, 256, 7, dtype=np.uint8)) * (n // 7 + 1))[:n]
        else:
            z = np.zeros(n, np.uint8)
            idx = rng.integers(0, n, n // 10)
            z[idx] = rng.integers(1, 256, len(idx), dtype=np.uint8)
            b = z.tobytes()
        bufs.append(b)
    _run(emu, tmp_path, bufs, hw=hw)
