"""Per-Write latency of the streaming drop-in (one long-lived Writer handle,
ez_writer_write through the C-ABI) for the reference's benchmark shape: many
small Writes of log events on one Writer (eazy_test.go:1156-1193), next to the
C oracle's Writer on one host thread.  Also a Reader.Read loop over the result.
Prints one JSON line.  Usage: python tests/perf_handle.py [--writes K]"""

import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402

import eazy_amd as ez  # noqa: E402
import oracle as orc  # noqa: E402
from eazy_amd import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--writes", type=int, default=2000)
    a = ap.parse_args()
    L = ez._lib()
    src = synth.logs(91, 64 << 20).tobytes()
    res = {}
    # warm-up Reader (first use of the K2j and K2t code objects, the pinned staging window, and the
    # per-device K2j workspace sized for the largest stream below, 8 MiB) so that the first size's
    # rate is not the process's one-time setup
    wr = ez.NewReaderBytes(orc.compress(1 << 20, 1024, [src[: 8 << 20]]))
    while wr.Read(4096)[1] == ez.OK:
        pass
    for size in (100, 400, 1024, 4096):
        ws = [src[k * size : (k + 1) * size] for k in range(a.writes)]
        h = C.c_void_p()
        assert L.ez_writer_new(1 << 20, 1024, 0, C.byref(h)) == 0
        cap = ez.compress_bound(size)
        buf = (C.c_uint8 * cap)()
        n = C.c_size_t()
        outs = []
        for w in ws[:20]:  # warm-up on a throwaway stream
            assert L.ez_writer_write(h, w, size, buf, cap, C.byref(n)) == 0
        assert L.ez_writer_reset(h) == 0
        lat = []
        for w in ws:
            t0 = time.perf_counter()
            assert L.ez_writer_write(h, w, size, buf, cap, C.byref(n)) == 0
            lat.append(time.perf_counter() - t0)
            outs.append(bytes(buf[: n.value]))
        L.ez_writer_free(h)
        gpu = b"".join(outs)
        ow = orc.Writer(1 << 20, 1024)
        t0 = time.perf_counter()
        for w in ws:
            ow.write(w)
        t_cpu = (time.perf_counter() - t0) / len(ws)
        assert gpu == ow.sink, f"size {size}: handle bytes differ from the oracle"
        lat = np.array(lat) * 1e6
        res[str(size)] = {"gpu_us_p50": float(np.median(lat)), "gpu_us_p99": float(np.percentile(lat, 99)),
                          "gpu_MiBps": size / (lat.mean() / 1e6) / 2**20,
                          "cpu_oracle_us": t_cpu * 1e6, "cpu_oracle_MiBps": size / t_cpu / 2**20}
        # the same Writes in batches of 64 (ez_writer_write_batch: one launch per batch)
        ends = (C.c_uint64 * 64)()
        for j in range(64):
            ends[j] = (j + 1) * size
        bcap = 64 * cap
        bbuf = (C.c_uint8 * bcap)()
        oe = (C.c_uint64 * 64)()
        assert L.ez_writer_new(1 << 20, 1024, 0, C.byref(h)) == 0
        outs_b, blat = [], []
        for j in range(0, len(ws) - 63, 64):
            t0 = time.perf_counter()
            assert L.ez_writer_write_batch(h, b"".join(ws[j : j + 64]), ends, 64, bbuf, bcap, oe) == 0
            blat.append(time.perf_counter() - t0)
            outs_b.append(bytes(bbuf[: oe[63]]))
        L.ez_writer_free(h)
        nb = len(outs_b) * 64
        assert b"".join(outs_b) == b"".join(outs[:nb]), f"size {size}: batched bytes differ from the per-Write bytes"
        res[str(size)]["batch64_us_per_write"] = float(np.mean(blat)) / 64 * 1e6
        res[str(size)]["batch64_MiBps"] = 64 * size / float(np.mean(blat)) / 2**20
        # Reader.Read(4 KiB) loop over the stream
        r = ez.NewReaderBytes(gpu)
        got = bytearray()
        t0 = time.perf_counter()
        while True:
            d, err = r.Read(4096)
            got += d
            if err == ez.EOF:
                break
            assert err == ez.OK
        t_r = time.perf_counter() - t0
        assert bytes(got) == b"".join(ws)
        res[str(size)]["reader_4k_MiBps"] = len(got) / t_r / 2**20
    # Reader.Read(4 KiB) loop over a 16 MiB stream: NewReaderBytes (whole-stream decode on the first Read,
    # ez_reader_set_whole) and NewReader over an io.Reader returning 64 KiB pieces (the README's usage:
    # each refill read ahead on the device)
    plain = src[: 16 << 20]
    comp = orc.compress(1 << 20, 1024, [plain[k : k + 65536] for k in range(0, len(plain), 65536)])
    rd = {}

    class Pieces:
        def __init__(self, b, piece):
            self.b, self.at, self.piece = b, 0, piece

        def read_go(self, k):
            m = min(k, self.piece, len(self.b) - self.at)
            d = self.b[self.at : self.at + m]
            self.at += m
            return d, (ez.EOF if self.at == len(self.b) else ez.OK)

    for mode in ("whole", "stream_64k"):
        r = ez.NewReaderBytes(comp) if mode == "whole" else ez.NewReader(Pieces(comp, 65536))
        got = bytearray()
        t0 = time.perf_counter()
        t1 = None
        while True:
            d, err = r.Read(4096)
            t1 = t1 or time.perf_counter()
            got += d
            if err == ez.EOF:
                break
            assert err == ez.OK
        t_r = time.perf_counter() - t0
        assert bytes(got) == plain
        rd[mode + "_MiBps"] = len(plain) / t_r / 2**20
        rd[mode + "_first_read_ms"] = (t1 - t0) * 1e3
        if mode == "stream_64k":
            rd["stream_64k_read_aheads"] = r.ahead_count
    t0 = time.perf_counter()
    assert orc.decompress(comp, 4096)[0] == plain
    rd["cpu_oracle_read4k_MiBps"] = len(plain) / (time.perf_counter() - t0) / 2**20
    # the same Read(4 KiB) loops through the C++ mirror (eazy_amd/cpp/eazy.hpp): the drop-in path
    # without the Python layer's per-call cost
    import subprocess
    import tempfile

    exe = os.path.join(ROOT, "tests", "cpp", "eazy_test")
    if os.path.exists(exe):
        with tempfile.TemporaryDirectory() as d:
            cf, pf = os.path.join(d, "c.bin"), os.path.join(d, "p.bin")
            open(cf, "wb").write(comp)
            open(pf, "wb").write(plain)
            p = subprocess.run([exe, "--perf-reader", cf, pf, "4096", "1"], capture_output=True, text=True, timeout=300)
            line = [x for x in p.stdout.splitlines() if x.startswith("{")]
            if p.returncode == 0 and line:
                j = json.loads(line[0])
                rd["cpp_whole_MiBps"] = j["MiBps"]
                rd["cpp_whole_first_read_ms"] = j["first_read_ms"]
            p = subprocess.run([exe, "--perf-stream", cf, pf, "4096", "65536"], capture_output=True, text=True, timeout=300)
            line = [x for x in p.stdout.splitlines() if x.startswith("{")]
            if p.returncode == 0 and line:
                j = json.loads(line[0])
                rd["cpp_stream_64k_MiBps"] = j["MiBps"]
                rd["cpp_stream_64k_read_aheads"] = j["read_aheads"]
            else:
                rd["cpp_stream_64k_error"] = (p.stdout + p.stderr)[-300:]
    print(json.dumps({"handle_path": res, "writes_per_size": a.writes, "reader_16MiB_read4k": rd,
                      "note": "ez_writer_write per call (Writes up to 48 KiB): one launch of K1L with the token writer fused, "
                              "input and output in the handle's coherent pinned buffer, completion by polling a flag; "
                              "batch64: ez_writer_write_batch of 64 Writes per call"}))


if __name__ == "__main__":
    main()
