"""WriteBatch on one Writer handle: k small Writes per ez_writer_write_batch call, K1L per Write
(the automatic choice: two or three launches per Write on the handle's stream) against the general
kernel (forced 'w': one launch for all k Writes).  Prints one JSON line."""

import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]

import eazy_amd as ez  # noqa: E402
import oracle as orc  # noqa: E402
from eazy_amd import synth  # noqa: E402


def run(kind, k, size, reps, src):
    L = ez._lib()
    ez.select_compress_kernel(kind)
    try:
        h = C.c_void_p()
        assert L.ez_writer_new(1 << 20, 1024, 0, C.byref(h)) == 0
        ends = (C.c_uint64 * k)(*[(j + 1) * size for j in range(k)])
        cap = k * ez.compress_bound(size)
        buf = (C.c_uint8 * cap)()
        oe = (C.c_uint64 * k)()
        outs, ts = [], []
        for r in range(reps + 1):
            data = src[r * k * size : (r + 1) * k * size]
            t0 = time.perf_counter()
            assert L.ez_writer_write_batch(h, data, ends, k, buf, cap, oe) == 0
            if r:
                ts.append(time.perf_counter() - t0)
            outs.append(bytes(buf[: oe[k - 1]]))
        L.ez_writer_free(h)
    finally:
        ez.select_compress_kernel("")
    w = orc.Writer(1 << 20, 1024)
    for r in range(reps + 1):
        for j in range(k):
            w.write(src[(r * k + j) * size : (r * k + j + 1) * size])
    assert b"".join(outs) == w.sink, f"{kind!r} k={k} size={size}: bytes differ from the oracle"
    t = sorted(ts)[len(ts) // 2]
    return {"ms_per_batch": t * 1e3, "us_per_write": t / k * 1e6, "MiBps": k * size / t / 2**20}


def main():
    src = synth.logs(17, 32 << 20).tobytes()
    res = {}
    for k, size in ((1000, 100), (64, 100), (64, 1024), (16, 4096), (1, 4096)):
        res[f"{k}x{size}"] = {"auto": run("", k, size, 5, src), "general": run("w", k, size, 5, src)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
