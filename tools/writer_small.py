"""Where a small Write's time goes on the handle path (the review's item: a 100-byte Write's fixed
cost): N Writes of S bytes on one NewWriter(MiB, 1024), per-call host latency; run under rocprofv3
--kernel-trace --hip-trace for the kernels' and the HIP calls' share.  python tools/writer_small.py [S] [N]"""

import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]

import numpy as np  # noqa: E402

import eazy_amd as ez  # noqa: E402
from eazy_amd import synth  # noqa: E402


def main():
    size = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    L = ez._lib()
    src = synth.logs(3, size * n).tobytes()
    h = C.c_void_p()
    assert L.ez_writer_new(1 << 20, 1024, 0, C.byref(h)) == 0
    cap = ez.compress_bound(size) + 64
    out = C.create_string_buffer(cap)
    got = C.c_size_t()
    lat = []
    for k in range(n):
        t0 = time.perf_counter()
        e = L.ez_writer_write(h, src[k * size : (k + 1) * size], size, out, cap, C.byref(got))
        lat.append(time.perf_counter() - t0)
        assert e == 0
    lat = np.array(lat[n // 10 :]) * 1e6
    print(f"{size} B Writes: p50 {np.median(lat):.1f} us, p99 {np.percentile(lat, 99):.1f} us, mean {lat.mean():.1f} us")
    L.ez_writer_free(h)


if __name__ == "__main__":
    main()
