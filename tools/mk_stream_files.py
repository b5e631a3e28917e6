"""Writes the perf_handle reader workload (16 MiB of synthetic logs, compressed as 64 KiB Writes on one
NewWriter(MiB, 1024), by the C oracle) to two files, for eazy_test --perf-stream under a profiler.
python tools/mk_stream_files.py COMP PLAIN"""

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import oracle as orc  # noqa: E402
from eazy_amd import synth  # noqa: E402

plain = synth.logs(2026, 16 << 20).tobytes()
comp = orc.compress(1 << 20, 1024, [plain[k : k + 65536] for k in range(0, len(plain), 65536)])
open(sys.argv[1], "wb").write(comp)
open(sys.argv[2], "wb").write(plain)
