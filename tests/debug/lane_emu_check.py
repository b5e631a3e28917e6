"""Run tools/lane_emu (host build of the K1 lane code) on a batch and diff
with the oracle stream by stream.  usage: lane_emu_check.py [count] [size] [seed]"""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import numpy as np

import oracle as orc
from eazy_amd import synth

count = int(sys.argv[1]) if len(sys.argv) > 1 else 512
size = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
seed = int(sys.argv[3]) if len(sys.argv) > 3 else 3
block, htable = 1 << 20, 1024
d = synth.logs(seed, count * size).tobytes()
bufs = [d[k * size : (k + 1) * size] for k in range(count)]
offs = np.concatenate([[0], np.cumsum([len(b) for b in bufs])]).astype(np.uint64)
with tempfile.TemporaryDirectory() as t:
    open(f"{t}/in", "wb").write(b"".join(bufs))
    open(f"{t}/off", "wb").write(offs.tobytes())
    subprocess.run([os.path.join(ROOT, "tools", "lane_emu"), f"{t}/in", f"{t}/off", str(block), str(htable), f"{t}/out", f"{t}/sz"], check=True)
    out = open(f"{t}/out", "rb").read()
    sz = np.frombuffer(open(f"{t}/sz", "rb").read(), np.uint64)
at = 0
bad = 0
for s, b in enumerate(bufs):
    got = out[at : at + int(sz[s])]
    at += int(sz[s])
    want = orc.compress(block, htable, [b])
    if got != want:
        bad += 1
        if bad == 1:
            k = next((j for j in range(min(len(got), len(want))) if got[j] != want[j]), min(len(got), len(want)))
            print(f"stream {s}: first diff at byte {k} (got {len(got)} want {len(want)})")
            print(" got ", got[max(0, k - 16) : k + 16].hex())
            print(" want", want[max(0, k - 16) : k + 16].hex())
print(f"{count - bad}/{count} streams identical")
