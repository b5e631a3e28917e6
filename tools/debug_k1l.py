"""K1L debugging (GPU): the planted-match streams of test_k1x_rounds through K1L forced, for each
(block, htable); prints the first differing byte against the oracle per stream."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import numpy as np
import torch

import eazy_amd as ez
import oracle as orc
from test_gpu_batch import _planted

rng = np.random.default_rng(41)
for e in (0, 1, 2, 5, 7, 8, 9, 20):
    _planted(rng, 70000, e, 1 << 20, zeros=e % 2 == 1)
small = [_planted(rng, 80000, e, 4096, zeros=True) for e in (3, 12, 40)]
dev = torch.device("cuda", 0)
lens = np.array([len(b) for b in small], np.int64)
offs = torch.from_numpy(np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)).to(dev)
data = torch.from_numpy(np.frombuffer(b"".join(small), np.uint8).copy()).to(dev)
ez.select_compress_kernel("l")
for block, htable in ((4096, 16), (4096, 4096), (1024, 256), (1 << 20, 1024)):
    cb = ez.compress_batch(data, offs, block, htable)
    packed, poff = ez.pack(cb)
    pk, po = packed.cpu().numpy(), poff.cpu().numpy()
    for s, b in enumerate(small):
        got = pk[po[s] : po[s + 1]].tobytes()
        want = orc.compress(block, htable, [b])
        if got != want:
            k = next((t for t in range(min(len(got), len(want))) if got[t] != want[t]), min(len(got), len(want)))
            print(f"block {block} ht {htable} stream {s}: differ at {k} of {len(want)} (got {len(got)}): got {got[k-4:k+12].hex()} want {want[k-4:k+12].hex()}")
        else:
            print(f"block {block} ht {htable} stream {s}: ok")
