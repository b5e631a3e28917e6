"""Debug helper (GPU box): compress a small batch and dump the first stream
whose bytes differ from the oracle to gpurun_out/k1_mismatch.json."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import numpy as np
import torch

import eazy_amd as ez
import oracle as orc
from eazy_amd import synth

count, size = int(sys.argv[1]) if len(sys.argv) > 1 else 64, 4096
host = synth.logs(3, count * size)
offs = synth.batch_offsets(count, size)
data = torch.from_numpy(host).cuda()
off = torch.from_numpy(offs).cuda()
cb = ez.compress_batch(data, off, ez.MiB, 1024, max_len=size)
torch.cuda.synchronize()
slots = cb.slots.cpu().numpy()
so = cb.slot_off.cpu().numpy()
sz = cb.sizes.cpu().numpy()
st = cb.status.cpu().numpy()
bad = 0
for s in range(count):
    want = orc.compress(ez.MiB, 1024, [host[offs[s]:offs[s + 1]].tobytes()])
    got = slots[so[s]:so[s] + sz[s]].tobytes()
    if got != want:
        bad += 1
        if bad == 1:
            json.dump({"stream": s, "status": int(st[s]), "input": host[offs[s]:offs[s + 1]].tobytes().hex(),
                       "want": want.hex(), "got": got.hex()}, open(os.path.join(ROOT, "gpurun_out", "k1_mismatch.json"), "w"))
print("mismatching streams:", bad, "of", count)
