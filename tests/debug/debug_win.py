"""Debug helper (not a test): general-kernel output vs the oracle on 64 KiB log streams,
first differing byte per stream (run with EZ_K1W_WIN=<bytes>)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch
import eazy_amd as ez
from oracle import oracle as orc
from eazy_amd import synth
ez.select_compress_kernel("w")
d = synth.logs(5, 8 * 65536).tobytes()
bufs = [d[k * 65536:(k + 1) * 65536] for k in range(8)]
data = torch.from_numpy(np.frombuffer(d, np.uint8).copy()).cuda()
off = torch.arange(9, dtype=torch.int64, device="cuda") * 65536
cb = ez.compress_batch(data, off, 1 << 20, 1024)
torch.cuda.synchronize()
sl, so, sz = cb.slots.cpu().numpy(), cb.slot_off.cpu().numpy(), cb.sizes.cpu().numpy()
for s in range(8):
    want = orc.compress(1 << 20, 1024, [bufs[s]])
    got = sl[so[s]:so[s] + sz[s]].tobytes()
    k = next((i for i in range(min(len(got), len(want))) if got[i] != want[i]), None)
    print(os.environ.get("EZ_K1W_WIN"), s, len(got), len(want), "first diff", k)
