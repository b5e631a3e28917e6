"""Debug helper (not a test): K1L forced ('l') on small batches vs the oracle; prints the first
differing stream, its length and the token walk around the first differing byte."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "oracle"))
import numpy as np, torch
import eazy_amd as ez
import oracle as orc
from eazy_amd import synth
kind = sys.argv[1] if len(sys.argv) > 1 else "l"
ez.select_compress_kernel(kind)
cases = {"logs4k": [synth.logs(3, 64 * 4096).tobytes()[k * 4096:(k + 1) * 4096] for k in range(64)],
         "rand": [np.random.default_rng(5).integers(0, 4, 3000, dtype=np.uint8).tobytes() for _ in range(8)],
         "runs": [(b"abcdefg" * 500)[:3000], bytes(3000), b"x" * 100 + bytes(500) + b"y" * 50]}
for name, bufs in cases.items():
    lens = np.array([len(b) for b in bufs]); offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    data = torch.from_numpy(np.frombuffer(b"".join(bufs), np.uint8).copy()).cuda()
    cb = ez.compress_batch(data, torch.from_numpy(offs).cuda(), 1 << 20, 1024)
    torch.cuda.synchronize()
    sl, so, sz, st = cb.slots.cpu().numpy(), cb.slot_off.cpu().numpy(), cb.sizes.cpu().numpy(), cb.status.cpu().numpy()
    bad = 0
    for s, b in enumerate(bufs):
        want = orc.compress(1 << 20, 1024, [b])
        got = sl[so[s]:so[s] + sz[s]].tobytes()
        if got != want:
            k = next((i for i in range(min(len(got), len(want))) if got[i] != want[i]), min(len(got), len(want)))
            if bad < 3:
                print(name, "stream", s, "len", len(b), "status", st[s], "sizes", len(got), len(want), "first diff", k)
                print("  got ", got[max(0, k - 12):k + 12].hex())
                print("  want", want[max(0, k - 12):k + 12].hex())
            bad += 1
    print(name, "bad streams", bad, "of", len(bufs))
