"""Which streams does the fast decoder hand to the exact decoder? (GPU helper)"""
import sys, os, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import eazy_amd as ez
from eazy_amd import synth

count = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
size = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
kind = sys.argv[3] if len(sys.argv) > 3 else ""  # first K2 kernel ('r', 'w', 't'; '' automatic)
host = synth.logs(1000, count * size)
offs = synth.batch_offsets(count, size)
dev = torch.device("cuda", 0)
data = torch.from_numpy(host).to(dev)
off = torch.from_numpy(offs).to(dev)
cb = ez.compress_batch(data, off, 1 << 20, 1024, max_len=size)
packed, poff = ez.pack(cb)
ws = torch.zeros(ez._lib().ez_decompress_workspace(count), dtype=torch.uint8, device=dev)
ez.select_decompress_kernel(kind)
out, sizes, status = ez.decompress_batch(packed, poff, off, workspace=ws, max_len=size)
torch.cuda.synchronize()
w = ws.view(torch.int32).cpu().numpy()
n = int(w[0])
ids = sorted(int(x) for x in w[1 : 1 + n])
pk = packed.cpu().numpy()
po = poff.cpu().numpy()
if os.environ.get("EZ_LIB", "").endswith("x4096.so"):  # debug build: hand-over codes in the statuses
    st = status.cpu().numpy(); sz = sizes.cpu().numpy()
    bad = np.nonzero(st >= 100)[0]
    print(json.dumps({"handover": [(int(s), int(st[s]) - 100, int(sz[s] & 0xffffffff), int(sz[s] >> 32), int(poff[s + 1] - poff[s])) for s in bad[:20]]}))
    sys.exit(0)
assert bool(torch.equal(out[: count * size], data)), "round trip"
res = {"slow": n, "ids": ids[:50], "status_nonzero": int((status != 0).sum()), "streams": []}
for s in ids[:8]:
    res["streams"].append({"s": s, "comp_len": int(po[s + 1] - po[s]), "head": pk[po[s] : po[s] + 32].tolist(), "tail": pk[max(po[s], po[s + 1] - 32) : po[s + 1]].tolist()})
os.makedirs("gpurun_out", exist_ok=True)
json.dump(res, open("gpurun_out/k2_slow.json", "w"))
print(json.dumps({k: res[k] for k in ("slow", "ids", "status_nonzero")}))
