"""K2j on one stream of a Reader refill's size (64 KiB of compressed log input, ~128 KiB out) and on
larger ones, repeated: per-call host time and, under rocprofv3 --kernel-trace --stats, its kernels.
python tools/k2j_small.py [compressed KiB ...]"""

import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import eazy_amd as ez  # noqa: E402
import oracle as orc  # noqa: E402
from eazy_amd import synth  # noqa: E402


def main():
    sizes = [int(a) for a in sys.argv[1:]] or [64, 256, 1024]
    dev = torch.device("cuda:0")
    for kib in sizes:
        plain = synth.logs(5, 2 * kib * 1024).tobytes()
        comp = orc.compress(1 << 20, 1024, [plain])
        c = torch.from_numpy(np.frombuffer(comp + bytes(64), np.uint8).copy()).to(dev)
        co = torch.tensor([0, len(comp)], dtype=torch.int64, device=dev)
        cap = 8 * len(comp) + 4096
        oo = torch.tensor([0, cap], dtype=torch.int64, device=dev)
        ws = torch.empty(ez._lib().ez_decompress_workspace(1), dtype=torch.uint8, device=dev)
        out = torch.empty(cap + 16, dtype=torch.uint8, device=dev)
        sz = torch.empty(1, dtype=torch.int64, device=dev)
        st = torch.empty(1, dtype=torch.int32, device=dev)
        for kind in ("j", "t"):
            ez.select_decompress_kernel(kind)
            try:
                ts = []
                for rep in range(12):
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    ez.decompress_batch(c, co, oo, out=out, sizes=sz, status=st, workspace=ws, max_len=cap, in_bytes=len(comp),
                                        out_bytes=cap)
                    torch.cuda.synchronize()
                    ts.append(time.perf_counter() - t0)
                ok = int(st[0]) == 0 and out[: len(plain)].cpu().numpy().tobytes() == plain
                print(f"{len(comp) >> 10} KiB in, {len(plain) >> 10} KiB out, '{kind}': median {1e3 * np.median(ts[2:]):.3f} ms "
                      f"({len(plain) / np.median(ts[2:]) / 2**20:.0f} MiB/s), ok {ok}", flush=True)
            finally:
                ez.select_decompress_kernel("")


if __name__ == "__main__":
    main()
