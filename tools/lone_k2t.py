"""Decode time of ONE long log stream on the batch path (count = 1, the Reader handle's
decode-ahead shape): K2t forced (or K2j with --kind j), CUDA-event timing over a few launches.  With EZ_LIB pointing at
an experiment build (make -C eazy_amd exp X=<bits>) the EZ_EXP phase skips of K2t give the
phase split (wrong bytes, timing only).  Usage: python tools/lone_k2t.py [MiB] [--check] [--kind t|j]"""

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import eazy_amd as ez  # noqa: E402
import oracle as orc  # noqa: E402
from eazy_amd import synth  # noqa: E402


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 16
    plain = synth.logs(91, mib << 20).tobytes()
    comp = orc.compress(1 << 20, 1024, [plain[k : k + 65536] for k in range(0, len(plain), 65536)])
    dev = torch.device("cuda:0")
    c = torch.from_numpy(np.frombuffer(comp, np.uint8).copy()).to(dev)
    coff = torch.tensor([0, len(comp)], dtype=torch.int64, device=dev)
    cap = 8 * len(comp) + 4096
    ooff = torch.tensor([0, cap], dtype=torch.int64, device=dev)
    kind = sys.argv[sys.argv.index("--kind") + 1] if "--kind" in sys.argv else "t"
    ez.select_decompress_kernel(kind)
    out, sizes, status = ez.decompress_batch(c, coff, ooff)
    torch.cuda.synchronize()
    if "--check" in sys.argv:
        assert int(status[0]) == 0 and int(sizes[0]) == len(plain)
        assert out[: len(plain)].cpu().numpy().tobytes() == plain
    ts = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ez.decompress_batch(c, coff, ooff, out=out, sizes=sizes, status=status)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ms = min(ts)
    print(f"lib={os.path.basename(ez.LIB_PATH)} K2{ez.decompress_kernel_last()} {mib} MiB stream ({len(comp)} B compressed): {ms:.2f} ms, "
          f"{len(plain) / ms / 1e3 / 1.048576:.1f} MiB/s, status {int(status[0])}")


if __name__ == "__main__":
    main()
