"""Why a stream of 2,000 x 100-byte Writes reads slower than one of 400-byte Writes: the Reader's
whole decode and the batch decoders on each, timed.  python tools/reader_small.py"""

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
    src = synth.logs(91, 8 << 20).tobytes()
    w0 = ez.NewReaderBytes(orc.compress(1 << 20, 1024, [src[: 8 << 20]]))
    while w0.Read(4096)[1] == ez.OK:
        pass
    for size in (100, 400):
        w = orc.Writer(1 << 20, 1024)
        for k in range(2000):
            w.write(src[k * size : (k + 1) * size])
        comp, plain = w.sink, src[: 2000 * size]
        r = ez.NewReaderBytes(comp)
        t0 = time.perf_counter()
        d, err = r.Read(4096)
        t1 = time.perf_counter()
        n = len(d)
        while err == ez.OK:
            d, err = r.Read(4096)
            n += len(d)
        t2 = time.perf_counter()
        print(f"{size} B Writes: {len(comp)} B in, {n} B out; first Read {1e3 * (t1 - t0):.2f} ms, rest {1e3 * (t2 - t1):.2f} ms, whole {r.whole_decoded}")
        dev = torch.device("cuda:0")
        c = torch.from_numpy(np.frombuffer(comp + bytes(64), np.uint8).copy()).to(dev)
        co = torch.tensor([0, len(comp)], dtype=torch.int64, device=dev)
        oo = torch.tensor([0, 8 * len(comp) + 4096], dtype=torch.int64, device=dev)
        for kind in ("j", "t", ""):
            ez.select_decompress_kernel(kind)
            try:
                for rep in range(3):
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    out, sz, st = ez.decompress_batch(c, co, oo, max_len=8 * len(comp) + 4096)
                    torch.cuda.synchronize()
                    t = time.perf_counter() - t0
                print(f"   batch '{kind}': {1e3 * t:.2f} ms, status {int(st[0])}, size {int(sz[0])}, ran {ez.decompress_kernel_last()!r}, ok {out[: len(plain)].cpu().numpy().tobytes() == plain}")
            finally:
                ez.select_decompress_kernel("")


if __name__ == "__main__":
    main()
