"""Experiment: C1 steps back to back on one stream (as bench.py) against steps pipelined over two
HIP streams (batch k's decompress beside batch k+1's compress, two buffer sets).  Timing only."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import eazy_amd as ez  # noqa: E402
from eazy_amd import synth  # noqa: E402

count, size, block, htable = 65536, 4096, 1 << 20, 1024
dev = torch.device("cuda:0")
data = torch.from_numpy(synth.logs(1000, count * size)).to(dev)
off = torch.from_numpy(synth.batch_offsets(count, size)).to(dev)
slot_off = ez.slot_offsets(off)


def bufs():
    cb = ez.CompressedBatch(torch.empty(int(slot_off[-1]) + 16, dtype=torch.uint8, device=dev), slot_off,
                            torch.empty(count, dtype=torch.int64, device=dev), torch.empty(count, dtype=torch.int32, device=dev))
    return dict(cb=cb, packed=torch.empty_like(cb.slots), poff=torch.empty(count + 1, dtype=torch.int64, device=dev),
                ws=torch.empty(ez._lib().ez_pack_workspace(count), dtype=torch.uint8, device=dev),
                dws=torch.empty(ez._lib().ez_decompress_workspace(count), dtype=torch.uint8, device=dev),
                out=torch.empty(count * size + 16, dtype=torch.uint8, device=dev),
                osz=torch.empty(count, dtype=torch.int64, device=dev), ost=torch.empty(count, dtype=torch.int32, device=dev))


B = [bufs(), bufs()]


def comp(b):
    ez.compress_batch(data, off, block, htable, max_len=size, out=b["cb"])
    ez.pack(b["cb"], b["packed"], b["poff"], b["ws"])


def decomp(b):
    ez.decompress_batch(b["packed"], b["poff"], off, out=b["out"], sizes=b["osz"], status=b["ost"], workspace=b["dws"], max_len=size)


sA = torch.cuda.current_stream()
sB = torch.cuda.Stream()
K = 20
for mode in ("serial", "pipelined", "serial", "pipelined"):
    for _ in range(3):
        comp(B[0]); decomp(B[0])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if mode == "serial":
        for k in range(K):
            comp(B[0]); decomp(B[0])
    else:
        done = [None, None]
        for k in range(K):
            b = B[k & 1]
            if done[k & 1] is not None:
                sA.wait_event(done[k & 1])  # batch k-2's decompress read these buffers
            comp(b)
            e = torch.cuda.Event()
            e.record(sA)
            sB.wait_event(e)
            with torch.cuda.stream(sB):
                decomp(b)
                d = torch.cuda.Event()
                d.record(sB)
            done[k & 1] = d
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / K * 1e3
    ok = all(torch.equal(x["out"][: count * size], data) for x in (B if mode == "pipelined" else B[:1]))
    print(mode, round(ms, 3), "ms/step", round(count * size / 2**30 / (ms / 1e3), 1), "GiB/s", "round trip ok" if ok else "ROUND TRIP DIFFERS")
