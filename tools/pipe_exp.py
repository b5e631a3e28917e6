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
S2 = [torch.cuda.Stream(), torch.cuda.Stream()]
lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (0, -1)
SP = [torch.cuda.Stream(priority=hi), torch.cuda.Stream(priority=lo)]
print("priority range", lo, hi)
k1ms = {}
for mode in ("serial", "twostream", "twoprio", "serial", "twostream", "twoprio"):
    for _ in range(3):
        comp(B[0]); decomp(B[0])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if mode == "serial":
        for k in range(K):
            comp(B[0]); decomp(B[0])
    elif mode in ("twostream", "twoprio"):  # each batch whole on its own stream, two in flight
        SS = S2 if mode == "twostream" else SP
        ev = torch.cuda.Event()
        ev.record(sA)
        for s2 in SS:
            s2.wait_event(ev)
        kev = []
        for k in range(K):
            with torch.cuda.stream(SS[k & 1]):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                ez.compress_batch(data, off, block, htable, max_len=size, out=B[k & 1]["cb"])
                e1.record()
                kev.append((e0, e1))
                ez.pack(B[k & 1]["cb"], B[k & 1]["packed"], B[k & 1]["poff"], B[k & 1]["ws"])
                decomp(B[k & 1])
        for s2 in SS:
            e2 = torch.cuda.Event()
            e2.record(s2)
            sA.wait_event(e2)
        torch.cuda.synchronize()
        k1ms[mode] = [round(a.elapsed_time(b), 3) for a, b in kev]
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
    ok = all(torch.equal(x["out"][: count * size], data) for x in (B if mode != "serial" else B[:1]))
    print(mode, round(ms, 3), "ms/step", round(count * size / 2**30 / (ms / 1e3), 1), "GiB/s", "round trip ok" if ok else "ROUND TRIP DIFFERS")
print("K1 event ms per step", k1ms)
