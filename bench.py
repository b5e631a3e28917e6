"""bench.py — device-resident eazy compress+decompress throughput on MI355X.

A step = one pass of the hot path over one batch resident in HBM:
  K1 compress (writer.go Writer.Write per stream) -> K3 pack -> K2 decompress
  (reader.go Reader.Read to EOF per stream).
Workload at N=1 (BASELINE.json configs[1], "c1"): 65,536 independent 4 KiB
log-like streams, NewWriter(MiB, 1024) each.  N>1 (configs[3], "c3"): ONE
global batch of 1,048,576 x 4 KiB streams split into contiguous whole-stream
shards over the ranks (strong scaling); the step adds the one real exchange of
the sharded path, an RCCL all-gather of per-stream compressed sizes into
global packed offsets (eazy_amd/dist.py); gathering the packed
payload to rank 0 is timed separately ("gather").  value = uncompressed GiB
processed by all ranks per second (GiB = 2^30 B).
Unsharded workloads keep two batches in flight (--inflight, default 2): step k
runs whole on HIP stream k mod 2 with its own buffers, so one batch's kernels
fill the SIMDs the other's leave idle; every timed step is still a full K1 + K3
+ K2 of its batch, and both batches' results are checked after the timed steps.
The launches alone (one batch at a time, after the timed region) are reported
as kernel_ms_isolated / roofline_isolated.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       (N>1: under python -m torch.distributed.run --nproc-per-node N bench.py --gpus N, or
        bench.py --gpus N alone, which starts that launcher as a child process itself)
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)

METRIC = "device-resident compress+decompress GiB/s, 1 MiB block, 1/2/4/8 MI355X"  # BASELINE.json
SHARDED = {"c3"}  # workloads whose stream count is the GLOBAL batch, split over the ranks
WORKLOADS = {
    # name: (streams per GPU (c3: in the whole job), bytes per stream, block, htable, description)
    "c1": (65536, 4096, 1 << 20, 1024, "c1: 65536 x 4 KiB log-like streams per GPU, block 1 MiB, htable 1024"),
    "c3": (1 << 20, 4096, 1 << 20, 1024,
           "c3: one batch of 1048576 x 4 KiB log-like streams sharded over the GPUs, block 1 MiB, htable 1024"),
    "c2": (4096, 256 << 10, 1 << 20, 1024, "c2: 4096 x 256 KiB log-like streams per GPU, block 1 MiB, htable 1024"),
    # C4, the gradient-wire retarget: tensor buckets bit-cast to bytes (Writes longer than the window)
    "c4": (64, 4 << 20, 1 << 20, 1024, "c4: 64 x 4 MiB fp32 N(0,1e-3) gradient buckets per GPU, block 1 MiB, htable 1024"),
    "c4h": (64, 4 << 20, 1 << 20, 1024, "c4h: 64 x 4 MiB bf16 N(0,1e-3) gradient buckets per GPU, block 1 MiB, htable 1024"),
    "c4s": (64, 4 << 20, 1 << 20, 1024, "c4s: 64 x 4 MiB fp32 buckets, 90% zeros, block 1 MiB, htable 1024"),
}


def workload_bytes(name, seed, total):
    """Host bytes of a workload (seeded): log events, or gradient buckets."""
    import numpy as np

    from eazy_amd import synth

    if name in ("c1", "c2"):
        return synth.logs(seed, total), "synthetic (seeded tlwire-like log events, eazy_amd/tools/synth.c)"
    if name == "c3":  # streams [first, last) of the global batch (rank-independent bytes)
        first, last, size = seed
        return (synth.global_logs(1000, first, last, size),
                "synthetic (seeded tlwire-like log events, eazy_amd/tools/synth.c; one global batch)")
    if name == "c4h":
        f = synth.f32(seed, total // 2)
        return (f.view(np.uint32) >> 16).astype(np.uint16).view(np.uint8), "synthetic (seeded bf16 = top half of N(0,1e-3) fp32)"
    f = synth.f32(seed, total // 4)
    if name == "c4s":
        rng = np.random.default_rng(seed)
        f[rng.random(f.shape[0]) < 0.9] = 0.0
        return f.view(np.uint8), "synthetic (seeded N(0,1e-3) fp32, 90% zeros)"
    return f.view(np.uint8), "synthetic (seeded N(0,1e-3) fp32)"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="auto", choices=["auto"] + sorted(WORKLOADS),
                    help="auto: c1 on one GPU (BASELINE configs[1]), c3 sharded over N>1 GPUs (configs[3])")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="bounded CPU-baseline sample duration")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-memory (PCIe-inclusive) measurement")
    ap.add_argument("--e2e-chunks", type=int, default=4, help="stream chunks of the overlapped host-memory measurement")
    ap.add_argument("--stream-bytes", type=int, default=0, help="override the workload's stream size (experiments)")
    ap.add_argument("--no-check", action="store_true", help="skip the round-trip checks (timing experiments only)")
    ap.add_argument("--same", action="store_true", help="every stream a copy of stream 0 (divergence experiments)")
    ap.add_argument("--streams", type=int, default=0, help="override the workload's stream count (experiments)")
    ap.add_argument("--traffic-json", default=None,
                    help="PMC-derived HBM bytes per launch (tools/traffic.py); default: the committed "
                         "profiles/traffic_<workload>.json when its kernel-source hash and shape match this run")
    ap.add_argument("--no-gather", action="store_true", help="N>1: skip the timed payload gather to rank 0")
    ap.add_argument("--inflight", type=int, default=0,
                    help="batches in flight: step k runs on HIP stream k mod this, each with its own buffers (0: 2, "
                         "or 1 for a sharded workload, whose step holds an RCCL exchange)")
    ap.add_argument("--rehearse", action="store_true",
                    help="CPU rehearsal of the N-rank launch and exchange (gloo, no kernels: each stream's payload is "
                         "its raw bytes); prints one JSON line with no throughput claim")
    return ap.parse_args()


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(nproc: int, argv: list[str]) -> int:
    """`python bench.py --gpus N` (N > 1) outside torch.distributed.run: start
    N ranks as ONE child process tree (torch.distributed.run, 127.0.0.1
    rendezvous) before anything here touches the GPU, let rank 0's JSON line
    through on the inherited stdout, and return the child's exit code."""
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + argv
    return subprocess.run(cmd, env=dict(os.environ)).returncode


def source_hash() -> str:
    """Hash of everything that decides the kernels' code (HIP sources, headers,
    build flags), comments and blank lines removed: PMC traffic measured at one
    hash is valid for any commit with the same hash.  Diagnostic-only code (the
    `#if (EZ_EXP ...)` blocks without an `#else`, EZ_PROF_MARK lines) is left out
    too: the product build compiles none of it."""
    import glob
    import hashlib
    import re

    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(ROOT, "eazy_amd", "csrc", "*"))) + [
        os.path.join(ROOT, "include", "eazy.h"), os.path.join(ROOT, "eazy_amd", "Makefile")]
    for f in files:
        text = open(f, "rb").read().decode("utf-8", "replace")
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        text = re.sub(r"#if \(EZ_EXP[^\n]*\n(?:(?!#else|#endif|#if).)*?#endif", "", text, flags=re.S)
        text = re.sub(r"\n\s*EZ_PROF_MARK\(\d+\);", "", text)
        lines = (re.sub(r"(^|\s)(//|#\s).*$", "", ln).rstrip() for ln in text.splitlines())
        h.update(os.path.basename(f).encode())
        h.update("\n".join(ln for ln in lines if ln).encode())
    return h.hexdigest()[:16]


def load_traffic(path, workload, count, size, dom):
    """HBM bytes per launch of the dominant stage from a PMC summary (FETCH_SIZE +
    WRITE_SIZE summed over the stage's kernels, FETCH_SIZE doubled only for the
    coalesced-stream kernels, tools/traffic.py) -> (bytes or None, provenance,
    {"raw": FETCH_SIZE as counted, "x2": every FETCH_SIZE doubled} or None)."""
    if path is None:
        path = os.path.join(ROOT, "profiles", f"traffic_{workload}.json")
        if not os.path.exists(path):
            return None, "no committed PMC summary for this workload", None
        t = json.load(open(path))
        key = (t.get("source_hash"), t.get("streams"), t.get("stream_bytes"))
        if key != (source_hash(), count, size):
            return None, f"{os.path.relpath(path, ROOT)} was measured on other kernel sources or shape", None
    elif not os.path.exists(path):
        return None, f"{path} missing", None
    else:
        t = json.load(open(path))
    kern = t.get("kernels", t)
    # the stage's kernels: K1 = the parses and writers (k1_*), K1x's rounds (kx_*), K1c's chunks (kc_*)
    # and the wide token writer (ke_*); K2 = the decoders (k2_*), K2j (kj_*) and the deferred-literal
    # copy (kd_copy); K3 = k3_*; per step (a kernel a step runs several times counts every dispatch)
    pre = {"k1_compress": ("k1_", "kx_", "kc_", "ke_"), "k2_decompress": ("k2_", "kd_", "kj_"), "k3_pack": ("k3_",)}[dom]
    # (per_step is null in a profile without a k3_gather dispatch to count steps by: the per-launch figure)
    def stage(key, per):
        vals = [v[per] if v.get(per) is not None else v.get(key) for k, v in kern.items() if k.startswith(pre) and v.get(key)]
        return sum(vals) if vals else None

    src = os.path.relpath(path, ROOT) if path.startswith(ROOT) else path
    alt = {"raw": stage("traffic_raw", "per_step_raw"), "x2": stage("traffic_x2", "per_step_x2")}
    return stage("traffic", "per_step"), f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, {src}", alt


def _oracle_pass(orc, host, offs, block, htable, threads, seconds, g_packed=None, g_off=None):
    """Chunks of 2,048 streams through the C oracle until `seconds` of CPU time
    or the whole batch; with the GPU's packed bytes given, every stream the
    oracle compressed is byte-compared with the GPU's (sizes and bytes)."""
    import numpy as np

    count = len(offs) - 1
    chunk = min(count, 2048)
    done_bytes, t_c, t_d, k, checked = 0, 0.0, 0.0, 0, 0
    while (t_c + t_d) < seconds and k < count // chunk:
        s0 = k * chunk
        o = (offs[s0 : s0 + chunk + 1] - offs[s0]).astype(np.int64)
        data = host[offs[s0] : offs[s0 + chunk]]
        n = np.diff(o)
        slot_off = np.concatenate([[0], np.cumsum(n + (n >> 2) + 32)]).astype(np.int64)
        t0 = time.perf_counter()
        slots, sizes = orc.compress_batch(block, htable, data, o, slot_off, threads)
        t1 = time.perf_counter()
        out, osz = orc.decompress_batch(slots, slot_off, sizes, o, threads)
        t2 = time.perf_counter()
        assert np.array_equal(out, data), "oracle round trip failed"
        if g_packed is not None:
            g_sz = np.diff(g_off[s0 : s0 + chunk + 1])
            bad = np.nonzero(g_sz != sizes)[0]
            assert len(bad) == 0, f"stream {s0 + bad[0]}: GPU compressed size {g_sz[bad[0]]} != oracle {sizes[bad[0]]}"
            keep = np.concatenate([np.arange(slot_off[s], slot_off[s] + sizes[s]) for s in range(chunk)])
            got = g_packed[g_off[s0] : g_off[s0 + chunk]]
            if not np.array_equal(slots[keep], got):
                for s in range(chunk):
                    w = slots[slot_off[s] : slot_off[s] + sizes[s]]
                    g = g_packed[g_off[s0 + s] : g_off[s0 + s + 1]]
                    assert np.array_equal(w, g), f"stream {s0 + s}: GPU compressed bytes differ from the oracle"
            checked += chunk
        t_c += t1 - t0
        t_d += t2 - t1
        done_bytes += int(o[-1])
        k += 1
    return done_bytes, t_c, t_d, k * chunk, checked


def cpu_baseline(host, offs, block, htable, seconds, g_packed, g_off):
    """The CPU restatement of the reference (oracle/, 'port') on a bounded
    sample of the same workload, one stream per task over the box's CPU share
    (16 threads), and again on one thread.  The multi-thread
    pass byte-compares every stream it compressed with the GPU's bytes."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc

    threads = max(1, min(16, os.cpu_count() or 1))
    count = len(offs) - 1
    done, t_c, t_d, streams, checked = _oracle_pass(orc, host, offs, block, htable, threads, seconds, g_packed, g_off)
    done1, t_c1, t_d1, streams1, _ = _oracle_pass(orc, host, offs, block, htable, 1, seconds / 2)
    gib, gib1 = done / 2**30, done1 / 2**30
    return {
        "value": gib / (t_c + t_d),
        "unit": "GiB/s",
        "cores": threads,
        "kind": "port",
        "compress_GiBps": gib / t_c,
        "decompress_GiBps": gib / t_d,
        "single_thread": {"value": gib1 / (t_c1 + t_d1), "compress_GiBps": gib1 / t_c1, "decompress_GiBps": gib1 / t_d1,
                          "cores": 1, "sample": f"{streams1} streams ({done1 / 2**20:.0f} MiB)"},
        "sample": f"{streams} of the {count} streams of this rank's batch ({done / 2**20:.0f} MiB), "
        f"C restatement of writer.go/reader.go (oracle/eazy_oracle.c, -O3), fresh NewWriter/NewReaderBytes per stream, "
        f"{threads} host threads",
    }, checked


def e2e(ez, data, off, cb, packed, poff, ws, dws, out, osz, ost, block, htable, size, total, comp_bytes, reps=5):
    """The path as the io.Writer / io.Reader caller sees it: the batch starts
    and ends in pinned host memory.  compress = H2D(input) + K1 + K3 +
    D2H(packed); decompress = H2D(packed) + K2 + D2H(output).  Not `value`."""
    import torch

    h_in = torch.empty(total, dtype=torch.uint8, pin_memory=True)
    h_in.copy_(data[:total].cpu())
    h_packed = torch.empty(comp_bytes, dtype=torch.uint8, pin_memory=True)
    h_out = torch.empty(total, dtype=torch.uint8, pin_memory=True)
    d_in = torch.empty_like(data)
    d_packed = torch.empty_like(packed)

    def comp():
        d_in[:total].copy_(h_in, non_blocking=True)
        ez.compress_batch(d_in, off, block, htable, max_len=size, out=cb)
        ez.pack(cb, packed, poff, ws)
        h_packed.copy_(packed[:comp_bytes], non_blocking=True)

    def decomp():
        d_packed[:comp_bytes].copy_(h_packed, non_blocking=True)
        ez.decompress_batch(d_packed, poff, off, out=out, sizes=osz, status=ost, workspace=dws, max_len=size)
        h_out.copy_(out[:total], non_blocking=True)

    t = {}
    for name, f in (("compress", comp), ("decompress", decomp)):
        f()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            f()
        torch.cuda.synchronize()
        t[name] = (time.perf_counter() - t0) / reps
    assert bool(torch.equal(h_out, h_in)), "host round trip differs"
    gib = total / 2**30
    return {"compress_GiBps": gib / t["compress"], "decompress_GiBps": gib / t["decompress"],
            "note": "pinned host -> HBM -> kernels -> pinned host, hipMemcpyAsync on the compute stream, one rank"}


def e2e_pipelined(ez, data, off, offs, cb, packed, poff, dws, out, osz, ost, block, htable, size, total, comp_bytes,
                  chunks=4, reps=5):
    """The host-memory path with the copies overlapped: the batch is cut into `chunks`
    runs of whole streams; chunk k+1's host->HBM copy (one copy stream), chunk k's
    kernels (the compute stream) and chunk k-1's HBM->host copy (a second copy
    stream) run at once.  Chunk offsets are absolute (in_off / slot_off / out_off
    views), so the kernels see sub-batches of the same buffers.  The packed bytes of
    the chunks, back to back, are the one-batch packing; both are checked."""
    import numpy as np
    import torch

    count = len(offs) - 1
    bounds = [count * k // chunks for k in range(chunks + 1)]
    h_in = torch.empty(total, dtype=torch.uint8, pin_memory=True)
    h_in.copy_(data[:total].cpu())
    h_ref = packed[:comp_bytes].cpu()
    packed = torch.empty_like(packed)  # this run's own packing: the caller's one-batch result stays intact
    h_packed = torch.empty(comp_bytes, dtype=torch.uint8, pin_memory=True)
    h_out = torch.empty(total, dtype=torch.uint8, pin_memory=True)
    h_size = torch.zeros(chunks, dtype=torch.int64, pin_memory=True)
    d_in = torch.empty_like(data)
    d_packed = torch.empty_like(packed)
    slot_host = cb.slot_off.cpu().numpy()
    comp = torch.cuda.current_stream()
    up, down = torch.cuda.Stream(), torch.cuda.Stream()
    ws = [torch.empty(ez._lib().ez_pack_workspace(bounds[k + 1] - bounds[k]), dtype=torch.uint8, device=data.device)
          for k in range(chunks)]
    pofs = [torch.empty(bounds[k + 1] - bounds[k] + 1, dtype=torch.int64, device=data.device) for k in range(chunks)]
    # the decompress side knows each chunk's framing (compressed sizes) as a reader would
    pk_host = [0]

    def comp_run():
        ev_c = []
        hb = 0
        up.wait_stream(comp)  # this run's uploads overwrite inputs the previous run's kernels read

        def drain(k):
            nonlocal hb
            ev_c[k].synchronize()
            n = int(h_size[k])
            base = int(slot_host[bounds[k]])
            with torch.cuda.stream(down):
                h_packed[hb : hb + n].copy_(packed[base : base + n], non_blocking=True)
            hb += n

        for k in range(chunks):
            a, b = bounds[k], bounds[k + 1]
            lo, hi = int(offs[a]), int(offs[b])
            e_in = torch.cuda.Event()
            with torch.cuda.stream(up):
                d_in[lo:hi].copy_(h_in[lo:hi], non_blocking=True)
                e_in.record()
            comp.wait_event(e_in)
            sub = ez.CompressedBatch(cb.slots, cb.slot_off[a : b + 1], cb.sizes[a:b], cb.status[a:b])
            ez.compress_batch(d_in, off[a : b + 1], block, htable, max_len=size, out=sub)
            base = int(slot_host[a])
            ez.pack(sub, packed[base:], pofs[k], ws[k])
            h_size[k : k + 1].copy_(pofs[k][-1:], non_blocking=True)
            e = torch.cuda.Event()
            e.record()
            down.wait_event(e)
            ev_c.append(e)
            if k >= 1:
                drain(k - 1)
        drain(chunks - 1)
        pk_host[0] = hb
        comp.wait_stream(down)  # the next run's kernels start after this run's copies out

    def decomp_run():
        hb = 0
        up.wait_stream(comp)
        for k in range(chunks):
            a, b = bounds[k], bounds[k + 1]
            n = int(h_size[k])
            base = int(slot_host[a])
            e_in = torch.cuda.Event()
            with torch.cuda.stream(up):
                d_packed[base : base + n].copy_(h_packed[hb : hb + n], non_blocking=True)
                e_in.record()
            hb += n
            comp.wait_event(e_in)
            ez.decompress_batch(d_packed[base:], pofs[k], off[a : b + 1], out=out, sizes=osz[a:b], status=ost[a:b],
                                workspace=dws, max_len=size)
            e = torch.cuda.Event()
            e.record()
            down.wait_event(e)
            lo, hi = int(offs[a]), int(offs[b])
            with torch.cuda.stream(down):
                h_out[lo:hi].copy_(out[lo:hi], non_blocking=True)
        comp.wait_stream(down)

    t = {}
    for name, f in (("compress", comp_run), ("decompress", decomp_run)):
        f()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            f()
        torch.cuda.synchronize()
        t[name] = (time.perf_counter() - t0) / reps
    assert pk_host[0] == comp_bytes and bool(torch.equal(h_packed, h_ref)), "chunked packing differs"
    assert bool(torch.equal(h_out, h_in)), "pipelined host round trip differs"
    assert int(cb.status.abs().sum()) == 0 and int(ost.abs().sum()) == 0, "pipelined statuses"
    gib = total / 2**30
    return {"compress_GiBps": gib / t["compress"], "decompress_GiBps": gib / t["decompress"], "chunks": chunks,
            "note": "copies overlapped with the kernels: host->HBM, kernels and HBM->host of consecutive stream "
                    "chunks on three HIP streams, one rank"}


def copy_peak(dev, nbytes: int = 1 << 30, reps: int = 5) -> float:
    """Achievable HBM bandwidth on this box (report both denominators): a
    device-to-device copy of `nbytes`, read + write bytes per second in GB/s."""
    import torch

    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    b.copy_(a)
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(reps):
        b.copy_(a)
    t1.record()
    torch.cuda.synchronize()
    gbs = 2 * nbytes * reps / (t0.elapsed_time(t1) / 1e3) / 1e9
    del a, b
    torch.cuda.empty_cache()
    return gbs


def checksum(x, chunk: int = 1 << 26) -> int:
    """Position-weighted byte checksum of a CUDA uint8 tensor (int64 wraparound
    is fine: both sides compute it the same way)."""
    import torch

    acc = torch.zeros((), dtype=torch.int64, device=x.device)
    for a in range(0, x.numel(), chunk):
        v = x[a : a + chunk].to(torch.int64)
        w = torch.arange(a, a + v.numel(), dtype=torch.int64, device=x.device) % 65521 + 1
        acc += (v * w).sum()
    return int(acc)


def gather_check(ez, ezd, R, packed, goff, count_all, first_all, data, size, dev, reps=3):
    """The optional payload gather of the sharded path, timed
    separately: every rank's packed shard to rank 0 at its global offset.  Then
    rank 0 decodes the gathered global batch (K2 over all streams) and compares
    each rank's range with that rank's input by checksum."""
    import torch

    total_c = int(goff[-1])
    out = torch.empty(total_c + 64, dtype=torch.uint8, device=dev) if R.is_root else None  # +64: decoder over-read slack
    ts = []
    for _ in range(reps):
        ezd.barrier(R)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ezd.gather_payload(packed, goff, count_all, R, out=out)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    (t,) = ezd.reduce_max([min(ts)], R, dev)
    sums = [0] * R.world
    mine = checksum(data[: (first_all[R.rank + 1] - first_all[R.rank]) * size])
    if R.world > 1:
        import torch.distributed as dist

        g = torch.zeros(R.world, dtype=torch.int64, device=dev)
        g[R.rank] = mine
        dist.all_reduce(g)
        sums = g.tolist()
    else:
        sums = [mine]
    if R.is_root:
        in_off = torch.arange(count_all + 1, dtype=torch.int64, device=dev) * size
        dec, dsz, dst = ez.decompress_batch(out, goff, in_off, max_len=size)
        assert int(dst.abs().sum()) == 0, "gathered batch: decode status"
        for k in range(R.world):
            a, b = first_all[k] * size, first_all[k + 1] * size
            assert checksum(dec[a:b]) == sums[k], f"gathered shard of rank {k} does not decode to its input"
    moved = total_c - (ezd.rank_bytes(goff, count_all, R.world)[0][1])
    return {"ms": t * 1e3, "bytes_to_root": moved, "GBps_into_root": moved / t / 1e9 if t > 0 else None,
            "note": "grouped point-to-point sends of each rank's packed shard to rank 0 at its global offset "
                    "(torch.distributed P2P over RCCL); rank 0 then decodes the whole gathered batch and checks "
                    "every rank's range against that rank's input checksum"}


def rehearse(args, R):
    """CPU rehearsal of the sharded path (`--rehearse`, gloo): the same
    launch, shard split, size all-gather, global offsets and payload gather as
    the GPU run, with every stream's payload its own bytes (no kernels, no
    oracle).  Rank 0 checks the gathered batch equals the global input."""
    import numpy as np
    import torch
    import torch.distributed as dist

    from eazy_amd import dist as ezd
    from eazy_amd import synth

    if R.world > 1:
        dist.init_process_group("gloo")
    count_all, size = (args.streams or 4096), (args.stream_bytes or 4096)
    first, last = ezd.shard_range(count_all, R)
    mine = torch.from_numpy(synth.global_logs(1000, first, last, size).copy())
    sizes = torch.full((last - first,), size, dtype=torch.int64)
    goff = ezd.global_offsets(ezd.exchange_sizes(sizes, count_all, R))
    assert int(goff[first]) == first * size and int(goff[last]) == last * size, "global offsets"
    out = ezd.gather_payload(mine, goff, count_all, R)
    total = ezd.reduce_sum([mine.numel()], R)[0]
    if R.is_root:
        want = synth.global_logs(1000, 0, count_all, size)
        assert total == count_all * size and np.array_equal(out.numpy(), want), "gathered batch differs"
        print(json.dumps({"metric": "rehearsal (CPU, gloo, no kernels)", "value": None, "n_gpus": R.world,
                          "streams_total": count_all, "streams_per_rank": ezd.shard_counts(count_all, R.world),
                          "bytes_gathered": int(goff[-1]), "gathered_equals_input": True}), flush=True)
    if R.world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    from eazy_amd import dist as ezd

    R = ezd.from_env()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if args.gpus != R.world:
        sys.exit(f"bench.py: --gpus {args.gpus} but the launch has {R.world} rank(s) (WORLD_SIZE)")
    if args.rehearse:
        return rehearse(args, R)

    import numpy as np
    import torch
    import torch.distributed as dist

    import eazy_amd as ez
    from eazy_amd import synth

    world, rank, local = R.world, R.rank, R.local
    # the rank's device is bound before RCCL starts, and named to it (no guess from the rank)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    wl = args.workload if args.workload != "auto" else ("c1" if world == 1 else "c3")
    count, size, block, htable, desc = WORKLOADS[wl]
    if args.stream_bytes:
        size = args.stream_bytes
        desc += f" (stream size overridden: {size} B)"
    if args.streams:
        count = args.streams
        desc += f" (stream count overridden: {count})"
    sharded = wl in SHARDED
    count_all = count if sharded else count * world
    first_all = [ezd.shard_range(count_all, ezd.Rank(k, world, k))[0] for k in range(world)] + [count_all]
    if sharded:
        first, last = ezd.shard_range(count_all, R)
        count = last - first
        host, data_desc = workload_bytes(wl, (first, last, size), count * size)
    else:
        host, data_desc = workload_bytes(wl, 1000 + rank, count * size)  # this rank's own independent streams
    total = count * size
    offs = synth.batch_offsets(count, size)
    if args.same:
        host = np.tile(host[:size], count)
    data = torch.from_numpy(host).to(dev)
    off = torch.from_numpy(offs).to(dev)
    slot_off = ez.slot_offsets(off)
    # batches in flight: step k on HIP stream k mod inflight with buffer set k mod inflight, so one
    # batch's kernels fill the SIMDs another's leave idle (k1_lean's drain: DESIGN §6); a stream runs
    # its steps in order, so a buffer set is free again when its stream reaches it
    inflight = args.inflight or (1 if sharded else 2)
    if sharded and inflight != 1:
        sys.exit("bench.py: a sharded workload's step holds an RCCL exchange; --inflight 1 only")

    def buffer_set():
        cbk = ez.CompressedBatch(
            torch.empty(int(slot_off[-1]) + 16, dtype=torch.uint8, device=dev),
            slot_off,
            torch.empty(count, dtype=torch.int64, device=dev),
            torch.empty(count, dtype=torch.int32, device=dev),
        )
        return {"cb": cbk, "packed": torch.empty_like(cbk.slots), "poff": torch.empty(count + 1, dtype=torch.int64, device=dev),
                "ws": torch.empty(ez._lib().ez_pack_workspace(count), dtype=torch.uint8, device=dev),
                "dws": torch.empty(ez._lib().ez_decompress_workspace(count), dtype=torch.uint8, device=dev),
                "out": torch.empty(total + 16, dtype=torch.uint8, device=dev),
                "osz": torch.empty(count, dtype=torch.int64, device=dev), "ost": torch.empty(count, dtype=torch.int32, device=dev)}

    sets = [buffer_set() for _ in range(inflight)]
    cb, packed, poff, ws, dws, out, osz, ost = (sets[0][k] for k in ("cb", "packed", "poff", "ws", "dws", "out", "osz", "ost"))
    streams = [torch.cuda.current_stream()] if inflight == 1 else [torch.cuda.Stream(device=dev) for _ in range(inflight)]
    for st_k in streams:
        st_k.wait_stream(torch.cuda.current_stream())  # the input's upload
    goff = [None]
    # the decompress call's extents (ez_batch.in_bytes / out_bytes), as a caller holding the packed
    # offsets on the host gives them: known after the warmup (the workload is fixed) and checked after
    # the timed steps; with them the decoder route needs no read-back inside the step
    hint = {"in_bytes": 0, "out_bytes": 0}

    def step(k=0, ev=None):
        b = sets[k % inflight]
        with torch.cuda.stream(streams[k % inflight]):  # (events record on the step's stream)
            if ev:
                ev[0].record()
            ez.compress_batch(data, off, block, htable, max_len=size, out=b["cb"])
            if ev:
                ev[1].record()
            ez.pack(b["cb"], b["packed"], b["poff"], b["ws"])
            if ev:
                ev[2].record()
            if sharded:  # the sharded path's exchange: per-stream sizes -> global packed offsets on every rank
                goff[0] = ezd.global_offsets(ezd.exchange_sizes(b["poff"][1:] - b["poff"][:-1], count_all, R))
            if ev:
                ev[3].record()
            ez.decompress_batch(b["packed"], b["poff"], off, out=b["out"], sizes=b["osz"], status=b["ost"], workspace=b["dws"],
                                max_len=size, **hint)
            if ev:
                ev[4].record()

    for k in range(args.warmup):
        step(k)
    torch.cuda.synchronize()
    if args.warmup:
        hint = {"in_bytes": int(poff[-1]), "out_bytes": total}

    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(5)] for _ in range(args.steps)]
    ezd.barrier(R)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(k, evs[k])
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    ezd.barrier(R)
    elapsed = t1 - t0
    k1 = sum(e[0].elapsed_time(e[1]) for e in evs) / args.steps
    k3 = sum(e[1].elapsed_time(e[2]) for e in evs) / args.steps
    xch = sum(e[2].elapsed_time(e[3]) for e in evs) / args.steps
    k2 = sum(e[3].elapsed_time(e[4]) for e in evs) / args.steps
    # correctness of the timed steps' results: statuses, sizes and the full round trip on device
    if not args.no_check:
        for b in sets[: min(inflight, args.steps)]:
            assert int(b["cb"].status.abs().sum()) == 0, "compress status"
            assert int(b["ost"].abs().sum()) == 0, "decompress status"
            assert bool(torch.equal(b["out"][:total], data)), "round trip differs"
            assert not hint["in_bytes"] or hint["in_bytes"] == int(b["poff"][-1]), "the decompress extent hint"
        if sharded:
            base = int(goff[0][first_all[rank]])
            assert torch.equal(goff[0][first_all[rank] : first_all[rank + 1] + 1] - base, poff), "global offsets"
    comp_bytes = int(poff[-1])
    # with batches in flight each launch shares the chip with the other batches' kernels, so its event
    # time is longer than the launch alone; the launches alone, after the timed region (untimed): one
    # stream, steps back to back
    iso = None
    if inflight > 1:
        ievs = [[torch.cuda.Event(enable_timing=True) for _ in range(5)] for _ in range(3)]
        torch.cuda.synchronize()
        for e in ievs:
            step(0, e)
        torch.cuda.synchronize()
        iso = [sum(e[a].elapsed_time(e[a + 1]) for e in ievs) / len(ievs) for a in (0, 1, 3)]
    elapsed, k1, k2, k3, xch = ezd.reduce_max([elapsed, k1, k2, k3, xch], R, dev)  # the job ends with its slowest rank
    (comp_all,) = ezd.reduce_sum([comp_bytes], R, dev)
    peak_meas = copy_peak(dev) if rank == 0 else None  # after the timed region: the second denominator

    ms = elapsed / args.steps * 1e3
    gib_step = count_all * size / 2**30
    value = gib_step / (ms / 1e3)
    # roofline of the dominant kernel: algorithmic bytes = input n + compressed c
    kern = {"k1_compress": k1, "k2_decompress": k2, "k3_pack": k3}
    dom = max(kern, key=kern.get)
    alg = total + comp_bytes  # per launch on this rank (n + c), SURVEY.md §8d
    achieved = alg / (kern[dom] / 1e3) / 1e9
    traffic, traffic_src, traffic_alt = load_traffic(args.traffic_json, wl, count, size, dom)

    par = (f"dp{world}: one global batch in contiguous whole-stream shards; RCCL all-gather of per-stream sizes "
           f"-> global offsets in the step" if sharded else
           f"dp{world} (independent stream shards per rank, no data-path collective)")
    res = {
        "metric": METRIC,
        "value": value,
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms,
        "higher_is_better": True,
        "scaling": "strong" if sharded else "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": data_desc,
        "config": {
            "workload": desc,
            "streams_total": count_all,
            "streams_per_gpu": count,
            "stream_bytes": size,
            "block": block,
            "htable": htable,
            "parallelism": par,
            "batches_in_flight": inflight,
        },
        "compress_GiBps": gib_step / ((k1 + k3) / 1e3),
        "decompress_GiBps": gib_step / (k2 / 1e3),
        "ratio": count_all * size / comp_all,
        "kernel_ms": {"k1_compress": k1, "k3_pack": k3, "k2_decompress": k2},
        "roofline": {
            "bound": "hbm",
            "kernel": dom,
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "traffic_raw": (traffic_alt or {}).get("raw"),
            "traffic_all_fetch_doubled": (traffic_alt or {}).get("x2"),
            "traffic_note": "HBM-side bytes per step of the dominant stage (FETCH_SIZE + WRITE_SIZE); FETCH_SIZE "
                            "doubled (the guide's gfx950 correction) only for coalesced-stream kernels, raw for the "
                            "scattered-gather kernels; Infinity-Cache hits are counted",
            "traffic_source": traffic_src,
            "source_hash": source_hash(),
            "algorithmic_bytes_per_launch": alg,
            "achievable_peak": peak_meas,
            "frac_of_achievable": achieved / peak_meas if peak_meas else None,
            "achievable_peak_note": "device-to-device copy of 1 GiB on this box (read + write GB/s), the second denominator",
        },
        "kernel_ms_note": ("event time of each launch in the timed steps, on its own stream; with batches in flight a "
                           "launch shares the chip with the other batch's kernels, so it is longer than the launch alone "
                           "(kernel_ms_isolated, roofline_isolated: the same launches one batch at a time, after the "
                           "timed region)" if inflight > 1 else "event time of each launch in the timed steps"),
        "cpu_baseline": None,
    }
    if iso is not None:
        k1i, k3i, k2i = ezd.reduce_max(iso, R, dev)
        res["kernel_ms_isolated"] = {"k1_compress": k1i, "k3_pack": k3i, "k2_decompress": k2i}
        res["compress_GiBps_isolated"] = gib_step / ((k1i + k3i) / 1e3)
        res["decompress_GiBps_isolated"] = gib_step / (k2i / 1e3)
        domi = {"k1_compress": k1i, "k2_decompress": k2i, "k3_pack": k3i}[dom]
        res["roofline_isolated"] = {"kernel": dom, "achieved": alg / (domi / 1e3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                    "frac": alg / (domi / 1e3) / 1e9 / HBM_PEAK_GBS}
    if sharded:
        res["kernel_ms"]["size_exchange"] = xch
        if not args.no_gather:
            res["gather"] = gather_check(ez, ezd, R, packed, goff[0], count_all, first_all, data, size, dev)
    if not args.no_e2e and world == 1:
        res["e2e"] = e2e(ez, data, off, cb, packed, poff, ws, dws, out, osz, ost, block, htable, size, total, comp_bytes)
        if count >= 2 * args.e2e_chunks:
            res["e2e"]["pipelined"] = e2e_pipelined(ez, data, off, offs, cb, packed, poff, dws, out, osz, ost, block, htable,
                                                    size, total, comp_bytes, chunks=args.e2e_chunks)
    if rank == 0 and not args.no_cpu:  # N > 1: rank 0's shard (the other ranks' streams are alike)
        cb_res, checked = cpu_baseline(host, offs, block, htable, args.cpu_seconds, packed.cpu().numpy(), poff.cpu().numpy())
        res["cpu_baseline"] = cb_res
        res["parity"] = {"streams_byte_compared_with_oracle": checked, "streams": count,
                         "round_trip_on_device": "all streams" if not args.no_check else "skipped"}
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
