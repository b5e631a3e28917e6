"""Round-6 hardening of the batch C-ABI, on the GPU (through include/eazy.h):

- K2j on a sub-batch view (absolute offsets into a larger batch's buffers) touches nothing outside
  the view's output (the review's ADVICE item on kj_expand / kj_jump / kj_gather);
- the decoder route is the same with and without the extent hints (ez_batch.in_bytes / out_bytes),
  which let a K2j-eligible batch be routed without reading the offsets back;
- the multi-device batches reuse pooled HIP streams and buffers: repeated calls do not grow device
  memory, and ez_release_cached returns it;
- two shards on one device overlap in time on the device (no global lock across K1c's passes);
- the Reader's refill offers the io.Reader what Go's more() does (the slice's capacity, not 1 KiB).
"""

import numpy as np
import pytest

import oracle as orc

pytestmark = pytest.mark.gpu

MiB = 1 << 20


def _log_batch(seed, lens):
    from eazy_amd import synth

    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    host = synth.logs(seed, int(offs[-1]))
    return host, offs


def test_k2j_sub_batch_view_leaves_outside_bytes(cuda):
    """Runs [a, b) of a batch of 1 MiB log streams decoded with K2j forced, each as a view with
    absolute offsets into the whole batch's buffers (sub-batch views): every run's
    streams decode to the input, and the output bytes before and after the run keep their sentinel
    (the previous K2j indexed its pointer array from byte 0 of out and wrote before out_off[0])."""
    import torch

    import eazy_amd as ez

    S, n = 12, 1 << 20
    lens = np.full(S, n, np.int64)
    lens[3] = n - 4097  # (slot ends off 16-byte alignment)
    host, offs = _log_batch(61, lens)
    data = torch.from_numpy(host).to(cuda)
    off = torch.from_numpy(offs).to(cuda)
    cb = ez.compress_batch(data, off, MiB, 1024, max_len=n)
    packed, poff = ez.pack(cb)
    torch.cuda.synchronize()
    assert int(cb.status.count_nonzero()) == 0
    # output slots 7 bytes apart from the inputs' (views' slot starts not 16-byte aligned)
    ooff = offs + 7 * np.arange(S + 1, dtype=np.int64) + 5
    d_ooff = torch.from_numpy(ooff).to(cuda)
    po = poff.cpu().numpy()
    ez.select_decompress_kernel("j")
    try:
        for a, b in ((0, 1), (2, 5), (5, 6), (7, 12), (3, 4)):
            out = torch.full((int(ooff[-1]) + 64,), 0xA5, dtype=torch.uint8, device=cuda)
            sz = torch.zeros(S, dtype=torch.int64, device=cuda)
            st = torch.full((S,), -1, dtype=torch.int32, device=cuda)
            ez.decompress_batch(packed, poff[a : b + 1], d_ooff[a : b + 1], out=out, sizes=sz[a:b], status=st[a:b],
                                max_len=int(np.diff(ooff).max()), in_bytes=int(po[b] - po[a]),
                                out_bytes=int(ooff[b] - ooff[a]))
            torch.cuda.synchronize()
            assert ez.decompress_kernel_last() == "j"
            assert int(st[a:b].count_nonzero()) == 0, (a, b)
            assert sz[a:b].cpu().tolist() == lens[a:b].tolist(), (a, b)
            o = out.cpu().numpy()
            for s in range(a, b):
                assert o[ooff[s] : ooff[s] + lens[s]].tobytes() == host[offs[s] : offs[s + 1]].tobytes(), (a, b, s)
            assert (o[: ooff[a]] == 0xA5).all(), f"run [{a}, {b}): bytes before the view's output were written"
            assert (o[ooff[b] :] == 0xA5).all(), f"run [{a}, {b}): bytes after the view's output were written"
            for s in range(a, b):  # the slot's slack after each stream's output
                assert (o[ooff[s] + lens[s] : ooff[s + 1]] == 0xA5).all(), (a, b, s)
    finally:
        ez.select_decompress_kernel("")


def test_k2_route_same_with_extent_hints(cuda):
    """The automatic decoder route with the caller's extent hints equals the route taken by
    reading the offsets back: a few long log streams (K2j), 4 MiB literal buckets (K2t), many
    short streams (K2r); the bytes agree too."""
    import torch

    import bench
    import eazy_amd as ez

    cases = []
    host, offs = _log_batch(62, np.full(8, 2 * MiB, np.int64))
    cases.append(("logs 8 x 2 MiB", host, offs, None))  # K2j when the output is >= 2 x the input
    f32, _ = bench.workload_bytes("c4", 3, 8 * (4 << 20))
    cases.append(("fp32 8 x 4 MiB", np.ascontiguousarray(f32), np.arange(9, dtype=np.int64) * (4 << 20), "t"))
    host, offs = _log_batch(63, np.full(512, 4096, np.int64))
    cases.append(("logs 512 x 4 KiB", host, offs, "r"))
    for name, host, offs, want in cases:
        data = torch.from_numpy(host).to(cuda)
        off = torch.from_numpy(offs).to(cuda)
        cb = ez.compress_batch(data, off, MiB, 1024)
        packed, poff = ez.pack(cb)
        po = poff.cpu().numpy()
        mx = int(np.diff(offs).max())
        routes = []
        for hints in ({}, {"in_bytes": int(po[-1]), "out_bytes": int(offs[-1])}):
            out, sz, st = ez.decompress_batch(packed, poff, off, max_len=mx, **hints)
            torch.cuda.synchronize()
            routes.append(ez.decompress_kernel_last())
            assert int(st.count_nonzero()) == 0, name
            assert torch.equal(out[: int(offs[-1])], data), name
        if want is None:
            want = "j" if int(offs[-1]) >= 2 * int(po[-1]) else "t"
        assert routes[0] == routes[1] == want, (name, routes)


def test_multi_device_calls_do_not_grow_memory(cuda):
    """20 ez_compress_batch_multi + ez_decompress_batch_multi calls on [0, 0]: the pooled HIP
    streams keep the K1 / K2 scratch keyed to two streams (the previous calls created fresh streams
    each time, leaving a scratch entry behind per call); device memory after the 2nd and the 20th
    call is within 64 MiB, and ez_release_cached returns it to within 64 MiB of the start."""
    import torch

    import eazy_amd as ez

    lens = np.full(96, 256 << 10, np.int64)
    lens[::5] = 3000
    host, offs = _log_batch(64, lens)
    ez.release_cached()
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info()[0]
    after = []
    for it in range(20):
        packed, poff, status = ez.compress_batch_multi(host, offs, MiB, 1024, devices=[0, 0])
        out, sizes, st = ez.decompress_batch_multi(packed, poff, offs, devices=[0, 0])
        assert (status == 0).all() and (st == 0).all() and out.tobytes() == host.tobytes(), it
        after.append(torch.cuda.mem_get_info()[0])
    slack = 64 << 20
    assert after[1] - after[-1] <= slack, f"device memory grew by {(after[1] - after[-1]) >> 20} MiB over 18 calls"
    ez.release_cached()
    torch.cuda.synchronize()
    free1 = torch.cuda.mem_get_info()[0]
    assert free0 - free1 <= slack, f"{(free0 - free1) >> 20} MiB not returned by ez_release_cached"


def test_multi_device_shards_overlap(cuda):
    """A C4s-shaped batch (fp32 buckets, 90 % zeros: K1x, then K1c's passes with their host
    synchronisations) split over [0, 0]: the two shards' device intervals (ez_multi_last_shards,
    HIP events on each shard's stream) overlap, i.e. neither shard waits for the other's
    launches; the packing equals the one-device call's."""
    import bench
    import eazy_amd as ez

    S, n = 16, 4 << 20
    host, _ = bench.workload_bytes("c4s", 5, S * n)
    host = np.ascontiguousarray(host)
    offs = np.arange(S + 1, dtype=np.int64) * n
    p1, o1, s1 = ez.compress_batch_multi(host, offs, MiB, 1024, devices=[0])
    best = None
    for _ in range(2):  # (the first call also allocates)
        p2, o2, s2 = ez.compress_batch_multi(host, offs, MiB, 1024, devices=[0, 0])
        shards = ez.multi_last_shards()
        assert len(shards) == 2 and all(d == 0 for d, _, _ in shards)
        (_, a0, a1), (_, b0, b1) = shards
        ov = min(a1, b1) - max(a0, b0)
        best = ov if best is None else max(best, ov)
    assert (s1 == 0).all() and (s2 == 0).all() and o1.tolist() == o2.tolist() and p1.tobytes() == p2.tobytes()
    assert best > 0, f"the two shards ran one after the other ({shards})"
    # and the batch round-trips
    out, sizes, st = ez.decompress_batch_multi(p2, o2, offs, devices=[0, 0])
    assert (st == 0).all() and out.tobytes() == host.tobytes()


def test_reader_refill_offers_go_capacity(cuda):
    """NewReader(io.Reader): more() offers the io.Reader r.b[end:cap(r.b)] (reader.go:516-543) --
    BufferSize when the buffer is empty, else the rest of the array append(r.b, 1024 zero bytes)
    leaves (Go 1.20's growslice and size classes) -- not 1 KiB; the bytes read are the stream."""
    import eazy_amd as ez

    host, _ = _log_batch(65, [3 * MiB])
    comp = orc.compress(MiB, 1024, [host.tobytes()])
    asks = []

    class Src:
        def __init__(self, b, piece):
            self.b, self.at, self.piece = b, 0, piece

        def read_go(self, k):
            asks.append(k)
            m = min(k, self.piece, len(self.b) - self.at)
            d = self.b[self.at : self.at + m]
            self.at += m
            return d, (ez.EOF if self.at == len(self.b) else ez.OK)

    r = ez.NewReader(Src(comp, 64 << 10))
    got = bytearray()
    while True:
        d, err = r.Read(4096)
        got += d
        if err != ez.OK:
            break
    assert err == ez.EOF and bytes(got) == host.tobytes()
    assert asks[0] == 64 << 10
    assert max(asks[1:]) > 32 << 10, f"the refills offered at most {max(asks[1:])} bytes"
    # the capacity rule itself
    assert ez._go_append_cap(65536, 65536 + 100) == 90112
    assert ez._go_append_cap(65536, 1029) == 65536
    assert ez._go_append_cap(16, 1041) == 1152


def test_bench_batches_in_flight(cuda):
    """bench.py's default schedule (two batches in flight on two HIP streams, each with its own
    buffers) completes every step and checks both batches' statuses and round trips itself; its
    line carries the launches-alone times beside the timed ones."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--no-cpu", "--no-e2e", "--steps", "3", "--warmup", "2",
                        "--streams", "8192"], capture_output=True, text=True, timeout=240, cwd=root)
    assert p.returncode == 0, p.stderr[-2000:]
    d = json.loads(p.stdout.strip().splitlines()[-1])
    assert d["config"]["batches_in_flight"] == 2 and d["value"] > 0
    assert set(d["kernel_ms_isolated"]) == {"k1_compress", "k3_pack", "k2_decompress"}
    assert 0 < d["roofline_isolated"]["frac"] < 1
