"""GPU parity of the batched hot path (K1 compress, K3 pack, K2 decompress)
against the CPU oracle, through the C-ABI (include/eazy.h).

Bar: bit-exact compressed bytes per stream and bit-exact round trips."""

import numpy as np
import pytest

import oracle as orc

pytestmark = pytest.mark.gpu

MiB = 1 << 20


@pytest.fixture(params=["", "S", "w", "x", "l"], ids=["auto", "split32", "general", "k1x", "k1l"], autouse=True)
def k1_kind(request):
    """Every batch test runs on the automatic K1 choice (K1s: the lean parse on the u16
    table at these shapes), on K1s with the u32 exchange table forced, on the
    general wave-per-stream kernel forced, on K1x's rounds forced and on K1L (the lean
    parse with the window's ring semantics) forced (where a batch qualifies: fresh single
    Writes, table <= 4096 entries)."""
    import eazy_amd as ez

    ez.select_compress_kernel(request.param)
    yield request.param
    ez.select_compress_kernel("")


def _run(cuda, bufs, block=MiB, htable=1024, magic=True):
    import torch

    import eazy_amd as ez

    lens = np.array([len(b) for b in bufs], np.int64)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    host = np.frombuffer(b"".join(bufs), np.uint8) if offs[-1] else np.zeros(0, np.uint8)
    data = torch.from_numpy(host.copy()).to(cuda) if len(host) else torch.zeros(1, dtype=torch.uint8, device=cuda)
    off = torch.from_numpy(offs).to(cuda)
    cb = ez.compress_batch(data, off, block, htable, append_magic=magic)
    packed, poff = ez.pack(cb)
    out, sizes, status = ez.decompress_batch(packed, poff, off)
    out2, sizes2, status2 = ez.decompress_batch(packed, poff, off, exact_only=True)
    mx = int(lens.max()) if len(lens) else 0
    others = [ez.decompress_batch(packed, poff, off, max_len=mx)]
    for kind in ("r", "w", "t", "j"):
        ez.select_decompress_kernel(kind)
        try:
            others.append(ez.decompress_batch(packed, poff, off, max_len=mx))
        finally:
            ez.select_decompress_kernel("")
    torch.cuda.synchronize()
    # the ring decoder (default), the wave-per-stream decoder and the exact decoder agree
    assert torch.equal(status, status2) and torch.equal(sizes, sizes2)
    assert torch.equal(out[: int(offs[-1])], out2[: int(offs[-1])])
    for o, z, st in others:
        assert torch.equal(st, status2) and torch.equal(z, sizes2)
        assert torch.equal(o[: int(offs[-1])], out2[: int(offs[-1])])
    return cb, packed.cpu().numpy(), poff.cpu().numpy(), out.cpu().numpy(), sizes.cpu().numpy(), status.cpu().numpy(), offs


def _check(cuda, bufs, block=MiB, htable=1024, magic=True):
    cb, pk, po, out, sizes, status, offs = _run(cuda, bufs, block, htable, magic)
    st = cb.status.cpu().numpy()
    for s, b in enumerate(bufs):
        assert st[s] == 0, f"stream {s}: compress status {st[s]}"
        want = orc.compress(block, htable, [b], append_magic=magic)
        got = pk[po[s] : po[s + 1]].tobytes()
        assert got == want, f"stream {s} (len {len(b)}): compressed bytes differ"
        assert status[s] == 0, f"stream {s}: decompress status {status[s]}"
        assert sizes[s] == len(b)
        assert out[offs[s] : offs[s + 1]].tobytes() == b


def test_log_batch_4k(cuda):
    from eazy_amd import synth

    d = synth.logs(3, 512 * 4096).tobytes()
    _check(cuda, [d[k * 4096 : (k + 1) * 4096] for k in range(512)])


def test_log_batch_64k(cuda):
    from eazy_amd import synth

    d = synth.logs(5, 8 * 65536).tobytes()
    _check(cuda, [d[k * 65536 : (k + 1) * 65536] for k in range(8)])


def test_ragged_and_edge_lengths(cuda):
    from eazy_amd import synth

    rng = np.random.default_rng(11)
    d = synth.logs(9, 1 << 20).tobytes()
    bufs = [b"", b"a", b"ab", b"abc", b"abcd", b"aaaaaaaaaaaa", bytes(64), bytes(7), bytes(9)]
    at = 0
    for n in rng.integers(0, 9000, 60):
        bufs.append(d[at : at + int(n)])
        at += int(n)
    _check(cuda, bufs)


def test_tiny_streams_at_batch_end(cuda):
    """The last streams start within the batch's final 16 bytes: K2r's header and literal loads
    are clamped to the batch's last 16 bytes (bytes past it read as 0), every decoder agrees."""
    from eazy_amd import synth

    d = synth.logs(13, 64 * 4096).tobytes()
    tail = [b"a", b"xyz", b"0123456789abcdef0", b"", b"q"]
    _check(cuda, [d[k * 4096 : (k + 1) * 4096] for k in range(64)] + tail)
    _check(cuda, [b"z"] + tail)


def test_many_streams_k1l_and_long_slots(cuda):
    """Batches past 256 streams: K1L (when forced) runs 4 streams per wave, up to 256
    one; and >= 12,288 streams with 64 KiB slots take the lane-per-stream decoder K2r by
    default (K2w below), both checked against the oracle and the exact decoder."""
    from eazy_amd import synth

    d = synth.logs(29, 1100 * 3000).tobytes()
    _check(cuda, [d[k * 3000 : (k + 1) * 3000] for k in range(1100)])
    # 12,288 streams, one of them 64 KiB: the slots hint (max_len) is >= 64 KiB
    small = synth.logs(31, 12287 * 64 + 65536).tobytes()
    bufs = [small[k * 64 : (k + 1) * 64] for k in range(12287)] + [small[12287 * 64 :]]
    _check(cuda, bufs)


def test_small_windows_and_tables(cuda):
    from eazy_amd import synth

    d = synth.logs(13, 1 << 16).tobytes()
    bufs = [d[k * 3000 : (k + 1) * 3000] for k in range(16)]
    for block, htable in ((32, 16), (128, 16), (512, 32), (1024, 512), (4096, 4), (1 << 16, 1 << 13)):
        _check(cuda, bufs, block, htable)


def test_no_magic(cuda):
    from eazy_amd import synth

    d = synth.logs(17, 1 << 16).tobytes()
    _check(cuda, [d[k * 4096 : (k + 1) * 4096] for k in range(16)], magic=False)


def test_random_and_runs(cuda):
    rng = np.random.default_rng(1)
    bufs = []
    for k in range(24):
        n = int(rng.integers(100, 20000))
        kind = k % 4
        if kind == 0:
            b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        elif kind == 1:
            b = rng.integers(0, 3, n, dtype=np.uint8).tobytes()
        elif kind == 2:
            b = (bytes(rng.integers(0, 256, 7, dtype=np.uint8)) * (n // 7 + 1))[:n]
        else:
            z = np.zeros(n, np.uint8)
            idx = rng.integers(0, n, n // 10)
            z[idx] = rng.integers(1, 256, len(idx), dtype=np.uint8)
            b = z.tobytes()
        bufs.append(b)
    _check(cuda, bufs)


def test_larger_than_window(cuda):
    """Writes longer than the window exercise ring-wrap and cut (A.10)."""
    rng = np.random.default_rng(2)
    bufs = []
    for block in (1024,):
        msg = bytearray(rng.integers(0x20, 0x78, 2 * block, dtype=np.uint8).tobytes())
        cp = b"0123456789abcdefgh"
        msg[: len(cp)] = cp
        msg[-len(cp) :] = cp
        bufs.append(bytes(msg))
        msg2 = bytearray(msg)
        msg2[len(msg2) - block + 3 : len(msg2) - block + 3 + len(cp)] = cp
        bufs.append(bytes(msg2))
        bufs.append((b"abcdefgh" * 600)[:4000] + bytes(rng.integers(0, 256, 3000, dtype=np.uint8)))
    _check(cuda, bufs, 1024, 512)
    _check(cuda, bufs, 1024, 32)


def test_split_kernel_selected(cuda, k1_kind):
    """The C1 shape runs K1s (parse + token writer) unless a test forces
    another kernel; K1s (T16 / T32) relies on same-address LDS stores / exchanges of
    one wave instruction applying in ascending lane order, which the library
    checks on the device (tools/mb_ldsatomic.hip shows the measurement) before
    choosing them."""
    import eazy_amd as ez

    want = {"": "s", "S": "s"}.get(k1_kind, k1_kind)
    assert ez.compress_kernel(MiB, 1024, 4096, 65536) == want
    assert ez.compress_kernel(MiB, 1 << 13, 4096, 65536) == "w"  # tables over 4096 entries: the general kernel
    # 2n > block: K1x's rounds, then the general kernel (forced 'w': the general kernel alone)
    assert ez.compress_kernel(MiB, 1024, 1 << 20, 4) == {"w": "w", "l": "l"}.get(k1_kind, "x")
    assert ez.compress_kernel(MiB, 1 << 13, 1 << 20, 4) == "w"


def _multi_write_check(cuda, streams, block=MiB, htable=1024):
    """streams: lists of Writes; the slot of each equals the oracle's sink bytes."""
    import torch

    import eazy_amd as ez

    data = b"".join(b"".join(ws) for ws in streams)
    in_off, w_idx, w_end = [0], [0], []
    pos = 0
    for ws in streams:
        for w in ws:
            pos += len(w)
            w_end.append(pos)
        in_off.append(pos)
        w_idx.append(len(w_end))
    t = lambda a: torch.tensor(a, dtype=torch.int64, device=cuda)
    host = np.frombuffer(data, np.uint8)
    dd = torch.from_numpy(host.copy()).to(cuda) if len(host) else torch.zeros(1, dtype=torch.uint8, device=cuda)
    cb = ez.compress_batch_writes(dd, t(in_off), t(w_idx), t(w_end), block, htable)
    torch.cuda.synchronize()
    st, sz, so = cb.status.cpu().numpy(), cb.sizes.cpu().numpy(), cb.slot_off.cpu().numpy()
    slots = cb.slots.cpu().numpy()
    for s, ws in enumerate(streams):
        assert st[s] == 0, (s, st[s])
        want = orc.compress(block, htable, ws)
        got = slots[so[s] : so[s] + sz[s]].tobytes()
        assert got == want, f"stream {s}: {len(ws)} Writes of {[len(w) for w in ws]}"


def test_multi_write_streams(cuda, k1_kind):
    """Streams that each receive several Writes (one NewWriter, k calls of
    Write, FlushThreshold 0): the slot holds the bytes the sink
    receives over the k calls, equal to the oracle's for the same Writes —
    ragged Writes, empty ones, ones shorter than a hash (4 bytes), one Write.
    K1s takes these (2 x length <= block); forced 'w' runs the general kernel."""
    if k1_kind == "S":
        pytest.skip("the u32-table K1s is covered by the automatic choice's long streams")
    from eazy_amd import synth

    rng = np.random.default_rng(21)
    d = synth.logs(23, 1 << 20).tobytes()
    streams, at = [], 0
    for s in range(96):
        k = int(rng.integers(1, 9))
        ws = []
        for _ in range(k):
            n = int(rng.choice([0, 1, 3, 4, 5, 17, int(rng.integers(0, 3000))]))
            ws.append(d[at : at + n])
            at += n
        streams.append(ws)
    _multi_write_check(cuda, streams)


def test_multi_write_streams_beyond_half_window(cuda, k1_kind):
    """Multi-Write streams longer than half the window run on the general kernel: the
    history of earlier Writes is read across Write boundaries, the ring wraps (block 4096 /
    32 KiB with Writes of up to 3 KiB / 40 KiB), far skips and the cut branch occur, and a
    1 MiB window with 3 x 400 KiB log Writes (writer.go:206-217, 280-296)."""
    if k1_kind:
        pytest.skip("one K1 choice suffices: these batches only fit the general kernel")
    import eazy_amd as ez
    from eazy_amd import synth

    assert ez.compress_kernel(4096, 64, 9000, 40) == "w"
    rng = np.random.default_rng(31)
    d = synth.logs(33, 4 << 20).tobytes()
    streams, at = [], 0
    for s in range(40):
        ws = []
        for _ in range(int(rng.integers(2, 6))):
            n = int(rng.integers(0, 3000))
            ws.append(d[at : at + n] if s % 3 else rng.integers(0, 4, n, dtype=np.uint8).tobytes())
            at += n
        streams.append(ws)
    _multi_write_check(cuda, streams, block=4096, htable=64)
    _multi_write_check(cuda, [[d[k * 40000 : (k + 1) * 40000] for k in range(j, j + 4)] for j in range(6)], block=1 << 15, htable=256)
    _multi_write_check(cuda, [[d[:409600], d[409600:819200], d[819200:1228800]], [d[2 << 20 :(2 << 20) + 700000], b"", d[:5000]]])


def test_sub_batches_through_offset_views(cuda):
    """offsets are absolute, so a run of whole streams [a, b) given
    as views (in_off[a:b+1], slot_off[a:b+1], sizes[a:b], status[a:b]) is a batch of
    its own.  Chunks compressed, packed and decompressed this way (ragged lengths, the
    chunk seams inside the input buffer) equal the one-batch result, byte for byte."""
    import torch

    import eazy_amd as ez
    from eazy_amd import synth

    rng = np.random.default_rng(23)
    lens = rng.integers(0, 6000, 300)
    lens[::37] = 0
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    host = synth.logs(21, int(offs[-1]))
    data = torch.from_numpy(host.copy()).to(cuda)
    off = torch.from_numpy(offs).to(cuda)
    mx = int(lens.max())
    cb = ez.compress_batch(data, off, MiB, 1024, max_len=mx)
    packed, poff = ez.pack(cb)
    want = packed[: int(poff[-1])].cpu()

    sub_cb = ez.CompressedBatch(torch.zeros_like(cb.slots), cb.slot_off, torch.empty_like(cb.sizes),
                                torch.empty_like(cb.status))
    out = torch.zeros(int(offs[-1]) + 16, dtype=torch.uint8, device=cuda)
    osz = torch.empty(len(lens), dtype=torch.int64, device=cuda)
    ost = torch.empty(len(lens), dtype=torch.int32, device=cuda)
    bounds = [0, 1, 77, 78, 200, 300]
    got = []
    for a, b in zip(bounds[:-1], bounds[1:]):
        sub = ez.CompressedBatch(sub_cb.slots, sub_cb.slot_off[a : b + 1], sub_cb.sizes[a:b], sub_cb.status[a:b])
        ez.compress_batch(data, off[a : b + 1], MiB, 1024, max_len=mx, out=sub)
        base = int(cb.slot_off[a])
        pk = torch.zeros(int(cb.slot_off[b]) - base + 16, dtype=torch.uint8, device=cuda)
        pk, po = ez.pack(sub, pk)
        got.append(pk[: int(po[-1])].cpu())
        ez.decompress_batch(pk, po, off[a : b + 1], out=out, sizes=osz[a:b], status=ost[a:b], max_len=mx)
    torch.cuda.synchronize()
    assert int(sub_cb.status.abs().sum()) == 0 and int(ost.abs().sum()) == 0
    assert torch.equal(sub_cb.sizes, cb.sizes)
    assert torch.equal(torch.cat(got), want), "chunked packing differs from the one-batch packing"
    assert torch.equal(osz.cpu(), torch.from_numpy(lens.astype(np.int64)))
    assert out[: int(offs[-1])].cpu().numpy().tobytes() == host.tobytes()


def test_batch_edge_streams(cuda, k1_kind):
    """Streams at the batch's edges (the lean parse copies a live stream that lacks 16 readable
    bytes before it or 64 after it inside the batch into a padded slot): many empty streams, then
    live ones starting at offset 0..12; tiny live streams ending in the last 64 bytes; a batch
    shorter than 16 bytes; single-stream batches."""
    from eazy_amd import synth

    d = synth.logs(29, 1 << 16).tobytes()
    head = [b""] * 37 + [d[:4], d[4:9], d[9:14], d[14:600]]
    tail = [d[600:4600]] + [d[4600 + 5 * k : 4605 + 5 * k] for k in range(14)] + [d[4700:4704]]
    _check(cuda, head + [d[5000:9000]] * 9 + tail)
    _check(cuda, [b"abcabcabcab"])
    _check(cuda, [d[:4096]])
    _check(cuda, [b"", d[:6000], b""])


def _planted(rng, n, events, block, zeros=False):
    """n random bytes with `events` copies planted: 6..40 bytes repeated from up to
    `block` + 64 bytes back (window matches, far skips, cuts), runs, and zero runs."""
    b = bytearray(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
    for p in np.sort(rng.integers(64, n - 64, events)):
        p = int(p)
        kind = int(rng.integers(0, 4 if zeros else 3))
        L = int(rng.integers(5, 40))
        if kind == 0:  # an earlier stretch
            d = int(rng.integers(1, min(p, block + 64)))
            for t in range(min(L, n - p)):
                b[p + t] = b[p - d + t]
        elif kind == 1:  # a short-period run
            per = int(rng.integers(1, 9))
            for t in range(per, min(L, n - p)):
                b[p + t] = b[p + t - per]
        elif kind == 2:  # the stream's first bytes again
            b[p : p + L] = b[:L]
        else:
            b[p : p + L] = bytes(L)
    return bytes(b)


def test_k1x_rounds(cuda, k1_kind):
    """K1x (ez_compress_spec.hip): fresh long streams whose emitting positions are judged all
    at once, one round per accepted position, the general kernel resolving each and taking
    the rest after 8 rounds.  Planted matches at every distance up to past the window, runs,
    zero runs, the stream's first bytes, fewer and more events than rounds, empty and tiny
    streams beside long ones; block 1 MiB / 4 KiB / 1 KiB, tables 16 .. 4096 entries."""
    if k1_kind == "S":
        pytest.skip("K1x's own shapes (automatic, K1x forced, and the general kernel alone with its LDS window)")
    from eazy_amd import synth

    rng = np.random.default_rng(41)
    f = synth.f32(43, 1 << 16).view(np.uint8).tobytes()
    bufs = [_planted(rng, 70000, e, MiB, zeros=e % 2 == 1) for e in (0, 1, 2, 5, 7, 8, 9, 20)]
    bufs += [f[: 1 << 18], (f[:100000] + bytes(300) + f[:70000]), b"", b"ab", b"abcde"]
    _check(cuda, bufs)
    small = [_planted(rng, 80000, e, 4096, zeros=True) for e in (3, 12, 40)]
    for block, htable in ((4096, 16), (4096, 4096), (1024, 256)):
        _check(cuda, small, block, htable)


def test_multi_device_batches_equal_one_device(cuda):
    """ez_compress_batch_multi / ez_decompress_batch_multi (host memory, contiguous whole-stream
    shards balanced by bytes, one host thread and HIP stream per device-list entry): the device
    list [0, 0] (two shards on the one card), [0, 0, 0] and [0] give the single-device batch's
    packing byte for byte (= the oracle's streams back to back) and the inputs back; ragged
    lengths with empty streams, and fewer streams than shards (an empty shard)."""
    import torch

    import eazy_amd as ez
    import oracle as orc
    from eazy_amd import synth

    rng = np.random.default_rng(41)
    lens = rng.integers(0, 9000, 301)
    lens[::17] = 0
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    host = synth.logs(43, int(offs[-1]))
    want = [orc.compress(MiB, 1024, [host[offs[s] : offs[s + 1]].tobytes()]) for s in range(len(lens))]
    want_packed = b"".join(want)
    want_off = np.concatenate([[0], np.cumsum([len(w) for w in want])]).astype(np.int64)
    # the single-device batch (device pointers, K1 + K3)
    cb = ez.compress_batch(torch.from_numpy(host).to(cuda), torch.from_numpy(offs).to(cuda), MiB, 1024)
    packed1, poff1 = ez.pack(cb)
    torch.cuda.synchronize()
    assert packed1[: int(poff1[-1])].cpu().numpy().tobytes() == want_packed
    for devs in ([0], [0, 0], [0, 0, 0], None):
        packed, poff, status = ez.compress_batch_multi(host, offs, MiB, 1024, devices=devs)
        assert (status == 0).all() and poff.tolist() == want_off.tolist(), devs
        assert packed.tobytes() == want_packed, devs
        out_off = offs + 0
        out, sizes, st = ez.decompress_batch_multi(packed, poff, out_off, devices=devs)
        assert (st == 0).all() and sizes.tolist() == lens.tolist(), devs
        assert out.tobytes() == host.tobytes(), devs
    # fewer streams than shards
    packed, poff, status = ez.compress_batch_multi(host[: offs[2]], offs[:3], MiB, 1024, devices=[0, 0, 0, 0])
    assert packed.tobytes() == b"".join(want[:2]) and (status == 0).all()
    # a slot one byte short: the stream's status is the decoder's, the others decode
    out_off = offs.copy()
    out_off[2:] -= 1
    if lens[1] > 0:
        out, sizes, st = ez.decompress_batch_multi(packed, poff, out_off[:3], devices=[0, 0])
        assert st[0] == 0 and st[1] != 0


@pytest.mark.gpu
def test_c1_full_batch_matches_oracle(cuda):
    """C1 at its full size (BASELINE.json configs[1]): 65,536 x 4 KiB synthetic log streams,
    NewWriter(MiB, 1024).Write(p) each (writer.go:133, :206). Every stream's bytes, packed, equal
    the C oracle's (oracle/eazy_oracle.c, 16 threads), and the automatic K2 decodes them all back on
    the device. The other tests in this file cover the edge shapes on a few hundred streams; this one
    runs the headline batch itself, through the same C-ABI calls bench.py times."""
    import torch

    import eazy_amd as ez
    from eazy_amd import synth

    n, S = 4096, 65536
    host = synth.logs(2025, n * S)
    offs = np.arange(S + 1, dtype=np.int64) * n
    cap = n + (n >> 2) + 64
    slot_off = np.arange(S + 1, dtype=np.int64) * cap
    slots, sizes = orc.compress_batch(MiB, 1024, host, offs, slot_off, 16)
    want = slots.reshape(S, cap)
    data = torch.from_numpy(host).to(cuda)
    off = torch.from_numpy(offs).to(cuda)
    cb = ez.compress_batch(data, off, MiB, 1024, append_magic=True)
    packed, poff = ez.pack(cb)
    torch.cuda.synchronize()
    assert int(cb.status.count_nonzero()) == 0
    po = poff.cpu().numpy()
    assert np.array_equal(np.diff(po), sizes), "compressed sizes differ from the oracle's"
    pk = packed[: int(po[-1])].cpu().numpy()
    # every stream's bytes: the packed stream s against the oracle's slot s
    keep = np.arange(cap)[None, :] < sizes[:, None]
    assert np.array_equal(pk, want[keep]), "compressed bytes differ from the oracle's"
    out, osz, ost = ez.decompress_batch(packed, poff, off, max_len=n)
    torch.cuda.synchronize()
    assert int(ost.count_nonzero()) == 0 and bool((osz == n).all())
    assert torch.equal(out[: n * S], data), "round trip differs"
