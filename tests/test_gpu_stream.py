"""The streaming drop-in (Writer / Reader handles over the C-ABI, compute on
the GPU) against the reference's own tests and the golden fixtures."""

import numpy as np
import pytest

import impls
import kat_suite as K
from golden_data import h, load

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def G(cuda):
    return impls.Gpu()


@pytest.mark.parametrize("t", K.ALL, ids=lambda f: f.__name__)
def test_reference_test(G, t):
    t(G)


def test_meta(G):
    import eazy_amd as ez

    K.t_meta(G, lambda m, l: ez.Encoder().meta(b"", m, l))


def test_sink_failure_resets(G):
    K.t_sink_failure_resets(G)


def _stream(G, block, ht, writes):
    w = G.W(block, ht)
    for p in writes:
        n, err = w.write(p)
        assert err == 0 and n == len(p)
    return w.sink


def test_golden_fuzz_writer(G):
    for e in load()["fuzz_writer"]:
        writes = [h(x) for x in e["writes"]]
        for block, ht in ((512, 32), (1 << 20, 1024)):
            assert _stream(G, block, ht, writes).hex() == e[f"stream_{block}_{ht}"], e["name"]
        r = G.Rb(h(e["stream_512_32"]))
        out = bytearray()
        while True:
            got, err = r.read(16)
            out += got
            if err == 1:
                break
            assert err == 0
        assert bytes(out) == b"".join(writes)


@pytest.mark.parametrize("buf", [16, 4096])
def test_golden_fuzz_reader(G, buf):
    for e in load()["fuzz_reader"]:
        r = G.Rs(h(e["input"]))
        out, errs = bytearray(), []
        while len(out) < (1 << 16):
            got, err = r.read(buf)
            out += got
            errs.append(err)
            if err not in (0, 10):
                break
        want = e[f"read{buf}"]
        assert errs == want["errs"], e["name"]
        assert bytes(out[: 1 << 16]).hex() == want["out"], e["name"]


def test_golden_multi_write(G):
    m = load()["multi_write"]
    writes = [h(x) for x in m["writes"]]
    assert _stream(G, 1 << 20, 1024, writes).hex() == m["stream_1048576_1024"]
    assert _stream(G, 2048, 64, writes).hex() == m["stream_2048_64"]
    r = G.Rb(h(m["stream_2048_64"]))
    got, err = r.read(1 << 20)
    assert err == 1 and got == b"".join(writes)


def test_golden_synthetic_batch(cuda):
    """K1/K2 batch path vs the fixtures (all three block/table configs)."""
    import torch

    import eazy_amd as ez

    syn = load()["synthetic_logs"]
    bufs = [h(e["input"]) for e in syn]
    offs = np.concatenate([[0], np.cumsum([len(b) for b in bufs])]).astype(np.int64)
    data = torch.from_numpy(np.frombuffer(b"".join(bufs), np.uint8).copy()).to(cuda)
    off = torch.from_numpy(offs).to(cuda)
    for block, ht in ((1 << 20, 1024), (1 << 17, 1024), (1024, 32)):
        cb = ez.compress_batch(data, off, block, ht)
        packed, poff = ez.pack(cb)
        torch.cuda.synchronize()
        pk, po = packed.cpu().numpy(), poff.cpu().numpy()
        for s, e in enumerate(syn):
            assert pk[po[s] : po[s + 1]].tobytes().hex() == e[f"stream_{block}_{ht}"]


def test_batch_decoder_errors_match_oracle(cuda):
    """K2 batch statuses on the FuzzReader corpus equal the oracle's
    NewReaderBytes + read-to-EOF result (bytes and first error)."""
    import torch

    import eazy_amd as ez
    import oracle as orc

    ins = [h(e["input"]) for e in load()["fuzz_reader"]]
    cap = 1 << 16
    offs = np.concatenate([[0], np.cumsum([len(b) for b in ins])]).astype(np.int64)
    comp = torch.from_numpy(np.frombuffer(b"".join(ins), np.uint8).copy()).to(cuda)
    coff = torch.from_numpy(offs).to(cuda)
    ooff = torch.arange(len(ins) + 1, dtype=torch.int64, device=cuda) * cap
    res = [ez.decompress_batch(comp, coff, ooff, exact_only=x) for x in (False, True)]
    torch.cuda.synchronize()
    for out, sizes, status in res:
        _cmp_oracle(ins, cap, out.cpu().numpy(), sizes.cpu().numpy(), status.cpu().numpy())
    # the ring decoder with a small-slot hint on the same corpus
    cap = 8192
    ooff = torch.arange(len(ins) + 1, dtype=torch.int64, device=cuda) * cap
    for kind in ("r", "w", "t"):
        ez.select_decompress_kernel(kind)
        try:
            out, sizes, status = ez.decompress_batch(comp, coff, ooff, max_len=cap)
            torch.cuda.synchronize()
        finally:
            ez.select_decompress_kernel("")
        _cmp_oracle(ins, cap, out.cpu().numpy(), sizes.cpu().numpy(), status.cpu().numpy())


def test_batch_decoders_on_damaged_streams(cuda):
    """Valid streams truncated, bit-flipped, padded, with breaks and with a
    second header (MetaReset mid-stream): the ring, wave and exact decoders
    all give the oracle's bytes and first error."""
    import torch

    import eazy_amd as ez
    import oracle as orc
    from eazy_amd import synth

    rng = np.random.default_rng(21)
    d = synth.logs(23, 48 * 4096).tobytes()
    good = [orc.compress(1 << 20, 1024, [d[k * 4096 : (k + 1) * 4096]]) for k in range(48)]
    ins = []
    for k, c in enumerate(good):
        c = bytearray(c)
        kind = k % 8
        if kind == 0:
            c = c[: int(rng.integers(1, len(c)))]
        elif kind == 1:
            for _ in range(3):
                c[int(rng.integers(0, len(c)))] ^= 1 << int(rng.integers(0, 8))
        elif kind == 2:
            at = int(rng.integers(9, len(c)))
            c = c[:at] + bytes(int(rng.integers(1, 20))) + c[at:]
        elif kind == 3:
            c = c + b"\x80\x1f" + bytes(3)
        elif kind == 4:
            c = c + good[(k + 1) % len(good)]
        elif kind == 5:
            c = c[:9] + b"\x80\x1f" + c[9:]
        elif kind == 6:
            c = c[:3] + c[9:]  # no magic meta: the reset meta alone
        ins.append(bytes(c))
    offs = np.concatenate([[0], np.cumsum([len(b) for b in ins])]).astype(np.int64)
    comp = torch.from_numpy(np.frombuffer(b"".join(ins), np.uint8).copy()).to(cuda)
    coff = torch.from_numpy(offs).to(cuda)
    for cap in (4096, 8192):
        ooff = torch.arange(len(ins) + 1, dtype=torch.int64, device=cuda) * cap
        for kind, kw in (("", {"max_len": cap}), ("r", {"max_len": cap}), ("w", {"max_len": cap}), ("t", {"max_len": cap}), ("", {}),
                         ("", {"exact_only": True})):
            ez.select_decompress_kernel(kind)
            try:
                out, sizes, status = ez.decompress_batch(comp, coff, ooff, **kw)
                torch.cuda.synchronize()
            finally:
                ez.select_decompress_kernel("")
            _cmp_oracle(ins, cap, out.cpu().numpy(), sizes.cpu().numpy(), status.cpu().numpy())


def _tag(t, n):
    """Encoder.Tag (writer.go:537-563) for lengths < 65916."""
    if n < 124:
        return bytes([t | n])
    if n < 380:
        return bytes([t | 0x7C, n - 124])
    return bytes([t | 0x7D]) + (n - 380).to_bytes(2, "little")


def _off(d, n):
    """Encoder.Offset (writer.go:565-597) for d >= n, d - n < 66044."""
    o = d - n
    if o < 252:
        return bytes([o])
    if o < 508:
        return bytes([0xFC, o - 252])
    return bytes([0xFD]) + (o - 508).to_bytes(2, "little")


def test_batch_decoders_ring_edge_distances(cuda):
    """Hand-built streams of short copies from 7.9-8.2 KiB back with short literals
    between them: next to the wave decoder's 8 KiB output ring (K2w), whose steps
    write ring slots close to the ones they read.  Every decoder gives the oracle's bytes."""
    import torch

    import eazy_amd as ez

    rng = np.random.default_rng(5)
    ins = []
    for lo, hi in ((7800, 8000), (8000, 8150), (8100, 8200), (8150, 8190), (8170, 8300), (100, 9000)):
        first = rng.integers(0, 256, 8400, dtype=np.uint8).tobytes()
        c = bytearray(b"\x80\x02eazy\x80\x10\x14" + _tag(0x00, len(first)) + first)
        n = len(first)
        while n < 70000:
            L = int(rng.integers(6, 40))
            c += _tag(0x80, L) + _off(int(rng.integers(lo, hi)), L)
            n += L
            k = int(rng.integers(1, 6))
            c += _tag(0x00, k) + rng.integers(0, 256, k, dtype=np.uint8).tobytes()
            n += k
        ins.append(bytes(c))
    offs = np.concatenate([[0], np.cumsum([len(b) for b in ins])]).astype(np.int64)
    comp = torch.from_numpy(np.frombuffer(b"".join(ins), np.uint8).copy()).to(cuda)
    coff = torch.from_numpy(offs).to(cuda)
    cap = 72 << 10
    ooff = torch.arange(len(ins) + 1, dtype=torch.int64, device=cuda) * cap
    for kind in ("", "w", "r", "t"):
        ez.select_decompress_kernel(kind)
        try:
            out, sizes, status = ez.decompress_batch(comp, coff, ooff, max_len=cap)
            torch.cuda.synchronize()
        finally:
            ez.select_decompress_kernel("")
        _cmp_oracle(ins, cap, out.cpu().numpy(), sizes.cpu().numpy(), status.cpu().numpy())


def _cmp_oracle(ins, cap, out, sizes, status):
    import eazy_amd as ez
    import oracle as orc

    for s, b in enumerate(ins):
        want, err, _ = orc.decompress(b, cap=cap)
        if err == 2:  # oracle output exceeded the capacity
            assert status[s] == ez.ENOSPC
            continue
        assert status[s] == err, s
        assert out[s * cap : s * cap + sizes[s]].tobytes() == want, s


def test_writer_cap_too_small_leaves_no_trace(cuda):
    """ez_writer_write with cap < ez_compress_bound(n) returns EZ_ENOSPC before
    anything reaches the device; retrying with room gives Go's bytes, and the
    next Write still matches (the handle's history was not touched)."""
    import ctypes as C

    import eazy_amd as ez
    import oracle as orc
    from eazy_amd import synth

    d = synth.logs(61, 3 * 4096).tobytes()
    p, q = d[:4096], d[4096:8192]
    L = ez._lib()
    h = C.c_void_p()
    assert L.ez_writer_new(1 << 20, 1024, 0, C.byref(h)) == 0
    try:
        n = C.c_size_t()
        small = (C.c_uint8 * 64)()
        assert L.ez_writer_write(h, p, len(p), small, 64, C.byref(n)) == ez.ENOSPC and n.value == 0
        outs = []
        for x in (p, q):
            cap = ez.compress_bound(len(x))
            buf = (C.c_uint8 * cap)()
            assert L.ez_writer_write(h, x, len(x), buf, cap, C.byref(n)) == 0
            outs.append(bytes(buf[: n.value]))
        assert b"".join(outs) == orc.compress(1 << 20, 1024, [p, q])
    finally:
        L.ez_writer_free(h)


def test_reader_large_stream_small_reads(cuda):
    """NewReaderBytes over a multi-MiB stream read 4 KiB (and 1000 B) at a time,
    the shape of io.Copy: the handle uploads input windows from r.i on, not the
    whole buffer per Read.  Includes a 200 KB literal (longer than the 64 KiB
    input window) and a NewReader (io.Reader refill) over the same bytes."""
    import io
    import time

    import eazy_amd as ez
    import oracle as orc
    from eazy_amd import synth

    rng = np.random.default_rng(3)
    plain = synth.logs(67, 3 << 20).tobytes() + rng.integers(0, 256, 200_000, dtype=np.uint8).tobytes() + \
        synth.logs(68, 1 << 20).tobytes()
    comp = orc.compress(1 << 20, 1024, [plain[k : k + 65536] for k in range(0, len(plain), 65536)])
    for size in (4096, 1000):
        r = ez.NewReaderBytes(comp)
        out = bytearray()
        t0 = time.perf_counter()
        while True:
            got, err = r.Read(size)
            out += got
            if err == ez.EOF:
                break
            assert err == ez.OK, err
        dt = time.perf_counter() - t0
        assert bytes(out) == plain, size
        print(f"Read({size}) loop over {len(comp)} compressed bytes: {dt * 1e3:.0f} ms")
    r = ez.NewReader(io.BytesIO(comp))
    out = bytearray()
    while True:
        got, err = r.Read(4096)
        out += got
        if err == ez.EOF:
            break
        assert err == ez.OK, err
    assert bytes(out) == plain


def test_writer_positions_past_4gib(cuda):
    """A Writer whose position crosses 2^32 (the table holds uint32(start + i),
    writer.go:216-217, so entries written past 2^32 look far away and are skipped): the handle's
    bytes equal the oracle's from the same state (testing hook on both: w.pos set, zero ring
    and table)."""
    import ctypes as C

    import eazy_amd as ez
    import oracle as orc
    from eazy_amd import synth

    d = synth.logs(71, 16 * 4096).tobytes()
    writes = [d[k * 4096 : (k + 1) * 4096] for k in range(16)]
    for p0 in ((1 << 32) - 10000, (1 << 32) - 1, (1 << 33) + 5):
        ow = orc.Writer(1 << 20, 1024)
        ow.set_pos(p0)
        for w in writes:
            ow.write(w)
        L = ez._lib()
        L.ez_writer_set_position.argtypes = [C.c_void_p, C.c_int64]
        h = C.c_void_p()
        assert L.ez_writer_new(1 << 20, 1024, 0, C.byref(h)) == 0
        try:
            assert L.ez_writer_set_position(h, p0) == 0
            outs, n = [], C.c_size_t()
            for w in writes:
                cap = ez.compress_bound(len(w))
                buf = (C.c_uint8 * cap)()
                assert L.ez_writer_write(h, w, len(w), buf, cap, C.byref(n)) == 0
                outs.append(bytes(buf[: n.value]))
        finally:
            L.ez_writer_free(h)
        assert b"".join(outs) == ow.sink, f"p0 = {p0:#x}"


class _Sink:
    """io.Writer recording every call; optionally one short write (the n-th call takes half)."""

    def __init__(self, short_at=None):
        self.calls, self.short_at = [], short_at

    def write(self, b):
        self.calls.append(bytes(b))
        return len(b) // 2 if len(self.calls) == self.short_at else len(b)


@pytest.mark.parametrize("block,ht,thr", [(1 << 20, 1024, 0), (1 << 20, 1024, 700), (4096, 64, -1), (1024, 32, 300), (2048, 16, 0)])
def test_write_batch_equals_writes(cuda, block, ht, thr):
    """Writer.WriteBatch (ez_writer_write_batch: k Writes in one launch on the handle's ring and
    table, the general kernel's multi-Write path with the ring as older history) gives the sink
    exactly the calls Write on each in turn gives it: ragged log Writes (empty, sub-hash, up to
    3 KiB) in batches of 1..40, windows of 1 KiB .. 1 MiB (the ring wraps inside a batch), every
    FlushThreshold regime; the stream equals the oracle's for the same Writes."""
    import eazy_amd as ez
    from eazy_amd import synth
    import oracle as orc

    rng = np.random.default_rng(block + ht + thr)
    d = synth.logs(71, 1 << 20).tobytes()
    writes, at = [], 0
    for _ in range(400):
        n = int(rng.choice([0, 1, 3, 4, 9, int(rng.integers(0, 400)), int(rng.integers(0, 3000))]))
        writes.append(d[at : at + n])
        at += n
    sinks = []
    for batched in (False, True):
        s = _Sink()
        w = ez.Writer(s, block, ht)
        w.FlushThreshold = thr
        j = 0
        while j < len(writes):
            k = int(rng.integers(1, 41)) if batched else 1
            if batched:
                assert w.WriteBatch(writes[j : j + k]) == sum(len(x) for x in writes[j : j + k])
            else:
                assert w.Write(writes[j]) == len(writes[j])
            j += k
        w.Flush()
        sinks.append(s.calls)
    assert sinks[1] == sinks[0]
    assert b"".join(sinks[1]) == orc.compress(block, ht, writes)


def test_write_batch_short_sink_write(cuda):
    """A short sink write inside a batch restarts the stream (writer.go:387-401); the Writes after
    it go to the new stream, as with Write one at a time."""
    import eazy_amd as ez
    from eazy_amd import synth

    d = synth.logs(73, 1 << 16).tobytes()
    writes = [d[k * 300 : (k + 1) * 300] for k in range(60)]
    calls = []
    for batched in (False, True):
        s = _Sink(short_at=5)
        w = ez.Writer(s, 1 << 20, 1024)
        if batched:
            w.WriteBatch(writes[:30])
            w.WriteBatch(writes[30:])
        else:
            for p in writes:
                w.Write(p)
        calls.append(s.calls)
    assert calls[1] == calls[0]


@pytest.mark.parametrize("block,ht", [(1 << 20, 1024), (4096, 4096), (65536, 256), (1024, 16)])
def test_handle_writes_k1l_and_general(cuda, block, ht):
    """Writer.Write on a handle takes K1L on the handle's ring and table (the Write and the ring's
    last 16 KiB staged in LDS up to 48 KiB Writes, global reads past that); the general kernel
    forced gives the same stream.  Writes of 20 B .. 200 KiB of logs and random bytes with planted
    repeats, windows of 1 KiB .. 1 MiB (far skips, the ring wrapping inside a Write, Writes longer
    than the window); the sink equals the oracle's for the same Writes."""
    import eazy_amd as ez
    import oracle as orc
    from eazy_amd import synth

    rng = np.random.default_rng(block + ht)
    d = synth.logs(77, 1 << 20).tobytes()
    r = rng.integers(0, 256, 1 << 18, dtype=np.uint8).tobytes()
    writes = [d[:20], d[20:5000], r[:60000], d[5000:205000], r[:3000] + d[:3000], d[205000:205100], r[1000:71000],
              d[:50000], d[300000:301000]]
    outs = []
    for kind in ("", "w"):
        ez.select_compress_kernel(kind)
        try:
            s = _Sink()
            w = ez.Writer(s, block, ht)
            for p in writes:
                assert w.Write(p) == len(p)
            w.Flush()
            outs.append(b"".join(s.calls))
        finally:
            ez.select_compress_kernel("")
    want = orc.compress(block, ht, writes)
    assert outs[0] == want, "K1L handle path"
    assert outs[1] == want, "general kernel"


def test_fast_decoders_checks_and_forms(cuda):
    """The fast decoders (K2r, K2t, K2w) on hand-built small streams: every check they make
    hands the stream to the exact decoder with the reference's result —
    slots one byte too small, BlockSizeLimit below a token's length, a copy farther than the
    window (MetaReset with a 32-byte block), a token before the window is set, a reset after
    output — and the long forms it parses itself (Len1/Len2 literals and copies, Off1/Off2/
    OffLong offsets, zero regions, short-period runs, copies reaching before the stream start).
    Statuses, sizes and bytes equal the oracle's for every slot size and limit."""
    import torch

    import eazy_amd as ez
    import oracle as orc

    rng = np.random.default_rng(11)
    hdr = b"\x80\x02eazy\x80\x10\x14"  # magic, reset to a 1 MiB block (reader.go continueMetaTag)

    def lit(b):
        return _tag(0x00, len(b)) + b

    def cpy(d, n, lng=False):  # a distance below the length (a run) takes the OffLong form, as Encoder.Offset
        return _tag(0x80, n) + (b"\xff" + _off(d, 0) if lng or d < n else _off(d, n))

    good = []
    # long forms: Len1 / Len2 literals, Len1 copies, Off1 / Off2 offsets, OffLong, zero region, runs
    a = rng.integers(0, 256, 300, dtype=np.uint8).tobytes()
    good.append(hdr + lit(a) + cpy(300, 200) + cpy(250, 130) + lit(b"x") + cpy(1, 40) + cpy(3, 33) + cpy(0, 100))
    b = rng.integers(97, 100, 700, dtype=np.uint8).tobytes()
    good.append(hdr + lit(b) + cpy(600, 500, lng=True) + cpy(509, 60) + cpy(253, 7) + lit(b"tail"))
    good.append(hdr + cpy(0, 64) + cpy(2000, 30) + lit(b"abc") + cpy(5, 9))  # zero history before the start
    good.append(hdr + b"\x00\x00\x00" + lit(b"pad") + b"\x00" + b"\x80\x1f" + cpy(3, 12))  # padding and a break
    bad = [
        b"\x80\x02eazy\x80\x10\x05" + lit(rng.integers(0, 256, 40, dtype=np.uint8).tobytes()) + cpy(36, 8),  # D > 32-byte window
        lit(b"no reset first") + hdr,  # a token before the window is set
        hdr + lit(b"abcdef") + b"\x80\x10\x14" + cpy(3, 4),  # a reset after output
    ]
    ins = good + bad
    lens = [len(orc.decompress(x, cap=1 << 20)[0]) for x in ins]
    offs = np.concatenate([[0], np.cumsum([len(x) for x in ins])]).astype(np.int64)
    comp = torch.from_numpy(np.frombuffer(b"".join(ins) + bytes(64), np.uint8).copy()).to(cuda)
    coff = torch.from_numpy(offs).to(cuda)
    for cap, limit in ((4096, 0), (max(lens), 0), (max(lens) - 1, 0), (4096, 64), (4096, 250)):
        ooff = torch.arange(len(ins) + 1, dtype=torch.int64, device=cuda) * cap
        res = {}
        for kind in ("r", "t", "w", ""):
            ez.select_decompress_kernel(kind)
            try:
                res[kind] = ez.decompress_batch(comp, coff, ooff, block_size_limit=limit, max_len=cap)
                torch.cuda.synchronize()
            finally:
                ez.select_decompress_kernel("")
        ex = ez.decompress_batch(comp, coff, ooff, block_size_limit=limit, exact_only=True)
        torch.cuda.synchronize()
        for kind, (out, sizes, status) in res.items():
            assert torch.equal(status, ex[2]) and torch.equal(sizes, ex[1]), (kind, cap, limit)
            for s in range(len(ins)):
                n = int(sizes[s])
                assert torch.equal(out[s * cap : s * cap + n], ex[0][s * cap : s * cap + n]), (kind, cap, limit, s)
        if limit == 0:
            for kind in ("r", "t"):
                _cmp_oracle(ins, cap, res[kind][0].cpu().numpy(), res[kind][1].cpu().numpy(), res[kind][2].cpu().numpy())


def test_reader_whole_decode_matches_read_by_read(cuda):
    """NewReaderBytes decodes the whole stream on its first Read (ez_reader_set_whole) and serves
    the Reads from it; with set_whole(0) (NewReader's mode) it decodes Read by Read.  Same bytes and the
    same error sequence for a multi-block stream (Reset metas at every 1 MiB block), a stream with a
    version header, streams with Break metas (in the middle, several back to back, at the very start and
    at the end: the Reads stop at each with ErrBreak, from the decoders' recorded break positions), a
    stream that expands more than 20x (the device slot grows past 8x the input), a truncated stream and
    one ending in an unsupported meta (both decline: the exact decoder's error)."""
    import eazy_amd as ez
    import impls
    from eazy_amd import synth

    G = impls.Gpu()
    plain = synth.logs(91, 3 << 20).tobytes()
    chunks = [plain[k : k + 200_000] for k in range(0, len(plain), 200_000)]

    def stream(brk=(), hdr=False, data=chunks):
        w = G.W(1 << 20, 1024)
        if hdr:
            w.append_magic = True
            assert w.write_header() == ez.OK
        for k, c in enumerate(data):
            for _ in range(brk.count(k)):
                assert w.write_break() == ez.OK
            assert w.write(c) == (len(c), ez.OK)
        for _ in range(brk.count(len(data))):
            assert w.write_break() == ez.OK
        return w.sink

    def read_all(r, size):
        out, errs = bytearray(), []
        for _ in range(100000):
            got, err = r.read(size)
            out += got
            errs.append(err)
            if err not in (ez.OK, ez.EBREAK):
                break
        return bytes(out), errs

    clean = stream()
    # 16 MiB of zero runs with a few other bytes: > 20x expansion (about 50,000x)
    dense_parts = [bytes(1 << 19) + bytes([k + 1]) * 64 for k in range(32)]
    dense = stream(data=dense_parts)
    assert len(b"".join(dense_parts)) > 20 * len(dense)
    cases = {"clean": (clean, True, plain, 0), "header": (stream(hdr=True), True, plain, 0),
             "break": (stream(brk=(len(chunks) // 2,)), True, plain, 1),
             "breaks": (stream(brk=(0, 3, 3, 3, 7, len(chunks))), True, plain, 6),
             "dense": (dense, True, b"".join(dense_parts), 0),
             "truncated": (clean[: len(clean) - 7], False, None, 0)}
    cases["unsupported_meta"] = (clean + bytes([K.Meta, 0x40 | K.MetaLen0]), False, None, 0)
    for name, (comp, ahead, want_plain, nbrk) in cases.items():
        for size in (4096, 200_000, 1 << 20):
            rb = G.Rb(comp)
            got, errs = read_all(rb, size)
            assert rb.r.whole_decoded == ahead, (name, size)
            rx = G.Rb(comp)
            ez._lib().ez_reader_set_whole(rx.r._h, 0)  # the same handle decoding Read by Read
            want, werrs = read_all(rx, size)
            assert not rx.r.whole_decoded
            assert errs == werrs, (name, size, errs[-3:], werrs[-3:])
            assert got == want, (name, size)
            if want_plain is not None:
                assert got == want_plain and errs[-1] == ez.EOF, name
            assert errs.count(ez.EBREAK) == nbrk, (name, size)


def test_reader_whole_decode_then_more_input(cuda):
    """A Reader set after NewReaderBytes (reader.go:27: a public field) supplies input after the
    decoded stream: the handle goes on Read by Read from the Reader's state at the stream's end
    (window size, position, the window's history), so copies in the new input that reach back into
    the first part decode exactly as on a handle that decoded everything Read by Read."""
    import eazy_amd as ez
    import impls
    from eazy_amd import synth

    G = impls.Gpu()
    plain = synth.logs(93, 1 << 20).tobytes()
    w = G.W(1 << 16, 1024)
    assert w.write(plain[: 600_000]) == (600_000, ez.OK)
    first = bytes(w.sink)
    assert w.write(plain[600_000:]) == (len(plain) - 600_000, ez.OK)
    second = bytes(w.sink)[len(first) :]
    results = []
    for whole in (1, 0):
        rb = G.Rb(first)
        ez._lib().ez_reader_set_whole(rb.r._h, whole)
        out, errs = bytearray(), []
        for k in range(10000):
            if k == 40:  # part-way through the first part: the rest comes from an io.Reader
                rb.r.Reader = impls._Src(second, True)
                rb.r.BufferSize = 64 << 10
            got, err = rb.read(8192)
            out += got
            errs.append(err)
            if err not in (ez.OK, ez.EBREAK):
                break
        results.append((bytes(out), errs, rb.r.whole_decoded))
    (a, ea, _), (b, eb, _) = results
    assert a == b == plain and ea == eb and ea[-1] == ez.EOF


def test_reader_whole_decode_reset(cuda):
    import eazy_amd as ez
    import impls
    from eazy_amd import synth

    G = impls.Gpu()
    plain = synth.logs(91, 3 << 20).tobytes()
    w = G.W(1 << 20, 1024)
    for k in range(0, len(plain), 200_000):
        assert w.write(plain[k : k + 200_000])[1] == ez.OK
    clean = w.sink

    def read_all(r, size):
        out = bytearray()
        for _ in range(100000):
            got, err = r.read(size)
            out += got
            if err not in (ez.OK, ez.EBREAK):
                break
        return bytes(out), err

    # ResetBytes starts a new whole decode; Reset(io.Reader) goes back to Read by Read
    rb = G.Rb(clean)
    assert rb.read(10)[0] == plain[:10] and rb.r.whole_decoded
    rb.reset_bytes(clean)
    assert not rb.r.whole_decoded
    assert rb.read(1 << 22)[0] == plain and rb.r.whole_decoded
    rb.reset(clean)
    rb.set(16 << 20, 64 << 10)  # (a NewReaderBytes Reader keeps BufferSize 0: Go's more() would read nothing)
    assert read_all(rb, 1 << 16)[0] == plain and not rb.r.whole_decoded
