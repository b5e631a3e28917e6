"""GPU parity at the BASELINE configurations other than C1 (SURVEY.md §8, configs
C2 and C4), and the long token forms, through the C-ABI (include/eazy.h).

* C2 — 256 KiB log Writes into NewWriter(MiB, 1024): K1s-T32 (the automatic
  choice at this shape) and the general K1 forced.
* C4 — gradient buckets bit-cast to bytes: fp32 N(0, 1e-3), bf16 (its top
  halves), 90 %-zero sparse fp32 (writeZeros, writer.go:407-439), at 256 KiB,
  1 MiB, 4 MiB and 16 MiB: Writes longer than the window (ring wrap and the cut
  branch) on K1x's rounds (the automatic choice) and on the
  general K1 alone.
* Len4 literals and Off4 offsets (writer.go:537-597; Decoder reader.go:346-514)
  from hand-built inputs; the CPU test below checks on the oracle that each
  input really produces the form it is meant to, so the GPU test cannot pass
  vacuously.

Bar: every stream's compressed bytes equal the oracle's, byte for byte, and
every K2 decoder (ring, wave, exact) returns the input."""

import numpy as np
import pytest

import oracle as orc

MiB = 1 << 20


def tokens(b: bytes):
    """Token walk of a compressed stream with the oracle's decoders:
    [(kind, length, tag bytes, offset bytes, offset field hex)]."""
    i, out = 0, []
    while i < len(b):
        if b[i] == 0:
            i += 1
            continue
        t, l, i2, e = orc.dec_tag(b, i)
        assert e == 0, (e, i)
        if t == 0x80 and l == 0:
            _, ml, i3, e = orc.dec_meta(b, i2)
            assert e == 0
            i = i3 + ml
            continue
        if t == 0:
            out.append(("l", l, i2 - i, 0, ""))
            i = i2 + l
        else:
            _, i3, e = orc.dec_offset(b, i2, l)
            assert e == 0
            out.append(("c", l, i2 - i, i3 - i2, b[i2:i3].hex()))
            i = i3
    return out


def long_form_inputs():
    """(name, bytes, htable, predicate on the oracle's tokens)."""
    rng = np.random.default_rng(5)
    r = rng.integers(0, 256, 64, dtype=np.uint8).tobytes()
    x = rng.integers(0, 256, 70000, dtype=np.uint8).tobytes()
    return [
        # a literal of >= 65,916 bytes: Len4 tag (writer.go:555-560)
        ("len4_literal", x, 1024, lambda t: any(k[0] == "l" and k[1] >= 65916 and k[2] == 5 for k in t)),
        # a window copy at distance >= 66,044 + l: Off4 (writer.go:590-595)
        ("off4_window", r + bytes(70000) + r, 1024,
         lambda t: any(k[0] == "c" and k[3] == 5 and k[4].startswith("fe") for k in t)),
        # a run-length copy longer than its distance >= 66,044: OffLong + Off4 (writer.go:568-572)
        ("offlong_off4_run", x + x + x[:5000], 16384,
         lambda t: any(k[0] == "c" and k[3] == 6 and k[4].startswith("fffe") for k in t)),
        # a copy longer than 65,916: Len4 copy tag
        ("len4_copy", x + x + x[:5000], 16384, lambda t: any(k[0] == "c" and k[1] >= 65916 and k[2] == 5 for k in t)),
    ]


def gradient_buckets():
    """C4 buckets: fp32 N(0,1e-3), bf16 halves, 90 % zeros; 256 KiB .. 16 MiB."""
    from eazy_amd import synth

    f = synth.f32(41, (16 * MiB) // 4)
    bf = (synth.f32(43, (4 * MiB) // 2).view(np.uint32) >> 16).astype(np.uint16)
    sp = synth.f32(47, (4 * MiB) // 4)
    sp[np.random.default_rng(47).random(sp.shape[0]) < 0.9] = 0.0
    fb = f.view(np.uint8).tobytes()
    return [fb[: 256 << 10], fb[: 1 * MiB], fb[: 4 * MiB], bf.view(np.uint8).tobytes(), sp.view(np.uint8).tobytes(), fb]


def test_long_form_inputs_produce_their_forms():
    """CPU: each hand-built input drives the oracle into the token form it names."""
    for name, b, ht, pred in long_form_inputs():
        t = tokens(orc.compress(MiB, ht, [b]))
        assert pred(t), f"{name}: the oracle's stream does not contain the form ({t[:4]})"


def _gpu_check(cuda, bufs, htable=1024, kinds=("",)):
    """Compress on the GPU (K1 kinds as given), byte-compare every stream with
    the oracle (multi-threaded C oracle), decode with every K2 decoder."""
    import eazy_amd as ez
    from test_gpu_batch import _run

    lens = np.array([len(b) for b in bufs], np.int64)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    host = np.frombuffer(b"".join(bufs), np.uint8).copy()
    cap = lens + (lens >> 2) + 64
    slot_off = np.concatenate([[0], np.cumsum(cap)]).astype(np.int64)
    slots, sizes = orc.compress_batch(MiB, htable, host, offs, slot_off, 8)
    want = [slots[slot_off[s] : slot_off[s] + sizes[s]].tobytes() for s in range(len(bufs))]
    for kind in kinds:
        ez.select_compress_kernel(kind)
        try:
            cb, pk, po, out, osz, ost, _ = _run(cuda, bufs, MiB, htable)
        finally:
            ez.select_compress_kernel("")
        st = cb.status.cpu().numpy()
        for s, b in enumerate(bufs):
            assert st[s] == 0, f"K1 {kind!r} stream {s}: compress status {st[s]}"
            assert pk[po[s] : po[s + 1]].tobytes() == want[s], f"K1 {kind!r} stream {s} (len {len(b)}): bytes differ"
            assert ost[s] == 0 and osz[s] == len(b), f"stream {s}: decompress status {ost[s]} size {osz[s]}"
            assert out[offs[s] : offs[s + 1]].tobytes() == b, f"stream {s}: round trip differs"
    return want


@pytest.mark.gpu
def test_c2_log_writes_256k(cuda):
    """C2 shape: 32 x 256 KiB log Writes, block 1 MiB, htable 1024 — K1s (T32)
    and the general K1 forced; K2w is the automatic decoder at this slot size."""
    import eazy_amd as ez
    from eazy_amd import synth

    assert ez.compress_kernel(MiB, 1024, 256 << 10, 4096) == "s"
    d = synth.logs(31, 32 * (256 << 10)).tobytes()
    _gpu_check(cuda, [d[k << 18 : (k + 1) << 18] for k in range(32)], kinds=("", "w"))


@pytest.mark.gpu
def test_c4_gradient_buckets(cuda):
    """C4 shape: fp32 / bf16 / sparse buckets of 256 KiB .. 16 MiB (Writes up to
    16x the window: ring wrap, cut, writeZeros, Len4 literals)."""
    import eazy_amd as ez

    assert ez.compress_kernel(MiB, 1024, 4 * MiB, 64) == "x"
    bufs = gradient_buckets()
    want = _gpu_check(cuda, bufs, kinds=("", "w"))
    t16 = tokens(want[-1])
    assert any(k[0] == "l" and k[2] == 5 for k in t16), "the 16 MiB fp32 bucket should carry Len4 literals"
    assert any(k[0] == "c" and k[4] == "ff00" for k in tokens(want[4])), "the sparse bucket should carry zero runs"


@pytest.mark.gpu
def test_long_token_forms(cuda):
    """Len4 literals / copies, Off4 and OffLong+Off4 offsets, byte-checked on the device."""
    for name, b, ht, _ in long_form_inputs():
        _gpu_check(cuda, [b, b[:4096], b], htable=ht)


@pytest.mark.gpu
def test_k2w_deferred_literals(cuda):
    """K2w defers literals of 16 KiB and more to a chip-wide copy (kd_copy) after giving its ring
    their last 8 KiB: copies that read back into such a literal from beyond the ring (distances
    16 KiB+), one to six long literals per stream (a stream defers up to 8; the rest are
    moved inline), long literals right after short tokens and at the stream's end."""
    rng = np.random.default_rng(61)
    R = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in (20000, 17000, 40000, 16384, 70000, 30001)]
    logs = __import__("eazy_amd.synth", fromlist=["logs"]).logs(63, 200000).tobytes()
    bufs = [
        R[0] + R[0][:3000] + R[0][100:700],                       # copies into the deferred literal
        logs[:5000] + R[1] + logs[:5000] + R[1][5:900] + R[2],     # log tokens around two long literals
        b"".join(R) + R[0][:64] + R[4][1000:1200] + R[5][7:99],    # six long literals, copies into several
        R[3],                                                      # exactly 16 KiB, the whole stream
        logs[:70000],                                              # no long literal
        b"".join(R + R[:4]) + R[2][:500],                           # ten long literals: eight deferred
    ]
    _gpu_check(cuda, bufs)


@pytest.mark.gpu
def test_c2_production_routing_k1l_four_per_wave(cuda):
    """C2's production route: more than 256 fresh 256 KiB log streams go from K1s to K1L
    at 4 streams per wave (u32 tables, trims, ring image); 260 streams, automatic choice,
    every stream byte-compared with the oracle and decoded by every K2 decoder."""
    import eazy_amd as ez
    from eazy_amd import synth

    assert ez.compress_kernel(MiB, 1024, 256 << 10, 260) == "s"
    d = synth.logs(37, 260 * (256 << 10)).tobytes()
    _gpu_check(cuda, [d[k << 18 : (k + 1) << 18] for k in range(260)])


@pytest.mark.gpu
def test_k2w_literal_longer_than_the_hint(cuda):
    """K2w defers literals of 16 KiB and more to kd_copy; the decode's max_len hint (64 KiB
    here) must not bound how much of a 256 KiB literal gets copied."""
    import torch

    import eazy_amd as ez

    rng = np.random.default_rng(67)
    bufs = [rng.integers(0, 256, 256 << 10, dtype=np.uint8).tobytes(), bytes(1000) + rng.integers(0, 256, 200000, dtype=np.uint8).tobytes()]
    want = [orc.compress(MiB, 1024, [b]) for b in bufs]
    dev = cuda
    comp = torch.from_numpy(np.frombuffer(b"".join(want) + bytes(64), np.uint8).copy()).to(dev)
    coff = torch.tensor([0, len(want[0]), len(want[0]) + len(want[1])], dtype=torch.int64, device=dev)
    ooff = torch.tensor([0, len(bufs[0]), len(bufs[0]) + len(bufs[1])], dtype=torch.int64, device=dev)
    for kind in ("w", "t", "j"):
        ez.select_decompress_kernel(kind)
        try:
            out, sz, st = ez.decompress_batch(comp, coff, ooff, max_len=64 << 10)
        finally:
            ez.select_decompress_kernel("")
        assert st.cpu().tolist() == [0, 0] and sz.cpu().tolist() == [len(b) for b in bufs], kind
        assert out[: len(bufs[0]) + len(bufs[1])].cpu().numpy().tobytes() == b"".join(bufs), kind


@pytest.mark.gpu
def test_k1x_refused_stream_leaves_others_exact(cuda):
    """A stream longer than the caller's max_len is refused (EINVAL); K1x's per-position
    scratch is indexed per stream, so the refused stream cannot shift or overwrite the
    others' tables: they stay oracle-exact."""
    import torch

    import eazy_amd as ez
    from eazy_amd import synth

    d = synth.logs(41, 700 << 10).tobytes()
    bufs = [d[: 300 << 10]] + [d[(300 + 100 * k) << 10 : (400 + 100 * k) << 10] for k in range(4)]
    lens = np.array([len(b) for b in bufs], np.int64)
    offs = torch.from_numpy(np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)).to(cuda)
    data = torch.from_numpy(np.frombuffer(b"".join(bufs), np.uint8).copy()).to(cuda)
    for kind in ("x", ""):
        ez.select_compress_kernel(kind)
        try:
            cb = ez.compress_batch(data, offs, MiB, 1024, max_len=128 << 10)
        finally:
            ez.select_compress_kernel("")
        st = cb.status.cpu().tolist()
        assert st[0] == ez.EINVAL and st[1:] == [0, 0, 0, 0], (kind, st)
        so, sz = cb.slot_off.cpu().numpy(), cb.sizes.cpu().numpy()
        slots = cb.slots.cpu().numpy()
        for s in range(1, 5):
            got = slots[so[s] : so[s] + sz[s]].tobytes()
            assert got == orc.compress(MiB, 1024, [bufs[s]]), f"K1 {kind!r} stream {s}: bytes differ"


@pytest.mark.gpu
def test_k2t_four_kib_ring_on_long_streams(cuda):
    """K2t takes its 4 KiB ring when that keeps every stream's wave resident at once and the
    8 KiB one would not (3,072 resident waves with 8 KiB rings on 256 CUs): 3,300 streams of
    5 - 24 KiB, so copies reach past the ring into output already in HBM and random streams of
    16 KiB and more defer their one long literal — 't' forced, every stream compared with its
    input."""
    import torch

    import eazy_amd as ez
    from eazy_amd import synth

    rng = np.random.default_rng(71)
    count = 3300
    lens = rng.integers(5000, 24577, count)
    logs = synth.logs(73, int(lens.sum())).tobytes()
    bufs, at = [], 0
    for k, n in enumerate(lens):
        if k % 97 == 0:
            bufs.append(rng.integers(0, 256, int(n), dtype=np.uint8).tobytes())
        else:
            bufs.append(logs[at : at + n])
            at += n
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    cap = lens + (lens >> 2) + 64
    slot_off = np.concatenate([[0], np.cumsum(cap)]).astype(np.int64)
    slots, sizes = orc.compress_batch(MiB, 1024, np.frombuffer(b"".join(bufs), np.uint8).copy(), offs, slot_off, 8)
    comp = b"".join(slots[slot_off[s] : slot_off[s] + sizes[s]].tobytes() for s in range(count))
    coff = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    d_comp = torch.from_numpy(np.frombuffer(comp + bytes(64), np.uint8).copy()).to(cuda)
    ez.select_decompress_kernel("t")
    try:
        out, sz, st = ez.decompress_batch(d_comp, torch.from_numpy(coff).to(cuda), torch.from_numpy(offs).to(cuda),
                                          max_len=int(lens.max()))
    finally:
        ez.select_decompress_kernel("")
    assert st.cpu().abs().sum().item() == 0 and sz.cpu().numpy().tolist() == lens.tolist()
    got = out[: int(offs[-1])].cpu().numpy().tobytes()
    for s in range(count):
        assert got[offs[s] : offs[s + 1]] == bufs[s], f"stream {s} (len {lens[s]}) differs"


@pytest.mark.gpu
def test_exactly_64k_streams_on_u16_tables(cuda):
    """Streams of exactly 64 KiB take K1s with u16 tables (visited positions < n - 3 fit 16 bits):
    logs, random bytes, a sparse stream and a run, byte-compared with the oracle and decoded."""
    from eazy_amd import synth

    rng = np.random.default_rng(79)
    d = synth.logs(83, 60 * 65536).tobytes()
    bufs = [d[k << 16 : (k + 1) << 16] for k in range(60)]
    sparse = np.frombuffer(rng.integers(0, 256, 65536, dtype=np.uint8).tobytes(), np.uint8).copy()
    sparse[rng.random(65536) < 0.9] = 0
    bufs += [rng.integers(0, 256, 65536, dtype=np.uint8).tobytes(), sparse.tobytes(), bytes(65536), (b"abc" * 21846)[:65536]]
    _gpu_check(cuda, bufs, kinds=("", "S", "l", "w"))


def _chain_stream(rng, n):
    """Bytes built to make Reader.read's copies read each other within one K2t round: short
    random literals, copies of a recent slice (often one that was itself a copy a few tokens
    back), runs of period 1 - 40 right after a literal, overlapping copies with distance >= 16,
    and zero stretches."""
    b = bytearray(rng.integers(0, 256, 40, dtype=np.uint8).tobytes())
    while len(b) < n:
        k = int(rng.integers(0, 6))
        if k == 0:
            b += rng.integers(0, 256, int(rng.integers(1, 12)), dtype=np.uint8).tobytes()
        elif k in (1, 2):  # a copy of a slice a little back
            d = int(rng.integers(6, min(len(b), 300) + 1))
            L = int(rng.integers(6, 60))
            for _ in range(L):
                b.append(b[-d])
        elif k == 3:  # a run after a short literal
            b += rng.integers(0, 256, int(rng.integers(1, 40)), dtype=np.uint8).tobytes()
            per = int(rng.integers(1, 41))
            for _ in range(int(rng.integers(8, 90))):
                b.append(b[-per])
        elif k == 4:  # an overlapping copy with distance >= 16
            d = min(int(rng.integers(16, 33)), len(b))
            for _ in range(int(rng.integers(d + 1, 3 * d))):
                b.append(b[-d])
        else:
            b += bytes(int(rng.integers(8, 64)))
    return bytes(b[:n])


@pytest.mark.gpu
def test_k2t_copy_chains_within_rounds(cuda):
    """K2t resolves, at each round's start, the copies whose sources are already final: inside
    a literal of the round, or (distance >= 16, not overlapping) inside an earlier copy of the
    round, whose own source they then read, repeatedly.  Streams made of such chains (and runs,
    overlapping copies, zero stretches), 1 KiB - 300 KiB, every K2 decoder against the input,
    statuses and sizes equal to the exact decoder's."""
    import torch

    import eazy_amd as ez

    rng = np.random.default_rng(89)
    lens = [1024, 4096, 5000, 20000, 65536, 70000, 300000] + [int(x) for x in rng.integers(2000, 40000, 25)]
    bufs = [_chain_stream(rng, n) for n in lens]
    want = [orc.compress(MiB, 1024, [b]) for b in bufs]
    coff = np.concatenate([[0], np.cumsum([len(w) for w in want])]).astype(np.int64)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    comp = torch.from_numpy(np.frombuffer(b"".join(want) + bytes(64), np.uint8).copy()).to(cuda)
    d_coff, d_offs = torch.from_numpy(coff).to(cuda), torch.from_numpy(offs).to(cuda)
    _, sz0, st0 = ez.decompress_batch(comp, d_coff, d_offs, exact_only=True)
    assert st0.abs().sum().item() == 0
    for kind in ("t", "w", "r", "j", ""):
        ez.select_decompress_kernel(kind)
        try:
            out, sz, st = ez.decompress_batch(comp, d_coff, d_offs, max_len=max(lens))
        finally:
            ez.select_decompress_kernel("")
        assert torch.equal(st, st0) and torch.equal(sz, sz0), kind
        got = out[: int(offs[-1])].cpu().numpy().tobytes()
        for s, b in enumerate(bufs):
            assert got[offs[s] : offs[s + 1]] == b, f"K2 {kind!r}: stream {s} (len {lens[s]}) differs"


def _defer_stream(rng, n_lit):
    """A literal long enough for K2t/K2w to defer (>= 16 KiB of random bytes), then what reads
    it back: a short-period run seeded by its last bytes, copies from its tail and its middle, and
    more of the same after some fresh bytes."""
    lit = rng.integers(0, 256, n_lit, dtype=np.uint8).tobytes()
    per = int(rng.integers(1, 16))
    out = lit + lit[-per:] * int(rng.integers(3, 40))
    out += lit[-200:-100] + lit[n_lit // 2 : n_lit // 2 + 300]
    out += rng.integers(0, 256, 50, dtype=np.uint8).tobytes() + lit[-24:] + lit[100:140]
    return out


@pytest.mark.gpu
def test_k2t_deferred_literal_neighbours(cuda):
    """K2t does not put a deferred literal (>= 16 KiB, moved later by kd_copy) into its ring: the
    copies and runs that read it right after take its bytes from the input.  Streams of a long
    literal followed by such readers, decoded in a small batch (the 32/64 KiB-ring K2t) and inside
    a batch of 1,100 streams (4/8 KiB rings), every K2 decoder against the input."""
    import torch

    import eazy_amd as ez
    from eazy_amd import synth

    rng = np.random.default_rng(97)
    defer = [_defer_stream(rng, int(n)) for n in rng.integers(16384, 90000, 12)]
    filler = [synth.logs(300 + k, 6000).tobytes() for k in range(1100 - len(defer))]
    for bufs in (defer, defer + filler):
        want = [orc.compress(MiB, 1024, [b]) for b in bufs]
        lens = [len(b) for b in bufs]
        coff = np.concatenate([[0], np.cumsum([len(w) for w in want])]).astype(np.int64)
        offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        comp = torch.from_numpy(np.frombuffer(b"".join(want) + bytes(64), np.uint8).copy()).to(cuda)
        d_coff, d_offs = torch.from_numpy(coff).to(cuda), torch.from_numpy(offs).to(cuda)
        for kind in ("t", "w", "j", ""):
            ez.select_decompress_kernel(kind)
            try:
                out, sz, st = ez.decompress_batch(comp, d_coff, d_offs)
            finally:
                ez.select_decompress_kernel("")
            assert st.abs().sum().item() == 0, kind
            got = out[: int(offs[-1])].cpu().numpy().tobytes()
            for s, b in enumerate(bufs):
                assert got[offs[s] : offs[s + 1]] == b, f"K2 {kind!r}: stream {s} (len {lens[s]}) of {len(bufs)} differs"


@pytest.mark.gpu
def test_decoder_routing_without_hint(cuda):
    """The batch decoder follows the largest output slot, measured on the device when the
    caller gives no max_len: C4-class buckets (4 MiB, literals) take K2t, a few long log streams
    (output at least twice the input) K2j, 16 KiB and 4 KiB streams K2r, each byte-exact against
    the input, with and without the hint."""
    import torch

    import eazy_amd as ez
    from eazy_amd import synth

    cases = [
        ([b.tobytes() for b in np.split(synth.f32(5, 4 * (1 << 20)).view(np.uint8), 4)], "t"),
        ([synth.logs(40 + k, 1 << 20).tobytes() for k in range(4)], "j"),
        ([synth.logs(6 + k, 16 << 10).tobytes() for k in range(8)], "r"),
        ([synth.logs(20 + k, 4096).tobytes() for k in range(40)] + [b"", b"x" * 17], "r"),
    ]
    for bufs, kind in cases:
        want = [orc.compress(MiB, 1024, [b]) for b in bufs]
        lens = [len(b) for b in bufs]
        coff = np.concatenate([[0], np.cumsum([len(w) for w in want])]).astype(np.int64)
        offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        comp = torch.from_numpy(np.frombuffer(b"".join(want) + bytes(64), np.uint8).copy()).to(cuda)
        d_coff, d_offs = torch.from_numpy(coff).to(cuda), torch.from_numpy(offs).to(cuda)
        for kw in ({}, {"max_len": max(lens)}):
            out, sz, st = ez.decompress_batch(comp, d_coff, d_offs, **kw)
            torch.cuda.synchronize()
            assert ez.decompress_kernel_last() == kind, (kind, kw, ez.decompress_kernel_last())
            assert st.abs().sum().item() == 0 and sz.cpu().tolist() == lens, kind
            got = out[: int(offs[-1])].cpu().numpy().tobytes()
            for s, b in enumerate(bufs):
                assert got[offs[s] : offs[s + 1]] == b, f"{kind}: stream {s} differs"


@pytest.mark.gpu
def test_k2j_chip_wide_decode(cuda):
    """K2j (token starts from speculative chunks -- 1 KiB, 256 bytes for batches of at most 96 KiB of
    input, as the single-stream batches below --, token records, pointer jumping over the
    copied bytes) on the shapes its steps must get right, each stream against the oracle (bytes,
    sizes, statuses): copy-of-copy chains across a whole long stream (log templates: every event's
    copy reads the previous event's), runs with distance < 16, OffLong-0 zero regions, copies
    reaching before the stream start, long literals (an entry that skips chunks), padding and
    Break metas between tokens, a stream ending in the middle of a token, a MetaReset after
    output (declines: the exact decoder's error), a slot one byte short, an empty stream; in one
    batch and one stream per batch."""
    import torch

    import eazy_amd as ez
    from eazy_amd import synth

    rng = np.random.default_rng(123)
    hdr = b"\x80\x02eazy\x80\x10\x14"
    logs = synth.logs(127, 3 << 20).tobytes()
    f = rng.standard_normal(300000).astype(np.float32).tobytes()
    zero = bytearray(400000)
    for q in range(0, len(zero), 37):
        zero[q] = q & 0xFF
    ins = [orc.compress(MiB, 1024, [logs]),                                   # 3 MiB of logs: deep chains
           orc.compress(MiB, 1024, [_chain_stream(rng, 500000)]),             # runs, overlapping copies
           orc.compress(MiB, 1024, [f]),                                      # one 1.2 MB literal
           orc.compress(MiB, 1024, [bytes(zero)]),                            # zero runs and patterns
           orc.compress(MiB, 1024, [logs[:70000], f[:5000], logs[70000:90000]]),  # multi-Write
           hdr + b"\x87\xff\x00" + b"\x03abc" + b"\x8a\xff\x05",          # a zero region, a run
           hdr + b"\x03abc" + b"\x86\x04" + b"\x02xy" + b"\x88\x40",        # copies from before the start
           orc.compress(MiB, 1024, [logs[:9000]]) + b"\x00" * 40 + b"\x80\x1f" + b"\x80\x1f" + b"\x05hello",
           orc.compress(MiB, 1024, [logs[:50000]])[:-3],                      # ends inside a token
           orc.compress(MiB, 1024, [logs[:3000]]) + b"\x80\x10\x14\x02ab",   # MetaReset after output
           b""]
    lens = [len(orc.decompress(x, cap=8 << 20)[0]) for x in ins]
    for cap_delta in (0, -1):
        caps = [n + 64 for n in lens]
        caps[0] = lens[0] + cap_delta  # (a slot one byte short: the exact decoder's ENOSPC)
        for batch in ([list(range(len(ins)))] + [[k] for k in range(len(ins))] if cap_delta == 0 else [list(range(len(ins)))]):
            sub = [ins[k] for k in batch]
            scap = [caps[k] for k in batch]
            coff = np.concatenate([[0], np.cumsum([len(x) for x in sub])]).astype(np.int64)
            ooff = np.concatenate([[0], np.cumsum(scap)]).astype(np.int64)
            comp = torch.from_numpy(np.frombuffer(b"".join(sub) + bytes(64), np.uint8).copy()).to(cuda)
            d_coff, d_ooff = torch.from_numpy(coff).to(cuda), torch.from_numpy(ooff).to(cuda)
            ez.select_decompress_kernel("j")
            try:
                out, sz, st = ez.decompress_batch(comp, d_coff, d_ooff, max_len=max(scap))
                torch.cuda.synchronize()
                assert ez.decompress_kernel_last() == "j"
            finally:
                ez.select_decompress_kernel("")
            ex = ez.decompress_batch(comp, d_coff, d_ooff, exact_only=True)
            torch.cuda.synchronize()
            assert torch.equal(st, ex[2]) and torch.equal(sz, ex[1]), (batch, st.tolist(), ex[2].tolist())
            o = out.cpu().numpy()
            for i, k in enumerate(batch):
                want, err, _ = orc.decompress(ins[k], cap=scap[i])
                if err == 2:  # the slot is too small: the status (ENOSPC, as the exact decoder's) is the result
                    assert int(st[i]) == ez.ENOSPC
                    continue
                n = int(sz[i])
                assert int(st[i]) == err and o[ooff[i] : ooff[i] + n].tobytes() == want, (k, n)


@pytest.mark.gpu
def test_c2_full_batch_matches_oracle(cuda):
    """C2 at its full size (BASELINE.json configs[2]): 4,096 x 256 KiB synthetic log streams
    into NewWriter(MiB, 1024), the automatic route (K1L + its token writer, K3, K2t). Every
    stream's packed bytes equal the C oracle's (16 threads) and decode back on the device."""
    import torch

    import eazy_amd as ez
    from eazy_amd import synth

    n, S = 256 << 10, 4096
    host = synth.logs(2026, n * S)
    offs = np.arange(S + 1, dtype=np.int64) * n
    cap = n + (n >> 2) + 64
    slot_off = np.arange(S + 1, dtype=np.int64) * cap
    slots, sizes = orc.compress_batch(MiB, 1024, host, offs, slot_off, 16)
    data = torch.from_numpy(host).to(cuda)
    off = torch.from_numpy(offs).to(cuda)
    cb = ez.compress_batch(data, off, MiB, 1024, append_magic=True)
    packed, poff = ez.pack(cb)
    torch.cuda.synchronize()
    assert int(cb.status.count_nonzero()) == 0
    po = poff.cpu().numpy()
    assert np.array_equal(np.diff(po), sizes), "compressed sizes differ from the oracle's"
    pk = packed[: int(po[-1])].cpu().numpy()
    keep = np.arange(cap)[None, :] < sizes[:, None]
    assert np.array_equal(pk, slots.reshape(S, cap)[keep]), "compressed bytes differ from the oracle's"
    del slots, keep
    out, osz, ost = ez.decompress_batch(packed, poff, off, max_len=n)
    torch.cuda.synchronize()
    assert int(ost.count_nonzero()) == 0 and bool((osz == n).all())
    assert torch.equal(out[: n * S], data), "round trip differs"


@pytest.mark.gpu
@pytest.mark.parametrize("wl", ["c4", "c4h", "c4s"])
def test_c4_full_batches_match_oracle(cuda, wl):
    """C4 at its full size (BASELINE.json configs[4]): 64 x 4 MiB gradient buckets bit-cast to bytes
    (fp32 N(0, 1e-3); its bf16 top halves; fp32 with 90 % zeros), the bench's own bytes
    (bench.workload_bytes), the automatic route (K1x's rounds, then K1c or K1L; K2t or K2j). Every
    stream's packed bytes equal the C oracle's and decode back on the device."""
    import torch

    import bench
    import eazy_amd as ez

    S, n = 64, 4 << 20
    host, _ = bench.workload_bytes(wl, 7, S * n)
    host = np.ascontiguousarray(host)
    offs = np.arange(S + 1, dtype=np.int64) * n
    cap = n + (n >> 2) + 64
    slot_off = np.arange(S + 1, dtype=np.int64) * cap
    slots, sizes = orc.compress_batch(MiB, 1024, host, offs, slot_off, 16)
    data = torch.from_numpy(host).to(cuda)
    off = torch.from_numpy(offs).to(cuda)
    cb = ez.compress_batch(data, off, MiB, 1024, append_magic=True)
    packed, poff = ez.pack(cb)
    torch.cuda.synchronize()
    assert int(cb.status.count_nonzero()) == 0
    po = poff.cpu().numpy()
    assert np.array_equal(np.diff(po), sizes), f"{wl}: compressed sizes differ from the oracle's"
    pk = packed[: int(po[-1])].cpu().numpy()
    keep = np.arange(cap)[None, :] < sizes[:, None]
    assert np.array_equal(pk, slots.reshape(S, cap)[keep]), f"{wl}: compressed bytes differ from the oracle's"
    out, osz, ost = ez.decompress_batch(packed, poff, off, max_len=n)
    torch.cuda.synchronize()
    assert int(ost.count_nonzero()) == 0 and bool((osz == n).all())
    assert torch.equal(out[: n * S], data), f"{wl}: round trip differs"
