"""K1c (the chunk-parallel parse of long fresh streams, ez_compress_split.hip: kc_parse, kc_stitch,
kc_gather, kc_v1, kc_v2, then K1L for the streams it cannot prove) against the oracle, through the
C-ABI.  K1c takes the batches K1L would (single fresh Writes of 64 KiB and more, table <= 4096
entries): C2's log streams directly, K1x's dense streams (longer than half the window) after its
rounds.

Bar: every stream's compressed bytes equal the oracle's and decode back; on log-like streams K1c
proves most streams itself (ez_compress_k1c_stats), so the parity is K1c's and not the fallback's;
on incompressible streams it falls back (no common copy end) and is still exact."""

import numpy as np
import pytest

import oracle as orc

pytestmark = pytest.mark.gpu

MiB = 1 << 20
KiB = 1 << 10


def _compress(cuda, bufs, block=MiB, htable=1024):
    import torch

    import eazy_amd as ez

    lens = np.array([len(b) for b in bufs], np.int64)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    host = np.frombuffer(b"".join(bufs), np.uint8)
    data = torch.from_numpy(host.copy()).to(cuda)
    off = torch.from_numpy(offs).to(cuda)
    ez.k1c_stats(True)
    try:
        cb = ez.compress_batch(data, off, block, htable)
        packed, poff = ez.pack(cb)
        torch.cuda.synchronize()
    finally:
        st = ez.k1c_stats(False)
    pk, po = packed.cpu().numpy(), poff.cpu().numpy()
    assert (cb.status.cpu().numpy() == 0).all()
    for s, b in enumerate(bufs):
        want = orc.compress(block, htable, [b])
        assert pk[po[s] : po[s + 1]].tobytes() == want, f"stream {s} (len {len(b)}): compressed bytes differ ({st})"
    out, sizes, status = ez.decompress_batch(packed, poff, off)
    torch.cuda.synchronize()
    assert (status.cpu().numpy() == 0).all()
    assert out[: int(offs[-1])].cpu().numpy().tobytes() == b"".join(bufs)
    return st


def _logs(seed, n):
    from eazy_amd import synth

    return synth.logs(seed, n).tobytes()


def test_k1c_log_streams(cuda):
    """C2's shape at 16 streams: 256 KiB log Writes, 8 chunks each."""
    d = _logs(61, 16 * 256 * KiB)
    bufs = [d[k * 256 * KiB : (k + 1) * 256 * KiB] for k in range(16)]
    st = _compress(cuda, bufs)
    assert st["proven"] + st["chunk"] + st["sync"] + st["judge"] + st["cap"] == 16, st
    assert st["proven"] >= 12, st


def test_k1c_ragged_and_boundaries(cuda):
    """Streams ending at, just past and just before chunk boundaries (64 KiB, 64 KiB + 3, 96 KiB,
    2 chunks - 1), ragged lengths up to 300 KiB, and short, empty and tiny streams beside them."""
    d = _logs(67, 4 * MiB)
    rng = np.random.default_rng(67)
    lens = [65536, 65539, 98304, 65535, 131072 + 7, 4096, 0, 3, 70000]
    lens += [int(v) for v in rng.integers(64 * KiB, 300 * KiB, 8)]
    bufs, at = [], 0
    for n in lens:
        bufs.append(d[at : at + n])
        at += n
    st = _compress(cuda, bufs)
    assert st["proven"] >= 8, st


def test_k1c_incompressible_falls_back(cuda):
    """Random bytes: no copy ends to stitch at, every stream goes to K1L, the bytes are still Go's."""
    rng = np.random.default_rng(71)
    bufs = [rng.integers(0, 256, 200 * KiB, dtype=np.uint8).tobytes() for _ in range(4)]
    st = _compress(cuda, bufs)
    assert st["proven"] + st["sync"] + st["chunk"] + st["judge"] == 4, st


def test_k1c_planted_events(cuda):
    """Random streams with many planted copies (distances up to past the window), short-period
    runs, zero runs and the stream's first bytes again: table entries far back, which the chunks'
    warm-up does not see, so the re-judgement (kc_recheck) decides."""
    from test_gpu_batch import _planted

    rng = np.random.default_rng(73)
    bufs = [_planted(rng, 256 * KiB, e, MiB, zeros=z) for e, z in ((400, False), (3000, True), (8000, True), (20000, False))]
    _compress(cuda, bufs)
    bufs = [_planted(rng, 160 * KiB, e, 64 * KiB, zeros=True) for e in (500, 5000)]
    _compress(cuda, bufs, 64 * KiB, 4096)


@pytest.mark.parametrize("htable", [256, 4096])
def test_k1c_tables(cuda, htable):
    d = _logs(79, 8 * 192 * KiB)
    _compress(cuda, [d[k * 192 * KiB : (k + 1) * 192 * KiB] for k in range(8)], MiB, htable)


def test_k1c_after_k1x(cuda):
    """Writes longer than half the window (K1x's rounds, then K1c from K1x's state): 1 MiB logs and
    90 %-zero fp32 in a 256 KiB window (ring image, far skips, the cut branch), 1 MiB in 1 MiB."""
    from eazy_amd import synth

    d = _logs(83, 4 * MiB)
    sp = synth.f32(89, MiB // 4)
    sp[np.random.default_rng(89).random(sp.shape[0]) < 0.9] = 0.0
    spb = sp.view(np.uint8).tobytes()
    bufs = [d[:MiB], d[MiB : 2 * MiB], spb, d[2 * MiB : 2 * MiB + 700 * KiB]]
    _compress(cuda, bufs, 256 * KiB, 1024)
    _compress(cuda, bufs, MiB, 1024)


@pytest.mark.parametrize("count", [8, 1100])
def test_wide_token_writer_small_slots(cuda, count):
    """The chip-wide token writer (ke_size / ke_scan / ke_write) after K1c (8 streams) and after
    K1L (1,100 streams: k1_emit<true>): slots of the exact size, one byte short, half, and shorter than the header;
    a short slot ends the output at a token boundary with ENOSPC, its bytes a prefix of Go's."""
    import torch

    import eazy_amd as ez

    n = 72 * KiB
    d = _logs(97, count * n)
    bufs = [d[k * n : (k + 1) * n] for k in range(count)]
    want = [orc.compress(MiB, 1024, [b]) for b in bufs]
    caps = []
    for k, w in enumerate(want):
        caps.append([len(w), len(w) - 1, len(w) // 2, 5, len(w) + 100][k % 5])
    slot = np.concatenate([[0], np.cumsum([(c + 15) & ~15 for c in caps])]).astype(np.int64)
    # (each slot's capacity is its exact cap: the next slot starts right after it)
    slot_cap = np.concatenate([[0], np.cumsum(caps)]).astype(np.int64)
    data = torch.from_numpy(np.frombuffer(d, np.uint8).copy()).to(cuda)
    off = torch.from_numpy(np.arange(count + 1, dtype=np.int64) * n).to(cuda)
    cb = ez.compress_batch(data, off, MiB, 1024, slot_off=torch.from_numpy(slot_cap).to(cuda))
    torch.cuda.synchronize()
    slots, sizes, status = cb.slots.cpu().numpy(), cb.sizes.cpu().numpy(), cb.status.cpu().numpy()
    for k, w in enumerate(want):
        c = caps[k]
        got = slots[slot_cap[k] : slot_cap[k] + int(sizes[k])].tobytes()
        if c >= len(w):
            assert status[k] == 0 and got == w, k
        else:
            assert status[k] == ez.ENOSPC, (k, status[k])
            assert int(sizes[k]) <= c and got == w[: int(sizes[k])], k
            if c >= 9:
                assert int(sizes[k]) > 0, k
    del slot


def test_k1c_full_1mib_batch(cuda):
    """The sweep's 1 MiB line at its full size: 1,024 x 1 MiB log Writes (longer than half the
    window: K1x's rounds hand the dense streams over, then K1c with its passes, K1L for what it
    cannot prove). Every stream equal to the oracle, decoded back; most proven by K1c itself."""
    d = _logs(67, 1024 * MiB)
    bufs = [d[k * MiB : (k + 1) * MiB] for k in range(1024)]
    st = _compress(cuda, bufs)
    assert st["proven"] + st["chunk"] + st["sync"] + st["judge"] + st["cap"] == 1024, st
    assert st["proven"] >= 512, st
