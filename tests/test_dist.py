"""The N>1 data path at world size 2 over gloo, launched exactly
like bench.py's multi-GPU path (torch.distributed.run): one global batch split
into contiguous whole-stream shards, an all-gather of per-stream compressed
sizes into global packed offsets, and the payload gathered to rank 0.  The
gathered bytes must equal the single-rank packing of the whole batch (the
streams' oracle bytes back to back).  The "gpu" variant compresses each shard
with the HIP kernels on cuda:0 (two ranks sharing the one GPU of the box)."""

import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import oracle as orc
from eazy_amd import dist as ezd

HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_layout_single_process():
    rs = [ezd.Rank(r, 4, r) for r in range(4)]
    assert [ezd.shard_range(10, r) for r in rs] == [(0, 2), (2, 5), (5, 7), (7, 10)]
    assert [ezd.shard_range(1 << 20, ezd.Rank(r, 8, r))[0] for r in range(8)] == [k << 17 for k in range(8)]
    assert ezd.shard_counts(10, 4) == [2, 3, 2, 3]
    assert ezd.reduce_max([1.5, 2], ezd.Rank(0, 1, 0)) == [1.5, 2.0]
    assert ezd.reduce_sum([3, 4], ezd.Rank(0, 1, 0)) == [3, 4]


def test_global_logs_rank_independent():
    """A rank's streams of the global batch do not depend on the split."""
    from eazy_amd import synth

    whole = synth.global_logs(5, 0, 40, 64, chunk=16)
    for a, b in ((0, 13), (13, 27), (27, 40), (16, 32)):
        assert np.array_equal(synth.global_logs(5, a, b, 64, chunk=16), whole[a * 64 : b * 64])
    assert np.array_equal(whole[: 16 * 64], synth.logs(5, 16 * 64))


def _run(tmp_path, mode, nproc=2):
    sys.path.insert(0, os.path.join(HERE, "helpers"))
    import dist_worker as dw

    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(HERE, "helpers", "dist_worker.py"), str(tmp_path), mode]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    host, offs = dw.global_batch()
    want = [orc.compress(1 << 20, 1024, [host[offs[s] : offs[s + 1]].tobytes()]) for s in range(dw.COUNT)]
    sizes = np.load(tmp_path / "sizes.npy")
    goff = np.load(tmp_path / "offsets.npy")
    packed = np.load(tmp_path / "packed.npy").tobytes()
    assert sizes.tolist() == [len(w) for w in want]
    assert goff.tolist() == np.concatenate([[0], np.cumsum([len(w) for w in want])]).tolist()
    assert packed == b"".join(want), "gathered packing differs from the single-rank packing"
    spans = [tuple(map(int, x.split(":"))) for x in open(tmp_path / "ranges.txt").read().split()]
    assert spans[0][0] == 0 and sum(n for _, n in spans) == len(packed)
    assert all(spans[k + 1][0] == spans[k][0] + spans[k][1] for k in range(len(spans) - 1))


def test_two_rank_gloo_exchange(tmp_path):
    _run(tmp_path, "cpu")


def test_bench_launches_ranks_itself():
    """`python bench.py --gpus 2` outside torchrun starts the 2 ranks itself (one
    child process tree) and rank 0's JSON line comes back on stdout; the
    rehearsal runs the same shard split, size all-gather and payload gather."""
    import json

    env = dict(os.environ, OMP_NUM_THREADS="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    bench = os.path.join(os.path.dirname(HERE), "bench.py")
    p = subprocess.run([sys.executable, bench, "--gpus", "2", "--rehearse", "--streams", "67", "--stream-bytes", "300"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["streams_per_rank"] == [33, 34] and res["gathered_equals_input"]
    assert res["bytes_gathered"] == 67 * 300


def test_c3_rehearsal_full_size():
    """C3 at full size on the CPU: `bench.py --gpus 8 --rehearse` over 1,048,576 x 4 KiB
    streams (gloo, 8 ranks: 131,072-stream shards, an 8 MiB int64 size all-gather, the
    global offsets, the 4 GiB payload gather to rank 0, checked against the input)."""
    import json

    env = dict(os.environ, OMP_NUM_THREADS="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    bench = os.path.join(os.path.dirname(HERE), "bench.py")
    p = subprocess.run([sys.executable, bench, "--gpus", "8", "--rehearse", "--streams", "1048576", "--stream-bytes", "4096"],
                       env=env, capture_output=True, text=True, timeout=900)
    assert p.returncode == 0, p.stderr[-3000:]
    res = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert res["n_gpus"] == 8 and res["streams_per_rank"] == [131072] * 8 and res["gathered_equals_input"]
    assert res["bytes_gathered"] == 1048576 * 4096


def test_bench_rejects_world_mismatch():
    """--gpus must equal the world size the launch ends up with."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    bench = os.path.join(os.path.dirname(HERE), "bench.py")
    p = subprocess.run([sys.executable, bench, "--gpus", "2", "--rehearse"], env=env, capture_output=True, text=True,
                       timeout=120)
    assert p.returncode != 0 and "WORLD_SIZE" in p.stderr


@pytest.mark.gpu
def test_two_rank_exchange_gpu_kernels(tmp_path, cuda):
    _run(tmp_path, "gpu")


@pytest.mark.gpu
def test_rccl_exchange_world1(tmp_path, cuda):
    """The RCCL binding on hardware, every round: one rank on the box's GPU with the nccl
    backend (RCCL), the device bound before the process group starts, the shard compressed by
    the HIP kernels, and the size all-gather (all_gather_into_tensor), payload gather and
    all-reduces run as RCCL collectives (no world-1 shortcut once a group exists); the global
    offsets and packed bytes must equal the oracle's packing of the whole batch."""
    _run(tmp_path, "nccl", nproc=1)


def test_collectives_without_group_shortcut():
    """Without a process group a world-1 run needs no collective; with one it takes them."""
    import torch

    r = ezd.Rank(0, 1, 0)
    assert not ezd._collective(r)
    t = torch.arange(5, dtype=torch.int64)
    assert ezd.exchange_sizes(t, 5, r).tolist() == t.tolist()
