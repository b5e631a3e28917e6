"""N>1 layout of the batch path on the CPU (gloo, world size 2): shards are
disjoint whole-stream ranges, the job time is the max over ranks, and the
job's byte counts are the sum of the independent shards.
Launched exactly like bench.py's multi-GPU path (torch.distributed.run)."""

import json
import os
import socket
import subprocess
import sys

import numpy as np

import oracle as orc
from eazy_amd import dist as ezd
from eazy_amd import synth

HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_layout_single_process():
    rs = [ezd.Rank(r, 4, r) for r in range(4)]
    assert [ezd.shard(10, r) for r in rs] == [(0, 10), (10, 20), (20, 30), (30, 40)]
    assert len({ezd.seed(1000, r) for r in rs}) == 4
    assert ezd.reduce_max([1.5, 2], ezd.Rank(0, 1, 0)) == [1.5, 2.0]
    assert ezd.reduce_sum([3, 4], ezd.Rank(0, 1, 0)) == [3, 4]


def test_two_rank_gloo(tmp_path):
    out = tmp_path / "r0.json"
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(HERE, "helpers", "dist_worker.py"), str(out)]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    r = json.load(open(out))
    assert r["world"] == 2 and r["ms"] == 2.0
    assert [x[:2] for x in r["ranges"]] == [[0, 32], [32, 64]]
    # the job's compressed bytes = the sum of each shard compressed alone
    want = 0
    for rank in range(2):
        host = synth.logs(1000 + rank, 32 * 1024)
        for s in range(32):
            want += len(orc.compress(1 << 20, 1024, [host[s * 1024 : (s + 1) * 1024].tobytes()]))
    assert r["comp"] == want and r["in"] == 2 * 32 * 1024
    assert [x[2] for x in r["ranges"]] != [0, 0]
