"""Worker for tests/test_dist.py, launched like bench.py's N>1 path:
python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 ...
It runs the sharded batch layout of eazy_amd.dist on the CPU (gloo), with the
C oracle standing in for the GPU kernels, and writes rank 0's view to argv[1]."""

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]

import numpy as np
import torch.distributed as dist

import oracle as orc
from eazy_amd import dist as ezd
from eazy_amd import synth

PER_RANK, SIZE = 32, 1024


def main():
    R = ezd.from_env()
    dist.init_process_group("gloo")
    host = synth.logs(ezd.seed(1000, R), PER_RANK * SIZE)
    offs = synth.batch_offsets(PER_RANK, SIZE)
    cap = np.diff(offs) + (np.diff(offs) >> 2) + 32
    slot_off = np.concatenate([[0], np.cumsum(cap)]).astype(np.int64)
    slots, sizes = orc.compress_batch(1 << 20, 1024, host, offs.astype(np.int64), slot_off, 1)
    comp = int(np.sum(sizes))
    ezd.barrier(R)
    fake_ms = 1.0 + R.rank  # the slowest rank sets the job's time
    (ms,) = ezd.reduce_max([fake_ms], R)
    total_in, total_comp = ezd.reduce_sum([PER_RANK * SIZE, comp], R)
    first, last = ezd.shard(PER_RANK, R)
    ranges = [None] * R.world
    dist.all_gather_object(ranges, [first, last, comp])
    if R.is_root:
        json.dump({"world": R.world, "ms": ms, "in": total_in, "comp": total_comp, "ranges": ranges}, open(sys.argv[1], "w"))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
