"""Worker for tests/test_dist.py, launched like bench.py's N>1 path:
python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 ...

It runs the sharded data path of eazy_amd.dist over gloo: every
rank takes its contiguous range of whole streams of ONE global batch (ragged
lengths, an uneven split), produces its packed shard, all-gathers the
per-stream compressed sizes into global offsets and sends its packed bytes to
rank 0.  argv: out_dir mode.  mode "cpu": the shard's bytes come from the C
oracle (no GPU in the container; the exchange code is the product's).  mode
"gpu": the shard is compressed and packed by the HIP kernels on cuda:0 (K1 +
K3 through the C-ABI), then the exchange runs on host copies (gloo).  mode
"nccl": the "gpu" shard, with the exchange on device tensors over RCCL (the
backend bench.py's N>1 path uses; launched at world size 1 on a one-GPU box, the
all-gather, payload gather and all-reduces still run as collectives).  Rank 0
writes the global sizes, offsets and packed bytes to out_dir."""

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]

import numpy as np
import torch
import torch.distributed as dist

from eazy_amd import dist as ezd

COUNT = 67


def global_batch():
    """The one global batch every rank slices (seeded, rank-independent)."""
    from eazy_amd import synth

    rng = np.random.default_rng(77)
    lens = rng.integers(0, 6000, COUNT)
    lens[::11] = 0
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    return synth.logs(79, int(offs[-1])), offs


def shard_packed(host, offs, mode):
    """(packed bytes, per-stream sizes) of the streams data[offs[0]:offs[-1]]."""
    o = (offs - offs[0]).astype(np.int64)
    data = host[offs[0] : offs[-1]]
    if mode == "gpu":
        import eazy_amd as ez

        dev = torch.device("cuda:0")
        d = torch.from_numpy(data.copy() if len(data) else np.zeros(1, np.uint8)).to(dev)
        cb = ez.compress_batch(d, torch.from_numpy(o).to(dev), ez.MiB, 1024)
        packed, poff = ez.pack(cb)
        torch.cuda.synchronize()
        assert int(cb.status.abs().sum()) == 0
        po = poff.cpu()
        return packed[: int(po[-1])].cpu(), (po[1:] - po[:-1]).to(torch.int64)
    import oracle as orc

    n = np.diff(o)
    slot_off = np.concatenate([[0], np.cumsum(n + (n >> 2) + 32)]).astype(np.int64)
    slots, sizes = orc.compress_batch(1 << 20, 1024, data, o, slot_off, 1)
    pk = b"".join(slots[slot_off[s] : slot_off[s] + sizes[s]].tobytes() for s in range(len(n)))
    return torch.frombuffer(bytearray(pk or b"\0"), dtype=torch.uint8), torch.from_numpy(sizes.astype(np.int64))


def main():
    out_dir, mode = sys.argv[1], sys.argv[2]
    R = ezd.from_env()
    dev = None
    if mode == "nccl":
        torch.cuda.set_device(R.local)
        dev = torch.device("cuda", R.local)
        dist.init_process_group("nccl", device_id=dev)
        assert dist.get_backend() == "nccl" and ezd._collective(R)
    else:
        dist.init_process_group("gloo")
    host, offs = global_batch()
    first, last = ezd.shard_range(COUNT, R)
    packed, sizes = shard_packed(host, offs[first : last + 1], "cpu" if mode == "cpu" else "gpu")
    if dev is not None:
        packed, sizes = packed.to(dev), sizes.to(dev)
    gsz = ezd.exchange_sizes(sizes, COUNT, R)
    goff = ezd.global_offsets(gsz)
    # this rank's shard lands at the global offset of its first stream
    assert int(goff[last]) - int(goff[first]) == int(sizes.sum())
    out = ezd.gather_payload(packed, goff, COUNT, R)
    total = ezd.reduce_sum([int(sizes.sum())], R, device=dev)[0]
    assert total == int(goff[-1])
    slowest = ezd.reduce_max([1.0 + R.rank], R, device=dev)[0]
    assert slowest == float(R.world)
    ezd.barrier(R)
    if dev is not None:
        gsz, goff, out = gsz.cpu(), goff.cpu(), out.cpu() if out is not None else None
    if R.is_root:
        np.save(os.path.join(out_dir, "sizes.npy"), gsz.numpy())
        np.save(os.path.join(out_dir, "offsets.npy"), goff.numpy())
        np.save(os.path.join(out_dir, "packed.npy"), out[: int(goff[-1])].numpy())
        with open(os.path.join(out_dir, "ranges.txt"), "w") as f:
            f.write(" ".join(f"{a}:{b}" for a, b in ezd.rank_bytes(goff, COUNT, R.world)))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
