"""Multi-GPU sharding of the read set.

Reads are independent given the global chunk heads (fixed by -n_threads and
the full query, IMSAME.c:414), so one query is split into contiguous read
ranges, one per rank; every rank holds a replica of the index.  The only
collective is a reduction of a few counters (RCCL over xGMI with the "nccl"
backend, gloo on CPU in the tests).
"""
import numpy as np


def shard_range(n_reads, rank, world):
    """Contiguous [from, to) of rank `rank` out of `world`."""
    return (n_reads * rank) // world, (n_reads * (rank + 1)) // world


def _device_for_backend():
    import torch
    import torch.distributed as dist
    if dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def all_reduce(values, op="sum"):
    """Reduce a short list of numbers across ranks (one collective)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=_device_for_backend())
    dist.all_reduce(t, op=dist.ReduceOp.SUM if op == "sum" else dist.ReduceOp.MAX)
    return [float(x) for x in t.cpu().tolist()]


def align_sharded(align_fn, n_reads, rank, world, n_threads):
    """Run align_fn(read_from, read_to, n_threads) -> per-read results on this
    rank's shard; returns (results, (from, to), [accepted_total, reads_total])."""
    a, b = shard_range(n_reads, rank, world)
    res = align_fn(a, b, n_threads)
    acc = int(np.count_nonzero(res["status"] == 1))
    tot = all_reduce([acc, b - a])
    return res, (a, b), [int(tot[0]), int(tot[1])]
