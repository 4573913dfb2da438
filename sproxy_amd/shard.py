"""Multi-GPU sharding for batched MD5.

Digests depend only on their own chunk, so a batch splits into contiguous
index ranges, one per GPU, with NO data-path collective; each rank hashes its
range on its own device and writes its digests to its slice of the output.
The only cross-rank traffic is control: a barrier before/after the timed
region and one scalar MAX reduction of the elapsed time.  These helpers take
the process group's device so the same code runs under RCCL ("nccl") on the
GPUs and under gloo on the CPU (tests/test_multi.py).
"""
import os

import torch
import torch.distributed as dist


def shard_range(n: int, rank: int, world: int):
    """[lo, hi) of rank's contiguous share of n chunks: [r*n/W, (r+1)*n/W)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    return n * rank // world, n * (rank + 1) // world


def env_rank():
    """(rank, world, local_rank) from torch.distributed.run's environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def barrier(world: int):
    if world > 1:
        dist.barrier()


def max_over_ranks(x: float, world: int, device="cpu") -> float:
    """MAX of a per-rank scalar (the slowest rank bounds the job)."""
    if world == 1:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x: float, world: int, device="cpu") -> float:
    if world == 1:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def aggregate_rate(bytes_per_rank: float, seconds: float, world: int, device="cpu") -> dict:
    """Whole-job throughput: bytes all ranks processed / max time over ranks."""
    total = sum_over_ranks(bytes_per_rank, world, device)
    tmax = max_over_ranks(seconds, world, device)
    return {"total_bytes": total, "max_seconds": tmax, "bytes_per_s": total / tmax if tmax else 0.0}
