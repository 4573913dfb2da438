"""Multi-GPU sharding and the control plane for batched MD5.

Digests depend only on their own chunk, so a batch splits into contiguous
index ranges, one per GPU, with NO data-path collective; each rank hashes its
range on its own device and writes its digests to its slice of the output.
The only cross-rank traffic is control: a barrier before/after the timed
region, scalar MAX/SUM reductions of elapsed time and bytes, and small object
gathers (each rank's rate, device and parity sample).  bench.py runs exactly
these functions; tests/test_multi.py runs them on world-size-2 gloo groups.

The backend is gloo (CPU) by default: a live RCCL communicator made the C2
kernel 3-5 % slower on its GPU (profiles/r05w/), and the control plane moves
a few scalars.  "nccl" (RCCL) carries the same calls on the GPUs.
"""
import os
import socket

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


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def init_group(world: int, backend: str = "gloo", device=None, always: bool = False) -> bool:
    """Bring the control plane up when world > 1 (or `always`: a one-rank
    group, the rehearsal of the N > 1 path on one GPU).  Rendezvous on
    127.0.0.1 from torch.distributed.run's environment (a one-rank group
    without a launcher picks a free port).  Returns whether a group is up."""
    if world == 1 and not always:
        return False
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if world == 1:
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        os.environ.setdefault("MASTER_PORT", str(free_port()))
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", device))
    else:
        dist.init_process_group("gloo")
    return True


def group_on() -> bool:
    return dist.is_available() and dist.is_initialized()


def _coll_device():
    return "cuda" if dist.get_backend() == "nccl" else "cpu"


def barrier():
    if group_on():
        dist.barrier()


def _reduce(x: float, op) -> float:
    if not group_on():
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=_coll_device())
    dist.all_reduce(t, op=op)
    return float(t.item())


def max_over_ranks(x: float) -> float:
    """MAX of a per-rank scalar (the slowest rank bounds the job)."""
    return _reduce(x, dist.ReduceOp.MAX)


def sum_over_ranks(x: float) -> float:
    return _reduce(x, dist.ReduceOp.SUM)


def gather_objects(obj) -> list:
    """Every rank's `obj`, in rank order (one element without a group)."""
    if not group_on():
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out


def aggregate_rate(bytes_per_rank: float, seconds: float) -> dict:
    """Whole-job throughput: bytes all ranks processed / max time over ranks."""
    total = sum_over_ranks(bytes_per_rank)
    tmax = max_over_ranks(seconds)
    return {"total_bytes": total, "max_seconds": tmax, "bytes_per_s": total / tmax if tmax else 0.0}


def close_group():
    """Final barrier and teardown (no rank leaves while another still reduces)."""
    if group_on():
        dist.barrier()
        dist.destroy_process_group()
