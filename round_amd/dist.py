"""Multi-GPU plumbing: one process per GPU, instance-range sharding, counter all-reduce.

Instances are independent, so the data path has no collective: rank r owns the
global instance ids [r*I, (r+1)*I) (weak scaling) and every random draw is keyed
on the global id, making results independent of the sharding. The only
exchange is one all-reduce(sum) of the psg_summary int64 counters (violation
counts, termination histogram, decided processes, digest) per batch — < 3 KB,
latency-bound. With backend "nccl" this is RCCL over xGMI; the
CPU tests run the same code over gloo.
"""
import torch
import torch.distributed as dist

from . import abi


def shard(rank: int, world: int, per_rank: int):
    """(first global instance id, count) owned by `rank` under weak scaling."""
    if not (0 <= rank < world):
        raise ValueError(f"rank {rank} outside world {world}")
    return rank * per_rank, per_rank


def shard_strong(rank: int, world: int, total: int):
    """(first id, count) for a fixed total split as evenly as possible (strong scaling)."""
    lo = total * rank // world
    hi = total * (rank + 1) // world
    return lo, hi - lo


def allreduce_summary(s: abi.Summary, device=None) -> abi.Summary:
    """Sum the counters of a Summary over all ranks; kernel_ns becomes the max."""
    vals = abi.summary_to_list(s)
    dev = device if device is not None else "cpu"
    t = torch.tensor(vals[:-1], dtype=torch.int64, device=dev)
    k = torch.tensor([vals[-1]], dtype=torch.int64, device=dev)
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        dist.all_reduce(k, op=dist.ReduceOp.MAX)
    return abi.summary_from_list(t.cpu().tolist() + k.cpu().tolist())


def allreduce_max(x: float, device=None) -> float:
    t = torch.tensor([x], dtype=torch.float64, device=device if device is not None else "cpu")
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def allgather_float(x: float, rank: int, world: int, device=None) -> list:
    """Every rank's value of x, in rank order (a zero vector with this rank's slot set,
    summed over ranks)."""
    t = torch.zeros(world, dtype=torch.float64, device=device if device is not None else "cpu")
    t[rank] = x
    if dist.is_available() and dist.is_initialized() and world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [float(v) for v in t.cpu().tolist()]
