"""Multi-GPU sharding of the hot path: one process per GPU, images partitioned.

The reference processes one image per request; its images are independent, so the
batch is split into contiguous per-rank shards and every rank runs the full pipeline
on its own GPU with no data-path collective (weak scaling).  Every image keeps its
global index, which fixes its noise / k-means seeds, so a result does not depend on
the world size or on which rank processed it.  The only collectives are control-plane:
a barrier around timed regions, a MAX of the per-rank wall time, and (optionally) the
gather of the small per-image result records to one rank.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple


def shard_bounds(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous, balanced [start, stop) of ``n`` items for ``rank`` of ``world``
    (the first n % world ranks take one extra item)."""
    if world < 1 or not 0 <= rank < world or n < 0:
        raise ValueError(f"bad shard request n={n} rank={rank} world={world}")
    q, r = divmod(n, world)
    start = rank * q + min(rank, r)
    return start, start + q + (1 if rank < r else 0)


def _dist():
    import torch.distributed as dist

    return dist if dist.is_available() and dist.is_initialized() else None


def max_over_ranks(value: float, device=None) -> float:
    """MAX of a per-rank scalar (bench timing); identity without a process group."""
    dist = _dist()
    if dist is None:
        return float(value)
    import torch

    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_gather(obj) -> List:
    """Every rank's ``obj`` (a small picklable record), in rank order, on every rank;
    ``[obj]`` without a process group."""
    dist = _dist()
    if dist is None:
        return [obj]
    out: List = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out


def barrier(device=None):
    import torch

    if device is not None and torch.cuda.is_available():
        torch.cuda.synchronize(device)
    dist = _dist()
    if dist is not None:
        dist.barrier()


def run_sharded(n_total: int, process: Callable[[int, int], Sequence], gather_to: Optional[int] = 0) -> Optional[List]:
    """Run ``process(start, stop)`` on this rank's shard of ``n_total`` images.

    ``process`` returns the per-image records of its shard (in order).  With
    ``gather_to`` set, the records of all ranks are gathered (gloo/RCCL object gather)
    and returned, in global order, on that rank (None elsewhere); with
    ``gather_to=None`` each rank returns only its own records."""
    dist = _dist()
    rank, world = (dist.get_rank(), dist.get_world_size()) if dist is not None else (0, 1)
    a, b = shard_bounds(n_total, rank, world)
    local = list(process(a, b))
    if len(local) != b - a:
        raise RuntimeError(f"rank {rank}: process returned {len(local)} records for {b - a} images")
    if dist is None or gather_to is None:
        return local
    parts = [None] * world if rank == gather_to else None
    dist.gather_object(local, parts, dst=gather_to)
    if rank != gather_to:
        return None
    out: List = []
    for p in parts:  # ranks hold consecutive shards
        out.extend(p)
    return out
