"""Multi-GPU sharding of a packet batch.

Packets are independent, so a batch splits into contiguous packet ranges, one per
GPU, balanced by bytes; each rank checksums its own range on its own device and
writes a disjoint slice of the output.  There is no data-path collective; the
only cross-rank operation is the max-over-ranks reduction of timings in bench.py.
"""
from __future__ import annotations

from typing import Sequence

import numpy as np


def shard_bounds(world: int, rank: int, *, count: int | None = None, lengths=None) -> tuple[int, int]:
    """[lo, hi) packet range of `rank` out of `world`.

    Uniform batches (`count`): an even split.  Ragged batches (`lengths`): split at
    the packet boundaries nearest to k * total_bytes / world, so every rank reads
    within one packet of total/world bytes.
    """
    if world < 1 or not 0 <= rank < world:
        raise ValueError("need 0 <= rank < world")
    if lengths is None:
        if count is None or count < 0:
            raise ValueError("give count or lengths")
        return count * rank // world, count * (rank + 1) // world
    ln = np.asarray(lengths, dtype=np.uint64)
    if ln.size == 0:
        return 0, 0
    ends = np.cumsum(ln, dtype=np.uint64)  # byte end of each packet
    total = int(ends[-1])

    def cut(k: int) -> int:
        if k <= 0:
            return 0
        if k >= world:
            return int(ln.size)
        target = total * k // world
        return int(np.searchsorted(ends, np.uint64(target), side="left")) + 1 if target else 0

    lo, hi = cut(rank), cut(rank + 1)
    return min(lo, hi), hi


def max_over_ranks(values: Sequence[float], device=None) -> list[float]:
    """Element-wise max of `values` over all ranks (identity without a process group)."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [float(v) for v in values]
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(v) for v in t.cpu()]
