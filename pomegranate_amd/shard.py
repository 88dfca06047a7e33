"""Block sharding across the GPUs of one node.

Blocks are independent (no cross-block dictionary: wrkmem is per call and
lzo1x_decompress keeps no state), so global block i goes to rank i mod G and
no block data crosses xGMI.  The only collective is the completion barrier: a
sum of per-rank error counts (RCCL all-reduce on the "nccl" backend, gloo in
the CPU tests) and a max of per-rank elapsed times for the report.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple


def round_robin(nglobal: int, rank: int, world: int) -> List[int]:
    """Global block ids owned by `rank`: i = rank, rank + G, rank + 2G, ..."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    return list(range(rank, nglobal, world))


def per_rank_bytes(sizes: Sequence[int], world: int) -> List[int]:
    """Uncompressed bytes each rank receives under round-robin (C4 imbalance)."""
    out = [0] * world
    for i, s in enumerate(sizes):
        out[i % world] += int(s)
    return out


def completion_barrier(dist, device, errors: int, elapsed_s: float) -> Tuple[int, float]:
    """All-reduce (sum errors, max elapsed) over the process group."""
    import torch
    if dist.get_backend() == "gloo":            # gloo collectives run on host tensors
        device = torch.device("cpu")
    t = torch.tensor([float(errors)], dtype=torch.float64, device=device)
    e = torch.tensor([float(elapsed_s)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    dist.all_reduce(e, op=dist.ReduceOp.MAX)
    return int(t.item()), float(e.item())
