"""Multi-GPU sharding of source rows (one process per GPU, torch.distributed).

Source rows are independent: attached sources are split into contiguous
blocks, one per rank; the only exchange step is the runahead minimum (all-reduce MIN
of one double) and, where a device-resident full table is needed, an all-gather of
the row shards (RCCL over xGMI with backend "nccl"; gloo on CPU for tests).
"""
from __future__ import annotations

import math


def shard_range(n_items: int, world: int, rank: int):
    """Contiguous block [lo, hi) of rank `rank` (blocks of ceil(n/world))."""
    blk = math.ceil(n_items / world) if world > 0 else n_items
    lo = min(n_items, rank * blk)
    hi = min(n_items, lo + blk)
    return lo, hi


def block_rows(n_items: int, world: int) -> int:
    return math.ceil(n_items / world) if world > 0 else n_items


def runahead_min(local_min, dist, group=None):
    """All-reduce MIN of the per-rank minimum path latency (tensor of shape [1])."""
    if dist is not None and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(local_min, op=dist.ReduceOp.MIN, group=group)
    return local_min


def allgather_rows(local_rows, n_total: int, dist, group=None):
    """All-gather row shards (each [rows_r, nt]) into a new full [n_total, nt] table.
    Shards are padded to the common block size for the collective."""
    import torch
    world = dist.get_world_size(group) if dist is not None and dist.is_initialized() else 1
    if world == 1:
        return local_rows
    blk = block_rows(n_total, world)
    pad = blk - local_rows.shape[0]
    send = local_rows if pad == 0 else torch.nn.functional.pad(local_rows, (0, 0, 0, pad))
    out = torch.empty((blk * world,) + tuple(send.shape[1:]), dtype=send.dtype, device=send.device)
    dist.all_gather_into_tensor(out, send.contiguous(), group=group)
    return out[:n_total]


def full_table(n_total: int, nt: int, world: int, rank: int, like, blk: int = 0):
    """A [blk * world, nt] table (blk defaults to ceil(n_total/world)) whose rank block is
    this rank's shard: rows are computed straight into `shard` and gathered in place
    (allgather_inplace), so the C4 table (20 GB per f64 array) never needs a second copy.
    With seeded plans the blocks hold each rank's plan rows (shd_route_plan_rows), padded
    to the largest block."""
    import torch
    blk = blk or block_rows(n_total, world)
    full = torch.empty((blk * world, nt), dtype=like.dtype, device=like.device)
    return full, full[rank * blk:(rank + 1) * blk]


def allgather_inplace(full, dist, group=None):
    """In-place all-gather of a full_table(): every rank's block to every rank."""
    world = dist.get_world_size(group) if dist is not None and dist.is_initialized() else 1
    if world == 1:
        return full
    rank = dist.get_rank(group)
    blk = full.shape[0] // world
    dist.all_gather_into_tensor(full, full[rank * blk:(rank + 1) * blk], group=group)
    return full
