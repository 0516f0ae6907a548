"""Multi-GPU sharding of source rows (one process per GPU, torch.distributed).

Source rows are independent.  The seeded plan (engine shd_route_plan_create)
assigns each rank whole subtrees of the seed forest, with the heavy top levels replicated
as helper rows (shard_range keeps the plain contiguous split for unplanned launches).  The
exchange steps are the runahead minimum (all-reduce MIN of one double) and, where a
device-resident full table is needed, an all-gather of the rows' upper triangles (RCCL
over xGMI with backend "nccl"; gloo on CPU for tests).
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


# ---- reduced table-assembly payload (upper triangles, u16 latency) -------------------
# The Path cache needs each unordered pair once (topology.c:1307-1336: the first writer
# stores both directions), so a rank sends only the upper triangle of its rows: row of
# attached position i keeps targets j >= i.  Segments are packed per rank in plan row
# order; the gathered buffer holds rank k's segment at k * seg (seg = the largest rank's
# element count).  Latency goes as u16 where exact (integer latencies below 65535 ms),
# reliability as f64: 10 B per triangle pair against 16 B per square pair.

def tri_offsets(pos, na: int):
    """int64 element offsets of each row's triangle segment (row of position p holds
    na - p entries), and the total."""
    import numpy as np
    pos = np.asarray(pos, np.int64)
    ln = na - pos
    off = np.zeros(len(pos) + 1, np.int64)
    np.cumsum(ln, out=off[1:])
    return off, int(off[-1])


class TriangleIndex:
    """Where pair (i, j), i <= j, of the attached list lives in the gathered payload:
    every rank's row positions in its plan order (all_gather'ed), one lookup table."""

    def __init__(self, pos_by_rank, na: int, seg: int):
        import numpy as np
        self.na, self.seg = na, seg
        self.rank_of = np.full(na, -1, np.int32)
        self.start = np.zeros(na, np.int64)  # element index of row i's segment
        for k, pos in enumerate(pos_by_rank):
            off, _ = tri_offsets(pos, na)
            pos = np.asarray(pos, np.int64)
            self.rank_of[pos] = k
            self.start[pos] = k * seg + off[:-1]

    def index(self, i, j):
        """element index of pair (i, j) (either order)."""
        import numpy as np
        i, j = np.minimum(i, j), np.maximum(i, j)
        return self.start[i] + (j - i)


LAT16_NONE = 0xFFFF  # u16 payload code of a NaN latency (no latency takes it: info["lat16"])


def decode_lat16(x):
    """u16 payload latencies back to the f64 table values: exact integers, 0xFFFF -> NaN."""
    import numpy as np
    x = np.asarray(x).view(np.uint16) if np.asarray(x).dtype == np.int16 else np.asarray(x, np.uint16)
    out = x.astype(np.float64)
    out[x == LAT16_NONE] = np.nan
    return out


def pack_triangle_host(lat_rows, rel_rows, pos, na: int, lat16: bool = True):
    """Host statement of shd_route_tri_payload_async (tests): the rows' triangles in row
    order, latency as u16 (NaN -> 0xFFFF) or f64."""
    import numpy as np
    off, tot = tri_offsets(pos, na)
    L = np.empty(tot, np.uint16 if lat16 else np.float64)
    R = np.empty(tot, np.float64)
    for r, p in enumerate(pos):
        seg = lat_rows[r, p:na]
        L[off[r]:off[r + 1]] = np.where(np.isnan(seg), LAT16_NONE, seg).astype(np.uint16) if lat16 else seg
        R[off[r]:off[r + 1]] = rel_rows[r, p:na]
    return L, R


def allgather_payload(lat_seg, rel_seg, seg: int, dist, group=None):
    """All-gather every rank's packed segment (padded to `seg` elements) into
    [world * seg] latency and reliability buffers (RCCL over xGMI with nccl)."""
    import torch
    world = dist.get_world_size(group)
    def pad(x):
        if x.numel() == seg:
            return x
        y = torch.empty(seg, dtype=x.dtype, device=x.device)
        y[: x.numel()] = x
        return y
    out_l = torch.empty(world * seg, dtype=lat_seg.dtype, device=lat_seg.device)
    out_r = torch.empty(world * seg, dtype=rel_seg.dtype, device=rel_seg.device)
    # u16 latencies travel as bytes (gloo has no 16-bit integer type)
    byt = lambda t: t.view(torch.uint8) if t.element_size() == 2 else t
    dist.all_gather_into_tensor(byt(out_l), byt(pad(lat_seg)), group=group)
    dist.all_gather_into_tensor(out_r, pad(rel_seg), group=group)
    return out_l, out_r


# ---- landmark rows of a multi-GPU landmark-only plan --------------------------------
# A landmark-only plan (C3-class graphs) seeds every row from its nearest landmark rows (the
# highest-degree vertices' exact rows).  Each rank computes an equal share of them
# (RoutePlan.refresh_async(what=REFRESH_MINE)) and the shares are all-gathered into every
# rank's store (u16 distances + u32 parent records per vertex, ~6 B x n per landmark: 57 MB
# for C3's 1024), instead of every rank computing all of them.

def bind_landmark_store(plan, world: int, device):
    """Caller-owned store tensors for `plan` (padded to world equal shares), bound to the plan
    (RoutePlan.bind_store): the buffers the all-gather writes.  None when the plan has no
    landmark store (not landmark-only, or built on the host)."""
    import torch
    lm = plan.landmarks()
    if lm is None:
        return None
    cnt = -(-lm["nland"] // world)
    drow = torch.empty((cnt * world, lm["row_stride"]), dtype=torch.int16, device=device)
    prow = torch.empty((cnt * world, lm["row_stride"]), dtype=torch.int32, device=device)
    plan.bind_store(drow, prow)
    return {"drow": drow, "prow": prow, "share": cnt, **lm}


def exchange_landmarks(store, dist, group=None):
    """All-gather every rank's share of the landmark rows into every rank's store (in place:
    RCCL all_gather_into_tensor over xGMI for nccl; staged through host memory for gloo,
    whose all-gather takes CPU tensors only).  Shares are equal (the store is padded)."""
    world = dist.get_world_size(group) if dist is not None and dist.is_initialized() else 1
    if world == 1 or store is None:
        return
    rank = dist.get_rank(group)
    cnt = store["share"]
    # (as bytes: neither RCCL nor gloo takes int16 tensors; a row of the store stays a row)
    import torch
    for buf in (store["drow"].view(torch.uint8), store["prow"].view(torch.uint8)):
        mine = buf[rank * cnt:(rank + 1) * cnt]
        if dist.get_backend(group) == "nccl":
            dist.all_gather_into_tensor(buf, mine, group=group)
        else:
            outs = [buf[k * cnt:(k + 1) * cnt].cpu() for k in range(world)]
            dist.all_gather(outs, mine.cpu().contiguous(), group=group)
            for k in range(world):
                if k != rank:
                    buf[k * cnt:(k + 1) * cnt].copy_(outs[k])


def landmark_exchange_bytes(store, world: int) -> int:
    """Bytes each rank receives in exchange_landmarks (the other ranks' shares)."""
    if store is None or world <= 1:
        return 0
    return (world - 1) * store["share"] * store["row_stride"] * 6
