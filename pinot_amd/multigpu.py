"""Multi-GPU layer of the segment query path: one process per GPU, segments sharded over ranks, and ONE
exchange step, the merge of the per-GPU partials, over torch.distributed (backend "nccl" = RCCL over xGMI on the GPU
box, "gloo" in the CPU tests).

Replaces the reference's cross-segment combine (operator/MCombineOperator.java:84-199,
operator/MCombineGroupByOperator.java:139-233) for partials that live on different GPUs:
  * aggregation-only: COUNT/SUM/AVG add, MIN/MAX take min/max (query/aggregation/function/*.combineTwoValues);
  * dense group-by: every rank holds the same dense table layout (pgx_query_dense_slots / pgx_query_dense_plane_op:
    plane 0 = int64 doc count, then one plane per function: 0 int64 add, 1 double add, 2 ordered-u64 min,
    3 ordered-u64 max) -> one all-reduce per plane kind, min/max on sign-flipped ordered encodings.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

PLANE_ADD_I64, PLANE_ADD_F64, PLANE_MIN_ORD, PLANE_MAX_ORD = range(4)
SIGN64 = -(1 << 63)


def shard(num_segments: int, world: int, rank: int, scaling: str) -> List[int]:
    """Segment ids of this rank.  "weak": every rank holds its own `num_segments` segments (fixed work per GPU);
    "strong": the global segment list is dealt round-robin (segment i -> GPU i mod world)."""
    if scaling == "weak":
        return [rank * num_segments + i for i in range(num_segments)]
    return list(range(rank, num_segments, world))


def merge_dense_planes(t, plane_ops: Sequence[int]) -> None:
    """In-place all-reduce of a dense partial group table `t` (int64 tensor, len(plane_ops) planes x slots)."""
    import torch
    import torch.distributed as dist
    nplanes = len(plane_ops)
    planes = t.view(nplanes, -1)
    adds = [p for p, op in enumerate(plane_ops) if op == PLANE_ADD_I64]
    if adds:
        if len(adds) == nplanes:
            dist.all_reduce(t)
        else:
            lo = 0
            while lo < len(adds):  # contiguous runs of int64-add planes go in one collective
                hi = lo
                while hi + 1 < len(adds) and adds[hi + 1] == adds[hi] + 1:
                    hi += 1
                dist.all_reduce(planes[adds[lo]:adds[hi] + 1])
                lo = hi + 1
    for p, op in enumerate(plane_ops):
        if op == PLANE_ADD_F64:
            x = planes[p].view(torch.float64).clone()
            dist.all_reduce(x)
            planes[p].copy_(x.view(torch.int64))
        elif op in (PLANE_MIN_ORD, PLANE_MAX_ORD):
            x = planes[p] ^ SIGN64  # ordered-unsigned -> ordered-signed
            dist.all_reduce(x, op=dist.ReduceOp.MIN if op == PLANE_MIN_ORD else dist.ReduceOp.MAX)
            planes[p].copy_(x ^ SIGN64)


def merge_aggregation(fns: Sequence[str], values: Sequence[Tuple[float, int]], device=None) -> List[Tuple[float, int]]:
    """Merge aggregation-only partials (value, count) per function across ranks: ONE all-reduce (sum) carries every
    count and every SUM/AVG value (doubles: counts are exact below 2^53); MIN and MAX get one collective each only
    when the query has them (they are latency-bound 8-byte messages on xGMI)."""
    import torch
    import torch.distributed as dist
    adds = [float(x[1]) for x in values] + [float(x[0]) for f, x in zip(fns, values) if f in ("count", "sum", "avg")]
    t = torch.tensor(adds, dtype=torch.float64, device=device)
    dist.all_reduce(t)
    counts = [int(v) for v in t[:len(fns)].tolist()]
    sums = iter(t[len(fns):].tolist())
    out = [None] * len(fns)
    for i, f in enumerate(fns):
        if f in ("count", "sum", "avg"):
            out[i] = (next(sums), counts[i])
    for f, op in (("min", dist.ReduceOp.MIN), ("max", dist.ReduceOp.MAX)):
        idx = [i for i, g in enumerate(fns) if g == f]
        if idx:
            m = torch.tensor([values[i][0] for i in idx], dtype=torch.float64, device=device)
            dist.all_reduce(m, op=op)
            for i, v in zip(idx, m.tolist()):
                out[i] = (v, counts[i])
    return out
