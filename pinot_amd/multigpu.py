"""Multi-GPU layer of the segment query path: one process per GPU, segments sharded over ranks, and ONE
exchange step, the merge of the per-GPU partials, over torch.distributed (backend "nccl" = RCCL over xGMI on the GPU
box, "gloo" in the CPU tests).

Replaces the reference's cross-segment combine (operator/MCombineOperator.java:84-199,
operator/MCombineGroupByOperator.java:139-233) for partials that live on different GPUs:
  * aggregation-only: COUNT/SUM/AVG add, MIN/MAX take min/max (query/aggregation/function/*.combineTwoValues);
  * dense group-by: every rank holds the same dense table layout (pgx_query_dense_slots / pgx_query_dense_plane_op:
    plane 0 = int64 doc count, then one plane per function: 0 int64 add, 1 double add, 2 ordered-u64 min,
    3 ordered-u64 max) -> one all-reduce per plane kind, min/max on sign-flipped ordered encodings;
  * sparse group-by (key spaces too wide for a dense table): groups routed by packed key to an owner rank with one
    all-to-all and merged on its device (device_sparse_merge); ranks whose results are not device-resident fall back to
    gathering groups to rank 0 by key value (gather_group_partials / merge_group_partials / trim_to_size).
Key identity across processes: union_key_domains (one key space per group-by column over every rank's dictionaries).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np

PLANE_ADD_I64, PLANE_ADD_F64, PLANE_MIN_ORD, PLANE_MAX_ORD = range(4)
SIGN64 = -(1 << 63)


def shard(num_segments: int, world: int, rank: int, scaling: str) -> List[int]:
    """Segment ids of this rank.  "weak": every rank holds its own `num_segments` segments (fixed work per GPU);
    "strong": the global segment list is dealt round-robin (segment i -> GPU i mod world)."""
    if scaling == "weak":
        return [rank * num_segments + i for i in range(num_segments)]
    return list(range(rank, num_segments, world))


def _fingerprint(dt, u) -> int:
    """63-bit fingerprint of one column's sorted distinct values (and their type)."""
    import hashlib
    h = hashlib.blake2b(digest_size=8)
    h.update(str(dt).encode())
    if dt == "STRING":
        for v in u:
            b = v.encode("utf-8")
            h.update(len(b).to_bytes(4, "little"))
            h.update(b)
    elif u is not None:
        h.update(np.ascontiguousarray(u).tobytes())
    return int.from_bytes(h.digest(), "little") >> 1


def _local_domain(segments, col):
    """(data type, sorted distinct values) of one group column over this rank's segments' dictionaries."""
    infos = [s.column(col) for s in segments]
    dt = infos[0].meta.data_type if infos else None
    if dt == "STRING":
        return dt, sorted({str(v) for i in infos for v in i.values}, key=lambda v: v.encode("utf-8"))
    if dt is None:
        return None, None
    kind = np.float64 if dt in ("FLOAT", "DOUBLE") else np.int64
    return dt, np.unique(np.concatenate([np.asarray(i.values, dtype=kind) for i in infos]))


def _gather_bytes(payload: bytes, device) -> List[bytes]:
    """all_gather of one variable-length byte string per rank as tensors (lengths first, then a padded uint8 tensor)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size()
    n = torch.tensor([len(payload)], dtype=torch.int64, device=device)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n)
    lens = [int(x.item()) for x in ns]
    cap = max(1, max(lens))
    buf = torch.zeros(cap, dtype=torch.uint8, device=device)
    if payload:
        buf[:len(payload)] = torch.frombuffer(bytearray(payload), dtype=torch.uint8).to(device)
    bufs = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(bufs, buf)
    return [bytes(b[:k].cpu().numpy().tobytes()) for b, k in zip(bufs, lens)]


_DOMAINS = None  # OrderedDict: this rank's local key -> (global fingerprint, [(data type, values)] of the union)
_DOMAINS_CAP = 32


def _h63(obj) -> int:
    import hashlib
    return int.from_bytes(hashlib.blake2b(repr(obj).encode(), digest_size=8).digest(), "little") >> 1


def _domain_cache_probe(local_key, device):
    """Collective hit-or-miss decision of the union-domain cache.  Every rank all-gathers (hash of its local key, the
    global fingerprint stored with its cached entry or -1).  The union depends on EVERY rank's segments, so an entry is
    used only when every rank holds one, all of them were stored under the same global fingerprint, and that
    fingerprint equals the hash of the local keys gathered now.  The decision is a function of the gathered tensor
    alone, so every rank takes the same branch and the collectives of the miss path stay in step (a rank whose segment
    set changed while another's did not makes every rank recompute).  Returns (entry or None, global fingerprint)."""
    import collections

    import torch
    import torch.distributed as dist
    global _DOMAINS
    if _DOMAINS is None:
        _DOMAINS = collections.OrderedDict()
    h = _h63(local_key)
    ent = _DOMAINS.get(local_key)
    mine = torch.tensor([h, ent[0] if ent is not None else -1], dtype=torch.int64, device=device)
    parts = [torch.zeros_like(mine) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, mine)
    rows = [tuple(int(v) for v in p.tolist()) for p in parts]
    g = _h63(tuple(r[0] for r in rows))
    hit = all(r[1] == g for r in rows)
    if hit:
        _DOMAINS.move_to_end(local_key)
        return ent[1], g
    return None, g


def _domain_cache_store(local_key, g, dom) -> None:
    _DOMAINS[local_key] = (g, dom)
    _DOMAINS.move_to_end(local_key)
    while len(_DOMAINS) > _DOMAINS_CAP:  # LRU bound: realtime snapshots get new uids every query
        _DOMAINS.popitem(last=False)


def union_key_domains(q, segments, device=None) -> None:
    """Cross-process key identity ("a host-side global dictionary per group-by column"): every rank
    contributes the distinct values of each group-by column over its segments' dictionaries, all ranks build the same
    sorted union, and the query plans its keys over it (pgx_query_set_key_domain).  Dense slots and packed sparse keys
    then mean the same group on every GPU whatever dictionaries the ranks hold, so the partials merge by slot (RCCL
    all-reduce) or by packed key (all-to-all + device merge) -- the value-keyed combine of
    MCombineGroupByOperator.java:166-191 without moving values.

    Cached per (group columns, every rank's segment set): one all-gather of 16 bytes per rank decides, on every rank
    alike, whether the cached union still holds (_domain_cache_probe).  On a miss: two all-reduces of per-column
    fingerprints (MIN, MAX); columns whose dictionaries are the same on every rank (the common case: one table, one
    schema, shared value domains) need no exchange at all; only the others all-gather their values as byte tensors
    (`device`: the process group's device, e.g. cuda:N under RCCL; None: CPU, gloo)."""
    import torch
    import torch.distributed as dist
    key = (tuple(q.group_cols), tuple(getattr(s, "uid", id(s)) for s in segments), dist.get_world_size())
    dom, gfp = _domain_cache_probe(key, device)
    if dom is None:
        local = [_local_domain(segments, col) for col in q.group_cols]
        fp = torch.tensor([_fingerprint(dt, u) for dt, u in local], dtype=torch.int64, device=device)
        lo, hi = fp.clone(), fp.clone()
        if len(local):
            dist.all_reduce(lo, op=dist.ReduceOp.MIN)
            dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        dom = []
        for g, (dt, u) in enumerate(local):
            if dt is not None and int(lo[g]) == int(hi[g]):
                dom.append((dt, u))
                continue
            if dt == "STRING":  # length-prefixed UTF-8 values
                payload = b"S" + b"".join(len(b).to_bytes(4, "little") + b for b in (v.encode("utf-8") for v in u))
            elif dt is None:
                payload = b""
            else:
                payload = dt.encode() + b"\0" + np.ascontiguousarray(u).tobytes()
            parts = _gather_bytes(payload, device)
            dts, vals = set(), []
            for p in parts:
                if not p:
                    continue
                if p[:1] == b"S":
                    dts.add("STRING")
                    i = 1
                    while i < len(p):
                        k = int.from_bytes(p[i:i + 4], "little")
                        vals.append(p[i + 4:i + 4 + k].decode("utf-8"))
                        i += 4 + k
                else:
                    t, raw = p.split(b"\0", 1)
                    dts.add(t.decode())
                    vals.append(np.frombuffer(raw, dtype=np.float64 if t in (b"FLOAT", b"DOUBLE") else np.int64))
            if not dts:  # no rank holds a segment with this column
                dom.append((None, None))
                continue
            if len(dts) != 1:
                raise ValueError("group column %s has different types across ranks: %s" % (q.group_cols[g], dts))
            t = dts.pop()
            if t == "STRING":
                dom.append((t, sorted(set(vals), key=lambda v: v.encode("utf-8"))))
            else:
                dom.append((t, np.unique(np.concatenate(vals))))
        _domain_cache_store(key, gfp, dom)
    for g, (dt, vals) in enumerate(dom):
        if dt is not None:
            q.set_key_domain(g, vals, dt)


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
    adding = ("count", "sum", "avg", "countmv", "summv", "avgmv")
    adds = [float(x[1]) for x in values] + [float(x[0]) for f, x in zip(fns, values) if f in adding]
    t = torch.tensor(adds, dtype=torch.float64, device=device)
    dist.all_reduce(t)
    counts = [int(v) for v in t[:len(fns)].tolist()]
    sums = iter(t[len(fns):].tolist())
    out = [None] * len(fns)
    for i, f in enumerate(fns):
        if f in adding:
            out[i] = (next(sums), counts[i])
    for f, op in (("min", dist.ReduceOp.MIN), ("max", dist.ReduceOp.MAX)):
        idx = [i for i, g in enumerate(fns) if g in (f, f + "mv")]  # MINMV / MAXMV combine like MIN / MAX
        if idx:
            m = torch.tensor([values[i][0] for i in idx], dtype=torch.float64, device=device)
            dist.all_reduce(m, op=op)
            for i, v in zip(idx, m.tolist()):
                out[i] = (v, counts[i])
    return out


# ------------------------------------------------------------------------------------------------
# Sparse (high-cardinality) group-by partials across GPUs ("hipMemcpy to host with a host hash-merge"):
# every rank compacts its groups to (key values per group column, one (value, count) pair per function), rank 0 gathers
# them, merges equal keys with the combine semantics of query/aggregation/function/*.combineTwoValues
# (CountAggregationFunction.java:79-87 long add, SumAggregationFunction.java:168-176 double add, Min/Max extremes,
# AvgAggregationFunction.java:116-125 pair add) and applies AggregationGroupByOperatorService.trimToSize
# (query/aggregation/groupby/AggregationGroupByOperatorService.java:59-77,284-361) to the merged groups.
# Keys are the group columns' VALUES, not dictIds: the segments of different GPUs have their own dictionaries, and the
# reference's combine is keyed by the value string (MCombineGroupByOperator.java:139-233).
# ------------------------------------------------------------------------------------------------
def gather_group_partials(key_cols, vals, cnts, root: int = 0):
    """Gather every rank's partial (key_cols: list of 1-D arrays, vals: float64 [nf, n], cnts: int64 [nf, n]) to
    `root`.  Returns the list of per-rank partials on the root, None elsewhere."""
    import torch.distributed as dist
    mine = ([np.ascontiguousarray(k) for k in key_cols], np.ascontiguousarray(vals), np.ascontiguousarray(cnts))
    world = dist.get_world_size()
    out = [None] * world if dist.get_rank() == root else None
    dist.gather_object(mine, out, dst=root)
    return out


def merge_group_partials(fns: Sequence[str], parts):
    """Merge partials with equal keys (sort-based: lexsort over the key columns, then reduceat per function).  Returns
    (key_cols, vals, cnts) with one row per distinct key, keys in ascending order."""
    parts = [p for p in parts if p is not None and len(p[0]) and len(p[0][0])]
    nf = len(fns)
    if not parts:
        return [], np.zeros((nf, 0)), np.zeros((nf, 0), dtype=np.int64)
    ncols = len(parts[0][0])
    cols = [np.concatenate([p[0][c] for p in parts]) for c in range(ncols)]
    vals = np.concatenate([p[1] for p in parts], axis=1)
    cnts = np.concatenate([p[2] for p in parts], axis=1)
    order = np.lexsort(tuple(reversed(cols)))  # lexsort: the LAST key is primary
    cols = [c[order] for c in cols]
    vals, cnts = vals[:, order], cnts[:, order]
    n = len(order)
    change = np.zeros(n, dtype=bool)
    change[0] = True
    for c in cols:
        change[1:] |= c[1:] != c[:-1]
    starts = np.flatnonzero(change)
    out_v = np.empty((nf, len(starts)))
    out_c = np.add.reduceat(cnts, starts, axis=1)
    for i, f in enumerate(fns):
        if f in ("min", "minmv"):  # MinMVAggregationFunction.combineTwoValues: Math.min
            out_v[i] = np.minimum.reduceat(vals[i], starts)
        elif f in ("max", "maxmv"):
            out_v[i] = np.maximum.reduceat(vals[i], starts)
        else:  # count (value unused), sum, avg and their MV forms: add
            out_v[i] = np.add.reduceat(vals[i], starts)
    return [c[starts] for c in cols], out_v, out_c


def trim_to_size(fns: Sequence[str], vals, cnts, top_n: int, total: int = None) -> List[np.ndarray]:
    """AggregationGroupByOperatorService.trimToSize over merged groups: above 20 x max(topN, 1000) groups keep, per
    function, the 5 x max(topN, 1000) best (MIN ascending, others descending, AVG by sum / count); otherwise every
    group.  Ties at the threshold are arbitrary, as in the reference's MinMaxPriorityQueue.  `total` is the number of
    merged groups the threshold applies to when `vals` holds only candidates (the per-rank trims of disjoint key
    partitions).  Returns the kept group indices per function."""
    n = vals.shape[1]
    min_trim = max(top_n, 1000)
    threshold, size = min_trim * 20, min_trim * 5
    total = n if total is None else total
    out = []
    for i, f in enumerate(fns):
        if total <= threshold or n <= size:
            out.append(np.arange(n))
            continue
        if f in ("count", "countmv"):
            score = cnts[i].astype(np.float64)
        elif f in ("avg", "avgmv"):
            c = cnts[i].astype(np.float64)
            score = np.divide(vals[i], c, out=np.zeros(n), where=c != 0)
        else:
            score = vals[i]
        if f not in ("min", "minmv"):
            score = -score
        out.append(np.argpartition(score, size - 1)[:size])
    return out


# ------------------------------------------------------------------------------------------------
# Device-side sparse merge (ranks planned the same key space: identical dictionaries, union_key_domains' fingerprint
# check).  Every rank's groups stay in HBM as records of 1 + planes words (packed key, count, then sum, min, max per value
# column: pgx_result_device_groups / pgx_result_record_words; f64 sums of FLOAT / DOUBLE columns merge as f64),
# are routed to rank hash(key) mod world with ONE all_to_all_single (RCCL send/recv over xGMI), merged there by the
# library's device hash merge (pgx_result_merge_groups), trimmed on the device (pgx_result_trim: the key partitions are
# disjoint, so the union of the per-partition top-K holds the global top-K), and only the kept groups -- as VALUES --
# go to rank 0, which applies trimToSize once more with the global group count.
# ------------------------------------------------------------------------------------------------
_GOLDEN = -7046029254386353131  # 0x9E3779B97F4A7C15 as a signed 64-bit constant


def group_destination(keys, world: int):
    """Destination rank of each packed group key: high bits of a multiplicative hash (identical on every rank)."""
    return ((keys * _GOLDEN) >> 40) % world


def _all_to_all(out, inp, out_splits, in_splits):
    import torch.distributed as dist
    if dist.get_backend() == "gloo" and inp.is_cuda:  # gloo rehearsal on a 1-GPU box: exchange through host memory
        o = out.cpu()
        dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits)
        out.copy_(o)
    else:
        dist.all_to_all_single(out, inp, out_splits, in_splits)


def exchange_group_records(recs, world: int):
    """all_to_all of [n, W] int64 group records by destination rank: returns this rank's [m, W] records."""
    import torch
    import torch.distributed as dist
    dest = group_destination(recs[:, 0], world)
    order = torch.argsort(dest, stable=True)
    recs = recs[order]
    send = torch.bincount(dest, minlength=world).to(torch.int64)
    recv = torch.empty_like(send)
    if dist.get_backend() == "gloo" and send.is_cuda:
        r = recv.cpu()
        dist.all_to_all_single(r, send.cpu())
        recv.copy_(r)
    else:
        dist.all_to_all_single(recv, send)
    in_splits, out_splits = send.tolist(), recv.tolist()
    out = torch.empty((sum(out_splits), recs.shape[1]), dtype=torch.int64, device=recs.device)
    _all_to_all(out, recs, out_splits, in_splits)
    return out


def device_sparse_merge(ctx, q, r, segments, device):
    """Merge a device-resident sparse group-by result across ranks (see above).  Returns (maps, total_groups, stats):
    on rank 0 one {rendered key: value} map per function after trimToSize (None elsewhere)."""
    import ctypes as C

    import torch
    import torch.distributed as dist

    from pinot_amd import engine as E
    from pinot_amd import native as N
    L = N.lib()
    world = dist.get_world_size()
    n = C.c_int64()
    w = C.c_int32()
    N.check(L.pgx_result_device_groups(r, C.byref(n), None))
    N.check(L.pgx_result_record_words(r, C.byref(w)))
    recs = torch.empty((max(n.value, 1), w.value), dtype=torch.int64, device=device)
    N.check(L.pgx_result_device_groups(r, C.byref(n), C.c_void_p(recs.data_ptr())))
    mine = exchange_group_records(recs[:n.value], world)
    st = (C.c_int64 * 4)()
    N.check(L.pgx_result_stats(r, st))
    stats = torch.tensor(list(st), dtype=torch.int64, device=device)
    dist.all_reduce(stats)
    s4 = (C.c_int64 * 4)(*stats.tolist())
    merged = C.c_void_p()
    torch.cuda.synchronize(device)
    N.check(L.pgx_result_merge_groups(ctx.handle, r, C.c_void_p(mine.data_ptr()), mine.shape[0], s4,
                                      C.byref(merged)))
    try:
        ng = C.c_int64()
        N.check(L.pgx_result_num_groups(merged, C.byref(ng)))
        total = torch.tensor([ng.value], dtype=torch.int64, device=device)
        dist.all_reduce(total)
        # union over the functions of the device trim's kept groups, then every function's value of each
        nf, ncols = len(q.fns), len(q.group_cols)
        idx = set()
        for i in range(nf):
            cap = C.c_int64(0)
            N.check(L.pgx_result_trim(merged, i, None, C.byref(cap)))
            sel = np.zeros(max(cap.value, 1), dtype=np.int64)
            N.check(L.pgx_result_trim(merged, i, sel.ctypes.data, C.byref(cap)))
            idx.update(sel[:cap.value].tolist())
        idx = np.array(sorted(idx), dtype=np.int64)
        m = len(idx)
        si = np.zeros(max(m * ncols, 1), dtype=np.int32)
        di = np.zeros(max(m * ncols, 1), dtype=np.int32)
        v = np.zeros(max(m * nf, 1))
        c = np.zeros(max(m * nf, 1), dtype=np.int64)
        N.check(L.pgx_result_gather(merged, idx.ctypes.data, m, si.ctypes.data, di.ctypes.data, v.ctypes.data,
                                    c.ctypes.data))
    finally:
        L.pgx_result_release(merged)
    fns = q.fns
    si, di = si[:m * ncols].reshape(ncols, m), di[:m * ncols].reshape(ncols, m)
    cols = [E._column_values(segments, col, si[g], di[g], q.domains.get(g)) for g, col in enumerate(q.group_cols)]
    vals, cnts = v[:m * nf].reshape(nf, m), c[:m * nf].reshape(nf, m)
    parts = gather_group_partials(cols, vals, cnts)  # kept groups only, as key values
    if dist.get_rank() != 0:
        return None, int(total.item()), list(s4)
    cols, vals, cnts = merge_group_partials(fns, parts)  # partitions are disjoint: this only concatenates
    keep = trim_to_size(fns, vals, cnts, q.request["group_by"].get("top_n", 10), total=int(total.item()))
    return E.render_group_maps(q, segments, cols, vals, cnts, keep), int(total.item()), list(s4)
