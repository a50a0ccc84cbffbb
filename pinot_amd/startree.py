"""Star-tree index builder (segment creation side of SURVEY 8a row a-18), writing the reference's OFF_HEAP format.

Restates core/startree/OffHeapStarTreeBuilder.java (paths relative to pinot-core/src/main/java/com/linkedin/pinot/):
  * default split order = dimensions by cardinality, descending, stable (computeDefaultSplitOrder, :535-555);
  * raw records sorted by the split order then the remaining dimensions (getSortOrder, :585-601);
  * constructStarTree (:620-711): per level, one child per value of the split dimension; a child whose range holds
    more than maxLeafRecords docs is split further; then a STAR child whose docs are the unique combinations of the
    range with the split dimension set to ALL (uniqueCombinations, :724-800: metrics summed), split further when
    rowsAdded >= maxLeafRecords;
  * createAggDocForAllNodes (:365-410): post-order, every node gets one aggregated doc (sum over its non-star
    children, or over its leaf range), dimension values = the node's path, ALL elsewhere;
and core/startree/StarTreeSerDe.java:183-328 for the OFF_HEAP bytes: header (magic, version, header size, dimension
name map, node count) then 7 x int32 per node in BFS order, children sorted by value (ALL = -1 first), native (LE)
byte order.

One deliberate difference: the reference builder sorts by its own first-seen value ids and re-maps the tree to segment
dictIds afterwards (segment/creator/impl/SegmentIndexCreationDriverImpl.java:291-347); here records are sorted by
segment dictIds directly.  That changes the order of docs inside a node's range, never which docs a node covers.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np

ALL = -1
MAGIC = 0xBADDA55B00DAD00D
VERSION = 1
DEFAULT_MAX_LEAF_RECORDS = 100000  # common/data/StarTreeIndexSpec.java:25-26
DEFAULT_SKIP_MATERIALIZATION_CARDINALITY = 10000  # StarTreeIndexSpec.DEFAULT_SKIP_MATERIALIZATION_CARDINALITY_THRESHOLD
SKIP_KEY = "star.tree.skip.materialization.for.dimensions"  # V1Constants.MetadataKeys.StarTree (:104-107)
SKIP_CARD_KEY = "star.tree.skip.materialization.cardinality"
INT_DEFAULT_NULL = -(1 << 31)      # FieldSpec default null for INT dimensions = the star value (:210-225)


@dataclass
class Node:
    dim: int
    value: int
    level: int
    start: int = -1
    end: int = -1
    agg: int = -1
    children: Optional[Dict[int, "Node"]] = None
    path: Dict[int, int] = field(default_factory=dict)


class _Table:
    """Record table grown by appends (star-node rows, aggregated docs): dims int32 (ALL = -1), metrics int64.  Kept as
    a list of contiguous blocks; every range the builder reads lies inside one block, so no re-concatenation."""

    def __init__(self, dims: np.ndarray, mets: np.ndarray):
        self.blocks = [(0, dims, mets)]
        self.starts = [0]  # block start rows, ascending (kept beside the blocks: no per-lookup rebuild)
        self.n = len(dims)

    def append(self, d: np.ndarray, m: np.ndarray) -> int:
        start = self.n
        self.blocks.append((start, d, m))
        self.starts.append(start)
        self.n += len(d)
        return start

    def rows(self, a, b):
        import bisect
        i = bisect.bisect_right(self.starts, a) - 1
        s0, d, m = self.blocks[i]
        assert b - s0 <= len(d), "range spans two blocks"
        return d[a - s0:b - s0], m[a - s0:b - s0]

    def all(self):
        return (np.concatenate([b[1] for b in self.blocks]), np.concatenate([b[2] for b in self.blocks]))


def _unique_ids(v: np.ndarray):
    """(sorted distinct values, index of each element's value): np.unique(v, return_inverse=True), through a presence
    table when the value range is small (integer columns of synthetic segments)."""
    v = np.asarray(v)
    if v.size and v.dtype.kind in "iu":
        lo, hi = int(v.min()), int(v.max())
        if hi - lo < (1 << 26):
            present = np.bincount((v - lo).astype(np.int64), minlength=hi - lo + 1) > 0
            lut = np.cumsum(present) - 1
            return np.flatnonzero(present).astype(np.int64) + lo, lut[v - lo]
        try:
            import pandas as pd  # hash-based factorisation: O(n) + a sort of the distinct values only
            codes, uniq = pd.factorize(v, sort=True)
            return np.asarray(uniq), codes.astype(np.int64)
        except ImportError:
            pass
    return np.unique(v, return_inverse=True)


def _lexsort(d: np.ndarray, order: Sequence[int]) -> np.ndarray:
    return np.lexsort(tuple(d[:, k] for k in reversed(order))) if len(d) else np.zeros(0, dtype=np.int64)


def build(dim_ids: np.ndarray, metrics: np.ndarray, cards: Sequence[int], max_leaf_records: int = DEFAULT_MAX_LEAF_RECORDS,
          split_order: Optional[Sequence[int]] = None, skip: Optional[Sequence[int]] = None,
          skip_cardinality: int = DEFAULT_SKIP_MATERIALIZATION_CARDINALITY, dense_limit: int = 1 << 22):
    """dim_ids: (N, D) int dictIds (no star values); metrics: (N, M) int64.
    Returns (tree_root, all_dims (T, D) with ALL=-1 for star, all_metrics (T, M), split_order, num_raw, skip).

    skipMaterializationForDimensions (OffHeapStarTreeBuilder.build :308-322): by default every dimension whose
    cardinality exceeds the threshold (computeDefaultDimensionsToSkipMaterialization :557-565); they leave the default
    split order, and the star-node rows hold ALL for them (uniqueCombinations :738-745).
    dense_limit: a range's distinct combinations are counted in a dense table when their key span is at most
    max(dense_limit, 2 x rows) (0: always sort; the output is the same either way)."""
    n, ndim = dim_ids.shape
    skip = set(skip) if skip else {k for k in range(ndim) if cards[k] > skip_cardinality}
    if split_order is None:
        split_order = [k for k in sorted(range(ndim), key=lambda k: -cards[k]) if k not in skip]  # stable
    else:
        skip -= set(split_order)
    sort_order = list(split_order) + [k for k in range(ndim) if k not in split_order]
    # one int64 sort key per row when the dims fit (ALL = -1 -> digit 0): a stable argsort of it orders rows exactly
    # as the lexicographic sort over sort_order, several times faster than np.lexsort
    radix = [int(dim_ids[:, k].max(initial=0)) + 2 for k in range(ndim)]
    span = 1
    for k in sort_order:
        span *= radix[k]

    def sort_key(d):
        key = np.zeros(len(d), dtype=np.int64)
        for k in sort_order:
            key = key * radix[k] + (d[:, k].astype(np.int64) + 1)
        return key

    def order_rows(d):
        if span < (1 << 62):
            key = sort_key(d)
            o = np.argsort(key, kind="stable")
            return o, key[o]
        return _lexsort(d, sort_order), None

    perm = order_rows(dim_ids)[0]
    tab = _Table(np.ascontiguousarray(dim_ids[perm]).astype(np.int32), np.ascontiguousarray(metrics[perm]).astype(np.int64))
    root = Node(ALL, ALL, 0)

    def unique_combinations(a, b, split_dim, dense_limit=dense_limit):
        d, m = tab.rows(a, b)
        d = d.copy()
        d[:, split_dim] = ALL
        for k in skip:
            d[:, k] = ALL
        if len(d) == 0:
            return d, m
        if span < (1 << 62):
            # the distinct sort keys of the range span few values (the prefix dims are constant): count them in a dense
            # table -- the same combinations in the same ascending-key order as sort + reduceat, in O(rows + span)
            key = sort_key(d)
            lo = int(key.min())
            width = int(key.max()) - lo + 1
            mabs = int(np.abs(m).max(initial=0))
            if dense_limit > 0 and width <= max(dense_limit, 2 * len(d)) and mabs * len(d) < (1 << 53):
                off = key - lo
                rep = np.empty(width, dtype=np.int64)
                rep[off] = np.arange(len(d))  # any row of a key: its dims are the combination
                present = np.flatnonzero(np.bincount(off, minlength=width))
                sums = np.stack([np.bincount(off, weights=m[:, j], minlength=width)[present]
                                 for j in range(m.shape[1])], axis=1) if m.shape[1] else np.zeros((len(present), 0))
                return d[rep[present]], np.rint(sums).astype(np.int64)
        o, key = order_rows(d)
        d, m = d[o], m[o]
        brk = np.ones(len(d), dtype=bool)
        brk[1:] = (key[1:] != key[:-1]) if key is not None else np.any(d[1:] != d[:-1], axis=1)
        starts = np.nonzero(brk)[0]
        return d[starts], np.add.reduceat(m, starts, axis=0)

    def construct(node: Node, a: int, b: int, level: int) -> int:
        if level == len(split_order):
            return 0
        sd = split_order[level]
        d, _ = tab.rows(a, b)
        col = d[:, sd]  # sorted within the range (its split_order prefix is constant): groups are contiguous runs
        first = np.concatenate([[0], np.flatnonzero(col[1:] != col[:-1]) + 1]) if len(col) else np.zeros(0, np.int64)
        vals = col[first]
        bounds = list(first) + [len(col)]
        node.children = {}
        added = 0
        for i, v in enumerate(vals.tolist()):
            child = Node(sd, int(v), node.level + 1, path={**node.path, sd: int(v)})
            node.children[int(v)] = child
            ca, cb = a + int(bounds[i]), a + int(bounds[i + 1])
            cdocs = 0
            if cb - ca > max_leaf_records:
                cdocs = construct(child, ca, cb, level + 1)
                added += cdocs
            if cdocs == 0:
                child.start, child.end = ca, cb
        star = Node(sd, ALL, node.level + 1, path=dict(node.path))
        node.children[ALL] = star
        ud, um = unique_combinations(a, b, sd)
        so = tab.append(ud, um)
        rows_added = len(ud)
        added += rows_added
        cdocs = 0
        if rows_added >= max_leaf_records:
            cdocs = construct(star, so, so + rows_added, level + 1)
            added += cdocs
        if cdocs == 0:
            star.start, star.end = so, so + rows_added
        return added

    construct(root, 0, n, 0)

    def agg_docs(node: Node) -> np.ndarray:
        if node.children is None:
            _, m = tab.rows(node.start, node.end)
            acc = m.sum(axis=0)
        else:
            acc = None
            for v, child in node.children.items():
                cm = agg_docs(child)
                if v == ALL:
                    continue  # the star child does not feed its parent's aggregate
                acc = cm.copy() if acc is None else acc + cm
        dims = np.full((1, ndim), ALL, dtype=np.int32)
        for k, v in node.path.items():
            dims[0, k] = v
        node.agg = tab.append(dims, acc.reshape(1, -1).astype(np.int64))
        return acc

    agg_docs(root)
    all_d, all_m = tab.all()
    return root, all_d, all_m, list(split_order), n, sorted(skip)


def serialize(root: Node, dim_names: Sequence[str]) -> bytes:
    """StarTreeSerDe.writeTreeOffHeapFormat: header + BFS nodes (7 x int32, native LE)."""
    nodes = []
    q = [root]
    while q:
        nodes.append(q.pop(0))
        ch = sorted((nodes[-1].children or {}).values(), key=lambda c: c.value)
        q.extend(ch)
    index = {id(x): i for i, x in enumerate(nodes)}
    names = b""
    for i, nm in enumerate(dim_names):
        e = nm.encode("utf-8")
        names += struct.pack("<ii", i, len(e)) + e
    header_size = 8 + 4 + 4 + 4 + len(names) + 4
    out = [struct.pack("<QiIi", MAGIC, VERSION, header_size, len(dim_names)), names, struct.pack("<i", len(nodes))]
    for x in nodes:
        ch = sorted((x.children or {}).values(), key=lambda c: c.value)
        cs = index[id(ch[0])] if ch else -1
        ce = index[id(ch[-1])] if ch else -1
        out.append(struct.pack("<7i", x.dim, x.value, x.start, x.end, x.agg, cs, ce))
    return b"".join(out)


def parse(buf: bytes):
    """StarTreeOffHeap.readHeader (core/startree/StarTreeOffHeap.java:95-150) -> (dim names by index, nodes array)."""
    magic, version, header_size, nd = struct.unpack_from("<QiIi", buf, 0)
    if magic != MAGIC:
        raise ValueError("not an OFF_HEAP star tree")
    pos = 20
    names = {}
    for _ in range(nd):
        i, ln = struct.unpack_from("<ii", buf, pos)
        names[i] = buf[pos + 8:pos + 8 + ln].decode("utf-8")
        pos += 8 + ln
    (nn,) = struct.unpack_from("<i", buf, pos)
    pos += 4
    nodes = np.frombuffer(buf, dtype="<i4", count=7 * nn, offset=pos).reshape(nn, 7)
    return names, nodes


def make_star_tree_segment(name: str, dims: Dict[str, np.ndarray], metrics: Dict[str, np.ndarray],
                           max_leaf_records: int = DEFAULT_MAX_LEAF_RECORDS, inverted: Sequence[str] = (),
                           skip_materialization: Optional[Sequence[str]] = None,
                           skip_cardinality: int = DEFAULT_SKIP_MATERIALIZATION_CARDINALITY, dense_limit: int = 1 << 22):
    """Build a v1 star-tree segment from raw INT dimension and metric values (SegmentIndexCreationDriverImpl.buildStarTree,
    :193-289): docs = raw docs in star-tree order, then the aggregated docs; star dimension values are the INT default
    null (Integer.MIN_VALUE), which therefore sits in every dimension dictionary."""
    from .segment import make_column, SegmentData
    dnames = list(dims)
    mnames = list(metrics)
    dicts, ids = [], []
    cards = []
    for k in dnames:
        v = np.asarray(dims[k], dtype=np.int64)
        dv, vid = _unique_ids(v)
        dicts.append(np.concatenate([[INT_DEFAULT_NULL], dv]) if (not len(dv) or dv[0] != INT_DEFAULT_NULL) else dv)
        ids.append(vid + (len(dicts[-1]) - len(dv)))  # the star value Integer.MIN_VALUE sorts first
        cards.append(len(dv))  # distinct dictIds present in the raw docs
    dim_ids = np.stack(ids, axis=1)
    mets = np.stack([np.asarray(metrics[k], dtype=np.int64) for k in mnames], axis=1)
    skip_idx = [dnames.index(k) for k in skip_materialization] if skip_materialization else None
    root, all_d, all_m, order, nraw, skipped = build(dim_ids, mets, cards, max_leaf_records, skip=skip_idx,
                                                     skip_cardinality=skip_cardinality, dense_limit=dense_limit)
    total = len(all_d)
    cols = []
    for i, k in enumerate(dnames):
        col_ids = all_d[:, i].astype(np.int64)
        col_ids[col_ids == ALL] = 0  # dictId of Integer.MIN_VALUE (smallest value)
        c = make_column(k, None, "INT", "DIMENSION", inverted=k in inverted, dictionary=dicts[i], dict_ids=col_ids)
        c.total_raw_docs = nraw
        cols.append(c)
    for j, k in enumerate(mnames):
        mv = all_m[:, j]
        md, mid = _unique_ids(mv)
        c = make_column(k, None, "INT" if md.max(initial=0) < (1 << 31) else "LONG", "METRIC", dictionary=md,
                        dict_ids=mid)
        c.total_raw_docs = nraw
        cols.append(c)
    seg = SegmentData(name, total, nraw, {c.name: c for c in cols})
    seg.star_tree = serialize(root, dnames)
    seg.metadata["startree.split.order"] = ",".join(dnames[k] for k in order)
    seg.metadata["startree.maxLeafRecords"] = str(max_leaf_records)
    seg.metadata[SKIP_CARD_KEY] = str(skip_cardinality)
    if skipped:
        seg.metadata[SKIP_KEY] = ",".join(dnames[k] for k in skipped)
    return seg
