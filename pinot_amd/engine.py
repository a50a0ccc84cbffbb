"""Host-side mirror of the reference's plan-maker / operator API over libpgx (the MI355X path).

Names and argument meaning follow pinot-core (paths relative to pinot-core/src/main/java/com/linkedin/pinot/core/):

  InstancePlanMakerImplV2.make_inner_segment_plan(segment, broker_request) -> PlanNode   (plan/maker/InstancePlanMakerImplV2.java:72-82)
  InstancePlanMakerImplV2.make_inter_segment_plan(segments, broker_request) -> Plan      (:93-109, plan/CombinePlanNode.java)
  PlanNode.run() -> Operator ; Operator.next_block() -> IntermediateResultsBlock          (plan/PlanNode.java:31, common/Operator.java:25-48)
  Operator.get_execution_statistics() -> ExecutionStatistics                              (operator/ExecutionStatistics.java:21-74)
  AggregationGroupByResult.get_group_key_iterator() / get_result_for_key(key, i)          (operator/aggregation/groupby/AggregationGroupByResult.java:56-113)

The per-segment predicate -> dictId resolution (a-4, operator/filter/predicate/*PredicateEvaluator.java) runs here on the
host, exactly where the Java caller would run its PredicateEvaluatorProvider before crossing the JNI boundary; every
doc-level step runs in the HIP kernel.  Unsupported shapes raise PgxError(PGX_ERR_UNSUPPORTED) so a caller can fall back
to the Java operators; nothing here computes results on the CPU.
"""
from __future__ import annotations

import ctypes as C
import itertools
import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import native as N
from .segment import Column, SegmentData

_DT = {"INT": N.PGX_INT, "LONG": N.PGX_LONG, "FLOAT": N.PGX_FLOAT, "DOUBLE": N.PGX_DOUBLE, "STRING": N.PGX_STRING}
_FN = {"count": N.PGX_COUNT, "sum": N.PGX_SUM, "min": N.PGX_MIN, "max": N.PGX_MAX, "avg": N.PGX_AVG,
       "countmv": N.PGX_COUNTMV, "summv": N.PGX_SUMMV, "minmv": N.PGX_MINMV, "maxmv": N.PGX_MAXMV, "avgmv": N.PGX_AVGMV}


# ------------------------------------------------------------------------------------------------
# Context / staged segments
# ------------------------------------------------------------------------------------------------
class Context:
    """One pgx_ctx bound to one HIP device (one process per GPU)."""

    def __init__(self, device: int = 0):
        L = N.lib()
        h = C.c_void_p()
        N.check(L.pgx_ctx_create(C.byref(N.CtxOpts(device, 0)), C.byref(h)))
        self.handle = h
        self.device = device

    def close(self):
        if self.handle:
            N.lib().pgx_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _java_double_str(x: float) -> str:
    """Double.toString formatting for FLOAT/DOUBLE group keys."""
    if x != x:
        return "NaN"
    if math.isinf(x):
        return "Infinity" if x > 0 else "-Infinity"
    if x == 0:
        return "-0.0" if math.copysign(1, x) < 0 else "0.0"
    a = abs(x)
    if 1e-3 <= a < 1e7:
        s = repr(float(x))
        if "e" in s or "E" in s:
            s = "%f" % x
        return s if "." in s else s + ".0"
    m, e = ("%.17e" % x).split("e")
    r = repr(float(x))
    digits = r.replace("-", "").replace(".", "").split("e")[0].lstrip("0") or "0"
    exp = int(e)
    mant = digits[0] + "." + (digits[1:].rstrip("0") or "0")
    return ("-" if x < 0 else "") + mant + "E" + str(exp)


@dataclass
class _ColInfo:
    meta: Column
    values: object  # numpy array (numeric) or list of str

    def index_of(self, raw: str) -> int:
        """Dictionary.indexOf: binary search, -(insertion point)-1 when absent (segment/index/readers/*Dictionary.java)."""
        dt = self.meta.data_type
        if dt == "STRING":
            width = self.meta.dict_width
            pad = self.meta.pad_char
            b = raw.encode("utf-8")
            key = raw if len(b) >= width else raw + pad * (width - len(b))
            padded = [v + pad * (width - len(v.encode("utf-8"))) for v in self.values]
            lo, hi = 0, len(padded)
            while lo < hi:
                mid = (lo + hi) // 2
                if padded[mid] < key:
                    lo = mid + 1
                else:
                    hi = mid
            return lo if lo < len(padded) and padded[lo] == key else -(lo + 1)
        if dt in ("INT", "LONG"):
            v = int(raw)  # Integer.parseInt / Long.parseLong semantics (raises on non-integers)
        elif dt == "FLOAT":
            v = float(np.float32(float(raw)))  # Float.parseFloat: the lookup is a float
        else:
            v = float(raw)
        arr = self.values
        pos = int(np.searchsorted(arr, v, side="left"))
        return pos if pos < len(arr) and arr[pos] == v else -(pos + 1)

    def string_of(self, dict_id: int) -> str:
        dt = self.meta.data_type
        v = self.values[dict_id]
        if dt == "STRING":
            return v
        if dt in ("INT", "LONG"):
            return str(int(v))
        if dt == "FLOAT":
            return _java_double_str(float(np.float32(v)))
        return _java_double_str(float(v))


STAR_SKIP_KEY = "star.tree.skip.materialization.for.dimensions"  # V1Constants.MetadataKeys.StarTree (:104-105)


def star_skip_dims(seg: SegmentData):
    """SegmentMetadataImpl reads the skip list as a PropertiesConfiguration list (comma separated, :345-355)."""
    v = (seg.metadata or {}).get(STAR_SKIP_KEY, "")
    return [x.strip() for x in v.split(",") if x.strip()]


_SEG_UID = itertools.count(1)


class IndexSegment:
    """A segment staged into HBM (Loaders.IndexSegment.load equivalent).  `uid` identifies the staged segment for the
    life of the process (caches keyed by segment sets: handles can be reused after a release)."""

    def __init__(self, ctx: Context, seg: SegmentData, device_buffers: Optional[Dict[str, int]] = None):
        self.uid = next(_SEG_UID)
        self.ctx = ctx
        self.data = seg
        self.name = seg.name
        self._cols: Dict[str, _ColInfo] = {}
        descs = (N.ColumnDesc * len(seg.columns))()
        keep = []
        for i, (name, c) in enumerate(seg.columns.items()):
            d = descs[i]
            nb = name.encode()
            keep.append(nb)
            d.name = nb
            d.data_type = _DT[c.data_type]
            d.cardinality = c.cardinality
            d.bits_per_element = c.bits
            d.is_sorted = int(c.is_sorted)
            d.dict_width = c.dict_width
            d.pad_char = ord(c.pad_char) if c.data_type == "STRING" else 0
            d.is_multi_value = int(c.is_mv)
            d.total_entries = c.total_entries
            for attr, data in (("fwd", c.fwd_bytes), ("sorted_pairs", c.sorted_bytes), ("dict", c.dict_bytes),
                               ("inv", c.inv_bytes)):
                if data is None:
                    setattr(d, attr, None)
                    continue
                buf = C.create_string_buffer(bytes(data), len(data))
                keep.append(buf)
                setattr(d, attr, C.cast(buf, C.c_void_p))
            d.fwd_len = len(c.fwd_bytes) if c.fwd_bytes is not None else 0
            d.sorted_len = len(c.sorted_bytes) if c.sorted_bytes is not None else 0
            d.dict_len = len(c.dict_bytes)
            d.inv_len = len(c.inv_bytes) if c.inv_bytes is not None else 0
        sd = N.SegmentDesc()
        sd.name = seg.name.encode()
        sd.total_docs = seg.total_docs
        sd.total_raw_docs = seg.total_raw_docs
        sd.num_columns = len(seg.columns)
        sd.columns = descs
        if seg.star_tree is not None:
            st = C.create_string_buffer(bytes(seg.star_tree), len(seg.star_tree))
            keep.append(st)
            sd.star_tree = C.cast(st, C.c_void_p)
            sd.star_tree_len = len(seg.star_tree)
        sd.mem = N.PGX_MEM_HOST
        skip = star_skip_dims(seg)
        if skip:
            arr = (C.c_char_p * len(skip))(*[x.encode() for x in skip])
            keep.append(arr)
            sd.num_star_skip_dims = len(skip)
            sd.star_skip_dims = arr
        h = C.c_void_p()
        N.check(N.lib().pgx_segment_stage(ctx.handle, C.byref(sd), C.byref(h)))
        self.handle = h
        del keep  # the library copied every host buffer during staging

    @classmethod
    def from_handle(cls, ctx: Context, seg: SegmentData, handle):
        """Wrap a segment the library staged itself (pgx_mutable_snapshot); `seg` carries the column metadata."""
        self = cls.__new__(cls)
        self.uid = next(_SEG_UID)
        self.ctx = ctx
        self.data = seg
        self.name = seg.name
        self._cols = {}
        self.handle = handle
        return self

    @classmethod
    def from_device(cls, ctx: Context, seg: SegmentData, fwd_device: Dict[str, int]):
        """Stage a segment whose forward indexes already live in HBM (synthetic benchmark data)."""
        self = cls.__new__(cls)
        self.uid = next(_SEG_UID)
        self.ctx = ctx
        self.data = seg
        self.name = seg.name
        self._cols = {}
        descs = (N.ColumnDesc * len(seg.columns))()
        keep = []
        dict_dev = []
        for i, (name, c) in enumerate(seg.columns.items()):
            d = descs[i]
            nb = name.encode()
            keep.append(nb)
            d.name = nb
            d.data_type = _DT[c.data_type]
            d.cardinality = c.cardinality
            d.bits_per_element = c.bits
            d.is_sorted = 0
            d.dict_width = c.dict_width
            d.fwd = C.c_void_p(fwd_device[name][0])
            d.fwd_len = fwd_device[name][1]
            p = C.c_void_p()
            N.check(N.lib().pgx_device_alloc(ctx.handle, len(c.dict_bytes), C.byref(p)))
            N.check(N.lib().pgx_copy_to_device(ctx.handle, p, c.dict_bytes, len(c.dict_bytes)))
            dict_dev.append(p)
            d.dict = p
            d.dict_len = len(c.dict_bytes)
            if c.inv_bytes is not None:  # inverted index bytes are host memory in either mode (pgx.h)
                ib = C.create_string_buffer(bytes(c.inv_bytes), len(c.inv_bytes))
                keep.append(ib)
                d.inv = C.cast(ib, C.c_void_p)
                d.inv_len = len(c.inv_bytes)
        sd = N.SegmentDesc()
        sd.name = seg.name.encode()
        sd.total_docs = seg.total_docs
        sd.total_raw_docs = seg.total_raw_docs
        sd.num_columns = len(seg.columns)
        sd.columns = descs
        sd.mem = N.PGX_MEM_DEVICE
        h = C.c_void_p()
        N.check(N.lib().pgx_segment_stage(ctx.handle, C.byref(sd), C.byref(h)))
        for p in dict_dev:
            N.lib().pgx_device_free(ctx.handle, p)
        self.handle = h
        return self

    def column(self, name: str) -> _ColInfo:
        if name not in self._cols:
            c = self.data.columns.get(name)
            if c is None:
                raise KeyError("segment %s has no column %s" % (self.name, name))
            vals = c.dictionary_values()
            if c.data_type != "STRING":
                vals = np.asarray(vals).astype(vals.dtype.newbyteorder("="))
            self._cols[name] = _ColInfo(c, vals)
        return self._cols[name]

    def device_bytes(self) -> int:
        v = C.c_uint64()
        N.check(N.lib().pgx_segment_device_bytes(self.handle, C.byref(v)))
        return v.value

    def destroy(self):
        if getattr(self, "handle", None):
            N.lib().pgx_segment_release(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


# ------------------------------------------------------------------------------------------------
# a-4: predicate -> dictId binding (PredicateEvaluatorProvider and the evaluators, operator/filter/predicate/)
# ------------------------------------------------------------------------------------------------
def _parse_range(rng: str):
    """RangePredicate (common/predicate/RangePredicate.java:31-57)."""
    s = rng.strip()
    a, b = s.split("\t\t")[0], s.split("\t\t")[1]
    lower, upper = a[1:], b[:-1]
    inc_lo = (lower == "*") if s.startswith("(") else True
    inc_hi = (upper == "*") if s.endswith(")") else True
    return lower, upper, inc_lo, inc_hi


def resolve_leaf(col: _ColInfo, leaf: dict):
    """Returns (lo, hi, words|None): docs match iff dictId in [lo,hi] (words None) or bit set in words."""
    card = col.meta.cardinality
    op = leaf["op"]
    if op == "RANGE":  # RangeOfflineDictionaryPredicateEvaluator.java:30-65
        lower, upper, inc_lo, inc_hi = _parse_range(leaf["values"][0])
        start = 0 if lower == "*" else col.index_of(lower)
        end = card - 1 if upper == "*" else col.index_of(upper)
        if start < 0:
            start = -(start + 1)
        elif not inc_lo and lower != "*":
            start += 1
        if end < 0:
            end = -(end + 1) - 1
        elif not inc_hi and upper != "*":
            end -= 1
        return (start, end, None) if end >= start else (0, -1, None)
    if op == "EQ":  # EqualsPredicateEvaluator.java:28-42
        i = col.index_of(leaf["values"][0])
        return (i, i, None) if i >= 0 else (0, -1, None)
    m = np.zeros(card, dtype=bool)
    if op == "IN":
        for v in leaf["values"]:
            i = col.index_of(v)
            if i >= 0:
                m[i] = True
    elif op in ("NEQ", "NOT_IN"):
        m[:] = True
        for v in leaf["values"]:
            i = col.index_of(v)
            if i >= 0:
                m[i] = False
    else:
        raise ValueError("unsupported predicate " + op)
    ids = np.nonzero(m)[0]
    if len(ids) == 0:
        return (0, -1, None)
    if ids[-1] - ids[0] + 1 == len(ids):
        return (int(ids[0]), int(ids[-1]), None)
    words = np.packbits(np.pad(m, (0, (-card) % 32)).reshape(-1, 32)[:, ::-1], axis=1,
                        bitorder="big").view(">u4").astype(np.uint32).reshape(-1)
    return (0, -1, np.ascontiguousarray(words))


def leaf_matching_ids(col: _ColInfo, leaf: dict) -> np.ndarray:
    """Boolean mask over dictIds of the ids the leaf's evaluator matches (PredicateEvaluator.getMatchingDictionaryIds)."""
    lo, hi, words = resolve_leaf(col, leaf)
    card = col.meta.cardinality
    if words is None:
        m = np.zeros(card, dtype=bool)
        if hi >= lo:
            m[lo:hi + 1] = True
        return m
    bits = np.unpackbits(words.astype(">u4").view(np.uint8), bitorder="big").reshape(-1, 32)[:, ::-1].reshape(-1)
    return bits[:card].astype(bool)


def _flatten_filter(tree):
    """FilterQueryTree -> postfix nodes + leaf list."""
    nodes, leaves = [], []

    def walk(t):
        if t["op"] in ("AND", "OR"):
            for c in t["children"]:
                walk(c)
            nodes.append((N.PGX_F_AND if t["op"] == "AND" else N.PGX_F_OR, len(t["children"])))
        else:
            nodes.append((N.PGX_F_LEAF, len(leaves)))
            leaves.append(t)

    if tree is not None:
        walk(tree)
    return nodes, leaves


# ------------------------------------------------------------------------------------------------
# Results
# ------------------------------------------------------------------------------------------------
@dataclass
class ExecutionStatistics:
    num_docs_scanned: int = 0
    num_entries_scanned_in_filter: int = 0
    num_entries_scanned_post_filter: int = 0
    num_total_raw_docs: int = 0

    def as_list(self):
        return [self.num_docs_scanned, self.num_entries_scanned_in_filter, self.num_entries_scanned_post_filter,
                self.num_total_raw_docs]


@dataclass
class GroupKey:
    group_id: int
    string_key: str


class AggregationGroupByResult:
    """operator/aggregation/groupby/AggregationGroupByResult.java:56-113 over the columnar pgx result."""

    def __init__(self, keys: List[str], values: List[list], fns: List[str], mode: str, raw_keys=None, key_parts=None):
        self._keys = keys
        self._values = values  # [group][fn]
        self.fns = fns
        self.storage_mode = mode
        self.raw_keys = raw_keys
        self.key_parts = key_parts  # [column][group]: each group column's rendered value (a field may hold tabs)

    def get_group_key_iterator(self):
        for i, k in enumerate(self._keys):
            yield GroupKey(i, k)

    def get_result_for_key(self, key: GroupKey, fn_index: int):
        return self._values[key.group_id][fn_index]

    def num_groups(self):
        return len(self._keys)

    def as_map(self) -> Dict[str, list]:
        return {k: v for k, v in zip(self._keys, self._values)}


@dataclass
class IntermediateResultsBlock:
    aggregation_result: Optional[list] = None
    aggregation_group_by_result: Optional[AggregationGroupByResult] = None
    trimmed: Optional[List[Dict[str, object]]] = None  # combine output after trimToSize (one map per function)
    stats: ExecutionStatistics = field(default_factory=ExecutionStatistics)

    def get_aggregation_result(self):
        return self.aggregation_result

    def get_aggregation_group_by_result(self):
        return self.aggregation_group_by_result


_MODES = {0: "ARRAY_BASED", 1: "LONG_MAP_BASED", 2: "ARRAY_MAP_BASED"}


class _Query:
    """A compiled pgx_query for one broker request."""

    def __init__(self, ctx: Context, request: dict):
        self.ctx = ctx
        self.request = request
        aggs = request["aggregations"]
        self.fns = [a["fn"] for a in aggs]
        self._keep = []
        agg_arr = (N.Agg * len(aggs))()
        for i, a in enumerate(aggs):
            agg_arr[i].fn = _FN[a["fn"]]
            col = None if a["column"] == "*" else a["column"].encode()
            self._keep.append(col)
            agg_arr[i].column = col
        gb = request.get("group_by")
        gcols = gb["columns"] if gb else []
        garr = (C.c_char_p * max(1, len(gcols)))(*[g.encode() for g in gcols])
        nodes, leaves = _flatten_filter(request.get("filter"))
        self.leaves = leaves
        narr = (N.FilterNode * max(1, len(nodes)))()
        for i, (op, arg) in enumerate(nodes):
            narr[i].op, narr[i].arg = op, arg
        larr = (N.Leaf * max(1, len(leaves)))()
        for i, lf in enumerate(leaves):
            cb = lf["column"].encode()
            self._keep.append(cb)
            larr[i].column = cb
            larr[i].kind = N.PGX_PRED[lf["op"]]
        # BrokerRequest debug option useStarTree=false (common/utils/request/RequestUtils.java:229-236)
        use_st = str((request.get("debug_options") or {}).get("useStarTree", "true")).lower() != "false"
        qd = N.QueryDesc(len(aggs), agg_arr, len(gcols), garr, gb["top_n"] if gb else 10, len(nodes), narr,
                         len(leaves), larr, 0 if use_st else N.PGX_Q_NO_STAR_TREE)
        self._keep += [agg_arr, garr, narr, larr]
        h = C.c_void_p()
        N.check(N.lib().pgx_query_compile(ctx.handle, C.byref(qd), C.byref(h)))
        self.handle = h
        self.group_cols = gcols
        self.domains = {}  # group column -> (sorted values, data type) of a caller-given key domain

    def predicates(self):
        """The leaves' raw predicate values for pgx_bind_predicates (a-4 runs inside the library)."""
        if getattr(self, "_preds", None) is None:
            keep = []
            arr = (N.Predicate * max(1, len(self.leaves)))()
            for l, leaf in enumerate(self.leaves):
                if leaf["op"] == "RANGE":
                    lower, upper, inc_lo, inc_hi = _parse_range(leaf["values"][0])
                    vals = [lower, upper]
                    arr[l].lower_inclusive, arr[l].upper_inclusive = int(inc_lo), int(inc_hi)
                else:
                    vals = list(leaf["values"])
                cv = (C.c_char_p * max(1, len(vals)))(*[v.encode("utf-8") for v in vals])
                keep.append(cv)
                arr[l].num_values = len(vals)
                arr[l].values = cv
            self._preds = (arr, keep)
        return self._preds[0]

    def bindings(self, segments: Sequence[IndexSegment], seg_array=None):
        """[segment][leaf] dictId-space bindings (PredicateEvaluatorProvider per segment), resolved by the library.
        `seg_array`: the segments' handles as a ctypes array when the caller already holds one (the Java side passes
        its long[] as is).  Returns (binding array, owner): keep the owner alive while the array is in use."""
        segs = seg_array if seg_array is not None else \
            (C.c_void_p * max(1, len(segments)))(*[s.handle.value for s in segments])
        h = C.c_void_p()
        N.check(N.lib().pgx_bind_predicates(self.handle, segs, len(segments), self.predicates(), C.byref(h)))
        owner = _Bindings(h)
        return N.lib().pgx_bindings_array(h), owner

    def execute(self, segments: Sequence[IndexSegment], flags: int = 0, dense_out=None, dense_out_bytes: int = 0):
        segs = (C.c_void_p * len(segments))(*[s.handle.value for s in segments])
        binds, keep = self.bindings(segments)
        opts = N.ExecOpts(0, dense_out, dense_out_bytes, flags)
        r = C.c_void_p()
        N.check(N.lib().pgx_execute(self.ctx.handle, self.handle, segs, len(segments), binds, C.byref(opts),
                                    C.byref(r)))
        return r

    def execute_async(self, segments: Sequence[IndexSegment], flags: int = 0):
        """pgx_execute_async: returns the pending result at once (the library copied the bindings); every accessor,
        or pgx_result_wait, waits for it."""
        segs = (C.c_void_p * len(segments))(*[s.handle.value for s in segments])
        binds, keep = self.bindings(segments)
        opts = N.ExecOpts(0, None, 0, flags)
        r = C.c_void_p()
        N.check(N.lib().pgx_execute_async(self.ctx.handle, self.handle, segs, len(segments), binds, C.byref(opts),
                                          C.byref(r)))
        return r

    def execute_multi(self, segments: Sequence[IndexSegment], contexts: Optional[Sequence[Context]] = None,
                      flags: int = 0):
        """pgx_execute_multi over segments staged on several contexts (one per device); the merged result lives on
        the first context's device and its group keys index into `segments`."""
        if contexts is None:
            contexts = []
            for s in segments:
                if all(s.ctx is not c for c in contexts):
                    contexts.append(s.ctx)
        ctxs = (C.c_void_p * len(contexts))(*[c.handle.value for c in contexts])
        segs = (C.c_void_p * len(segments))(*[s.handle.value for s in segments])
        binds, keep = self.bindings(segments)
        opts = N.ExecOpts(0, None, 0, flags)
        r = C.c_void_p()
        N.check(N.lib().pgx_execute_multi(ctxs, len(contexts), self.handle, segs, len(segments), binds,
                                          C.byref(opts), C.byref(r)))
        return r

    def set_key_domain(self, g: int, values, data_type: str):
        """pgx_query_set_key_domain: group column g's key space becomes `values` (sorted distinct, the union of the
        column's dictionaries over every process's segments), so ranks plan identical keys.  The result's
        keys for that column then come back as (-1, index into values); `render_key` reads them from here."""
        L = N.lib()
        if values is None:
            N.check(L.pgx_query_set_key_domain(self.handle, g, 0, 0, None, None, None))
            self.domains.pop(g, None)
            return
        t = {"INT": N.PGX_INT, "LONG": N.PGX_LONG, "FLOAT": N.PGX_FLOAT, "DOUBLE": N.PGX_DOUBLE,
             "STRING": N.PGX_STRING}[data_type]
        if data_type == "STRING":
            vals = sorted(set(str(v) for v in values), key=lambda v: v.encode("utf-8"))
            arr = (C.c_char_p * max(1, len(vals)))(*[v.encode("utf-8") for v in vals])
            N.check(L.pgx_query_set_key_domain(self.handle, g, t, len(vals), None, None, arr))
            keep = np.array(vals, dtype=object)
        elif data_type in ("INT", "LONG"):
            keep = np.unique(np.asarray(values, dtype=np.int64))
            N.check(L.pgx_query_set_key_domain(self.handle, g, t, len(keep), keep.ctypes.data, None, None))
        else:
            keep = np.unique(np.asarray(values, dtype=np.float64))
            N.check(L.pgx_query_set_key_domain(self.handle, g, t, len(keep), None, keep.ctypes.data, None))
        self.domains[g] = (keep, data_type)

    def close(self):
        if getattr(self, "handle", None):
            N.lib().pgx_query_release(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class _Bindings:
    """Owner of a pgx_bindings handle."""

    def __init__(self, h):
        self.h = h

    def __del__(self):
        if self.h:
            N.lib().pgx_bindings_release(self.h)
            self.h = None


def _render_value(data_type: str, v) -> str:
    """Dictionary.getStringValue of one group value (keys are dictionary values joined by tab)."""
    if data_type == "STRING":
        return str(v)
    if data_type in ("INT", "LONG"):
        return str(int(v))
    if data_type == "FLOAT":
        return _java_double_str(float(np.float32(v)))
    return _java_double_str(float(v))


def render_key(q: _Query, segments: Sequence[IndexSegment], g: int, seg_index: int, dict_id: int) -> str:
    """Group column g's value of one result key: a segment's dictionary entry, or (seg_index -1) an entry of the
    query's key domain (pgx_query_set_key_domain)."""
    if seg_index < 0:
        vals, dt = q.domains[g]
        return _render_value(dt, vals[dict_id])
    return segments[seg_index].column(q.group_cols[g]).string_of(int(dict_id))


def decode_result(q: _Query, r, segments: Sequence[IndexSegment], trim: bool = False) -> IntermediateResultsBlock:
    L = N.lib()
    st = (C.c_int64 * 4)()
    N.check(L.pgx_result_stats(r, st))
    blk = IntermediateResultsBlock(stats=ExecutionStatistics(*list(st)))
    if not q.group_cols:
        out = []
        for i, fn in enumerate(q.fns):
            v, c = C.c_double(), C.c_int64()
            N.check(L.pgx_result_agg(r, i, C.byref(v), C.byref(c)))
            if fn in ("count", "countmv"):
                out.append(int(c.value))  # MutableLongValue
            elif fn in ("avg", "avgmv"):
                out.append((v.value, int(c.value)))  # AvgPair(sum, count): count = values for AVGMV
            else:
                out.append(v.value)
        blk.aggregation_result = out
        return blk
    ng = C.c_int64()
    N.check(L.pgx_result_num_groups(r, C.byref(ng)))
    n = ng.value
    mode = C.c_int32()
    N.check(L.pgx_result_group_mode(r, C.byref(mode)))
    key_parts = []
    raw = []
    for g, col in enumerate(q.group_cols):
        si = np.zeros(max(n, 1), dtype=np.int32)
        di = np.zeros(max(n, 1), dtype=np.int32)
        N.check(L.pgx_result_group_keys(r, g, si.ctypes.data, di.ctypes.data))
        key_parts.append([render_key(q, segments, g, int(si[i]), int(di[i])) for i in range(n)])
        raw.append(di[:n].copy())
    keys = ["\t".join(p[i] for p in key_parts) for i in range(n)]
    vals = []
    for i, fn in enumerate(q.fns):
        v = np.zeros(max(n, 1), dtype=np.float64)
        c = np.zeros(max(n, 1), dtype=np.int64)
        N.check(L.pgx_result_group_values(r, i, v.ctypes.data, c.ctypes.data))
        if fn in ("count", "countmv"):
            vals.append([int(x) for x in c[:n]])
        elif fn in ("avg", "avgmv"):  # AvgPair(sum, count): count = values for AVGMV
            vals.append([(float(a), int(b)) for a, b in zip(v[:n], c[:n])])
        else:
            vals.append([float(x) for x in v[:n]])
    per_group = [[vals[f][i] for f in range(len(q.fns))] for i in range(n)]
    blk.aggregation_group_by_result = AggregationGroupByResult(keys, per_group, q.fns, _MODES[mode.value],
                                                               raw_keys=raw, key_parts=key_parts)
    if trim:
        trimmed = []
        for i in range(len(q.fns)):
            cap = C.c_int64(n)
            idx = np.zeros(max(n, 1), dtype=np.int64)
            N.check(L.pgx_result_trim(r, i, idx.ctypes.data, C.byref(cap)))
            trimmed.append({keys[j]: per_group[j][i] for j in idx[:cap.value]})
        blk.trimmed = trimmed
    return blk


def trim_and_gather(q: _Query, r):
    """Combine trim of a group-by result (pgx_result_trim, AggregationGroupByOperatorService.trimToSize) and the
    kept groups only (pgx_result_gather): per function (seg_index[ncols, n], dict_id[ncols, n], value[n], count[n]).
    For results that stay in device memory neither call reads the other groups back."""
    L = N.lib()
    ncols, nf = len(q.group_cols), len(q.fns)
    out = []
    total = C.c_int64(0)
    N.check(L.pgx_result_num_groups(r, C.byref(total)))
    shared = None  # every function keeps every group (the trim rule depends on the group count only): one gather
    for i in range(nf):
        if shared is None:
            cap = C.c_int64(0)
            N.check(L.pgx_result_trim(r, i, None, C.byref(cap)))
            n = cap.value
            idx = np.empty(max(n, 1), dtype=np.int64)
            N.check(L.pgx_result_trim(r, i, idx.ctypes.data, C.byref(cap)))
            si = np.empty(max(n * ncols, 1), dtype=np.int32)
            di = np.empty(max(n * ncols, 1), dtype=np.int32)
            v = np.empty(max(n * nf, 1), dtype=np.float64)
            c = np.empty(max(n * nf, 1), dtype=np.int64)
            N.check(L.pgx_result_gather(r, idx.ctypes.data, n, si.ctypes.data, di.ctypes.data, v.ctypes.data,
                                        c.ctypes.data))
            if n == total.value:
                shared = (n, si, di, v, c)
        else:
            n, si, di, v, c = shared
        out.append((si[:n * ncols].reshape(ncols, n), di[:n * ncols].reshape(ncols, n), v[i * n:(i + 1) * n],
                    c[i * n:(i + 1) * n]))
    return out


def trimmed_maps(q: _Query, r, segments: Sequence[IndexSegment]) -> List[Dict[str, object]]:
    """trim_and_gather rendered like the reference's trimmed combine output: one {string key: value} map per
    function (count -> int, avg -> (sum, count), others -> float)."""
    maps = []
    for fn, (si, di, v, c) in zip(q.fns, trim_and_gather(q, r)):
        m = {}
        for j in range(len(v)):
            key = "\t".join(render_key(q, segments, g, int(si[g, j]), int(di[g, j])) for g in range(len(q.group_cols)))
            m[key] = int(c[j]) if fn in ("count", "countmv") else (
                (float(v[j]), int(c[j])) if fn in ("avg", "avgmv") else float(v[j]))
        maps.append(m)
    return maps


def _column_values(segments: Sequence[IndexSegment], col: str, si: np.ndarray, di: np.ndarray,
                   domain=None) -> np.ndarray:
    """Values of (segment index, dictId) pairs of one group column, vectorised per distinct segment dictionary;
    segment index -1 reads the query's key domain for the column (`domain`: (values, data type))."""
    infos = [seg.column(col) for seg in segments]
    strings = infos[0].meta.data_type == "STRING"
    out = np.empty(len(si), dtype=object if strings else np.float64 if infos[0].meta.data_type in ("FLOAT", "DOUBLE")
                   else np.int64)
    for s in np.unique(si):
        m = si == s
        vals = domain[0] if s < 0 else infos[int(s)].values
        out[m] = (np.asarray(vals, dtype=object) if strings else np.asarray(vals))[di[m]]
    return out.astype(str) if strings else out


def group_partials(q: _Query, r, segments: Sequence[IndexSegment]):
    """Every group of a group-by result as (key_cols: one array of group-column VALUES per column, vals float64
    [nf, n], cnts int64 [nf, n]): the per-GPU partial of the cross-GPU sparse merge (multigpu.merge_group_partials)."""
    L = N.lib()
    ng = C.c_int64()
    N.check(L.pgx_result_num_groups(r, C.byref(ng)))
    n = ng.value
    cols = []
    for g, col in enumerate(q.group_cols):
        si = np.zeros(max(n, 1), dtype=np.int32)
        di = np.zeros(max(n, 1), dtype=np.int32)
        N.check(L.pgx_result_group_keys(r, g, si.ctypes.data, di.ctypes.data))
        cols.append(_column_values(segments, col, si[:n], di[:n], q.domains.get(g)))
    nf = len(q.fns)
    vals = np.zeros((nf, max(n, 1)))
    cnts = np.zeros((nf, max(n, 1)), dtype=np.int64)
    for i in range(nf):
        N.check(L.pgx_result_group_values(r, i, vals[i].ctypes.data, cnts[i].ctypes.data))
    return cols, vals[:, :n], cnts[:, :n]


def render_group_maps(q: _Query, segments: Sequence[IndexSegment], key_cols, vals, cnts, kept) -> List[Dict[str, object]]:
    """Merged (and trimmed: `kept` = group indices per function) groups as the reference's trimmed combine output:
    one {string key: value} map per function, keys rendered like Dictionary.getStringValue (values joined by tab)."""
    types = [segments[0].column(col).meta.data_type for col in q.group_cols]
    maps = []
    for i, fn in enumerate(q.fns):
        m = {}
        for j in kept[i]:
            key = "\t".join(_render_value(dt, c[j]) for dt, c in zip(types, key_cols))
            m[key] = int(cnts[i, j]) if fn in ("count", "countmv") else (
                (float(vals[i, j]), int(cnts[i, j])) if fn in ("avg", "avgmv") else float(vals[i, j]))
        maps.append(m)
    return maps


# ------------------------------------------------------------------------------------------------
# Operators / plan nodes / plan maker
# ------------------------------------------------------------------------------------------------
# Shape limits of ONE library query (pinot_amd/csrc/pgx_internal.h:12-15: kMaxAggs, kMaxQCols).  The reference has
# none (AggregationFunctionFactory builds any number of functions; FilterPlanNode.java:62-170 any number of columns), so
# a request past them runs as several library queries over slices of its functions (_GpuOperator._run_slices).
MAX_AGGS = 8
MAX_COLS = 16
_EXT_BASE_SLOTS = {"minmaxrange": 2}  # extended.py _base_request: MIN + MAX; histogram functions add no slot


def agg_slices(request: dict, max_aggs: int = MAX_AGGS, max_cols: int = MAX_COLS) -> List[List[int]]:
    """Consecutive slices of the request's function indices such that each slice, with the request's filter and GROUP
    BY, fits one library query: at most `max_aggs` aggregation slots (an extended slice's base query holds COUNT(*)
    plus the slots extended.py's _base_request gives; AVGMV keeps a second plane for its value count, pgx_mv.cpp:158)
    and at most `max_cols` distinct columns (filter leaves, group columns, aggregated columns).  One slice when the
    request fits as it is; a single function past the limits on its own stays one slice (the library refuses it)."""
    from .pql import EXT_FUNCTIONS, EXT_MV_FUNCTIONS
    aggs = request["aggregations"]
    _, leaves = _flatten_filter(request.get("filter"))
    fixed = {lf["column"] for lf in leaves} | set((request.get("group_by") or {}).get("columns", []))

    def slots(idx):
        fns = [aggs[i]["fn"] for i in idx]
        if any(f in EXT_FUNCTIONS or f in EXT_MV_FUNCTIONS for f in fns):
            return 1 + sum(_EXT_BASE_SLOTS.get(f, 0 if (f in EXT_FUNCTIONS or f in EXT_MV_FUNCTIONS) else
                                               (2 if f == "avgmv" else 1)) for f in fns)
        return len(fns) + sum(1 for f in fns if f == "avgmv")

    def ncols(idx):
        return len(fixed | {aggs[i]["column"] for i in idx if aggs[i]["column"] != "*"})

    out, cur = [], []
    for i in range(len(aggs)):
        if cur and (slots(cur + [i]) > max_aggs or ncols(cur + [i]) > max_cols):
            out.append(cur)
            cur = []
        cur.append(i)
    out.append(cur)
    return out


class _GpuOperator:
    """Gpu{Aggregation,AggregationGroupBy}Operator: returns exactly one IntermediateResultsBlock (blockId 0), then None
    (operator/aggregation/groupby/AggregationGroupByOperator.java:81-85)."""

    def __init__(self, ctx, request, segments, combine: bool):
        self.ctx = ctx
        self.request = request
        self.segments = list(segments)
        self.combine = combine
        self._done = False
        self._stats = None

    def open(self):
        return True

    def close(self):
        return True

    def next_block(self):
        if self._done:
            return None
        slices = agg_slices(self.request)
        if len(slices) > 1:
            blk = self._run_slices(slices)
            self._stats = blk.stats
            self._done = True
            return blk
        from . import extended
        if extended.has_extended(self.request):  # decomposed into GPU sub-queries on the host (extended.py)
            blk = extended.run(self.ctx, self.request, self.segments, combine=self.combine)
            if self.request.get("group_by") and blk.aggregation_group_by_result.num_groups() == 0 and not self.combine:
                blk.aggregation_group_by_result = None
            self._stats = blk.stats
            self._done = True
            return blk
        q = _Query(self.ctx, self.request)
        r = q.execute(self.segments)
        try:
            blk = decode_result(q, r, self.segments, trim=self.combine and bool(q.group_cols))
        finally:
            N.lib().pgx_result_release(r)
            q.close()
        if q.group_cols and blk.aggregation_group_by_result.num_groups() == 0 and not self.combine:
            blk.aggregation_group_by_result = None  # DefaultGroupByExecutor.java:221-224: no blocks -> null result
        self._stats = blk.stats
        self._done = True
        return blk

    nextBlock = next_block

    def _run_slices(self, slices: List[List[int]], use_star_tree: bool = True) -> IntermediateResultsBlock:
        """A request past one library query's shape limits (agg_slices): one operator per slice of its functions,
        same filter and GROUP BY, results concatenated in function order.  Every function's result (and, at the
        combine, its trimmed map: AggregationGroupByOperatorService.trimToSize runs per function) depends on the
        filter and the group keys only, so the slices' results are the whole request's."""
        aggs = self.request["aggregations"]
        blocks = []
        for s in slices:
            sub = dict(self.request, aggregations=[aggs[i] for i in s])
            if not use_star_tree:
                sub["debug_options"] = dict(self.request.get("debug_options") or {}, useStarTree="false")
            blocks.append(type(self)(self.ctx, sub, self.segments, self.combine).next_block())
        # a slice's block served by the star-tree differs from a raw-docs block in docs scanned or in entries scanned
        # in filter (a filter matching nothing scans the same 0 docs either way)
        docs = {(b.stats.num_docs_scanned, b.stats.num_entries_scanned_in_filter) for b in blocks}
        if len(docs) > 1 and use_star_tree:
            # a slice answered from the star-tree and another from the raw docs: the reference plans the request as a
            # whole, and the star-tree only serves it when every function qualifies (StarTreeUtils), so all raw
            return self._run_slices(slices, use_star_tree=False)
        from .extended import _projection_count
        st0 = blocks[0].stats
        stats = ExecutionStatistics(st0.num_docs_scanned, st0.num_entries_scanned_in_filter,
                                    st0.num_docs_scanned * _projection_count(self.request), st0.num_total_raw_docs)
        fns = [a["fn"] for a in aggs]
        if not self.request.get("group_by"):
            res = [v for b in blocks for v in b.get_aggregation_result()]
            return IntermediateResultsBlock(aggregation_result=res, stats=stats)
        out = IntermediateResultsBlock(stats=stats)
        gbs = [b.get_aggregation_group_by_result() for b in blocks]
        if all(g is not None for g in gbs):
            first = gbs[0]
            keys = [k.string_key for k in first.get_group_key_iterator()]
            maps = [g.as_map() for g in gbs]
            if any(len(g) != len(keys) or any(k not in g for k in keys) for g in maps[1:]):
                raise N.PgxError(N.PGX_ERR_INTERNAL, "aggregation slices found different groups")
            per_group = [[v for g in maps for v in g[k]] for k in keys]
            out.aggregation_group_by_result = AggregationGroupByResult(
                keys, per_group, fns, first.storage_mode, raw_keys=first.raw_keys, key_parts=first.key_parts)
        elif any(g is not None for g in gbs):
            raise N.PgxError(N.PGX_ERR_INTERNAL, "aggregation slices found different groups")
        if self.combine:
            out.trimmed = [m for b in blocks for m in b.trimmed]
        return out

    def get_execution_statistics(self) -> ExecutionStatistics:
        return self._stats


class AggregationOperator(_GpuOperator):
    pass


class AggregationGroupByOperator(_GpuOperator):
    pass


class PlanNode:
    def __init__(self, op_factory):
        self._f = op_factory

    def run(self):
        return self._f()


class Plan:
    """GlobalPlanImplV0 over InstanceResponsePlanNode(CombinePlanNode(...)) (plan/GlobalPlanImplV0.java:52-75)."""

    def __init__(self, op):
        self._op = op
        self.result = None

    def execute(self):
        self.result = self._op.next_block()
        return self.result


class InstancePlanMakerImplV2:
    """plan/maker/InstancePlanMakerImplV2.java:72-109 for aggregation and aggregation-group-by queries."""

    def __init__(self, ctx: Context):
        self.ctx = ctx

    def make_inner_segment_plan(self, segment: IndexSegment, broker_request: dict) -> PlanNode:
        cls = AggregationGroupByOperator if broker_request.get("group_by") else AggregationOperator
        return PlanNode(lambda: cls(self.ctx, broker_request, [segment], combine=False))

    def make_inter_segment_plan(self, segments: Sequence[IndexSegment], broker_request: dict) -> Plan:
        cls = AggregationGroupByOperator if broker_request.get("group_by") else AggregationOperator
        return Plan(cls(self.ctx, broker_request, segments, combine=True))

    makeInnerSegmentPlan = make_inner_segment_plan
    makeInterSegmentPlan = make_inter_segment_plan
