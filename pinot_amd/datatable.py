"""The server -> broker wire format: DataTable bytes.

A Pinot server answers each instance request with ONE serialized DataTable (InstanceResponseOperator ->
IntermediateResultsBlock.getDataTable, core/operator/blocks/IntermediateResultsBlock.java:147-235); the broker parses it
back (DataTable(byte[]), common/utils/DataTable.java:204-277) before BrokerReduceService.reduceOnDataTable.  This module
writes and reads exactly that layout, so a GPU server is wire-compatible with a Java broker and vice versa:

    header (52 bytes, big-endian ints): version | numRows | numCols | 5 x (start, length) for
        dictionary | metadata | schema | fixed-size rows | variable-size data          (DataTable.java:315-378)
    dictionary: count, then per STRING column: name, count, (id, utf8 value) pairs       (:419-440)
    metadata:   count, then (utf8 key, utf8 value) pairs                                 (:380-396)
    schema:     count, column names, column type NAMES (DataSchema.toBytes, DataTableBuilder.java:549-572)
    rows:       fixed-width cells (DataTableBuilder.java:118-170): LONG / DOUBLE 8 B, INT 4 B, STRING 4-B dictionary
                id, OBJECT (offset, length) into the variable section, where version 2 (the custom ser/de the server
                registers, server/starter/ServerBuilder.java:138) prefixes every object with its 4-byte type id
                (DataTableBuilder.setColumn(int, Object), :330-342)
    objects:    DataTableCustomSerDe (core/util/DataTableCustomSerDe.java:164-475): String utf8, MutableLong / Double 8 B,
                DoubleArrayList (n, doubles), AvgPair (double sum, long count), MinMaxRangePair (double, double),
                HyperLogLog (stream-lib getBytes), HashMap (size, key type, value type, then length-prefixed
                key / value objects), IntOpenHashSet (size, ints)

The server side mirrors getAggregationResultDataTable (one row, one column per function: LONG count_star, DOUBLE
sum / min / max, OBJECT for the rest) and getAggregationGroupByResultDataTable (one row per function: STRING function
name, OBJECT HashMap<group string, intermediate>), then attachMetadataToDataTable (numDocsScanned,
numEntriesScannedInFilter, numEntriesScannedPostFilter, totalDocs, "Exception<code>" entries).  Java HashMap iteration
order (the order the reference writes map entries and metadata) is reproduced for String keys: buckets of
(h ^ h >>> 16) & (capacity - 1) over String.hashCode at the capacity a default HashMap grows to, entries of one bucket
in insertion order.  IntOpenHashSet's order is fastutil's internal table order in the reference and ascending here;
readers of the format do not depend on it.
"""
from __future__ import annotations

import struct
from typing import Dict, List, Optional, Sequence

from . import hll as HLL
from . import qdigest as QD

V1, V2 = 1, 2
HEADER_BYTES = 52

# FieldSpec.DataType names used by DataSchema (common/data/FieldSpec.java:209-228) and fixed cell widths
CELL_BYTES = {"BOOLEAN": 1, "BYTE": 1, "CHAR": 2, "SHORT": 2, "INT": 4, "LONG": 8, "FLOAT": 8, "DOUBLE": 8,
              "STRING": 4, "OBJECT": 8}

# DataTableSerDe.DataType ids (common/utils/DataTableSerDe.java:30-41)
T_OBJECT, T_STRING, T_MUTABLE_LONG, T_DOUBLE, T_DOUBLE_ARRAY, T_AVG_PAIR, T_MIN_MAX_RANGE, T_HLL, T_QDIGEST, \
    T_HASHMAP, T_INT_SET = -1, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9

NUM_DOCS_SCANNED = "numDocsScanned"
NUM_ENTRIES_SCANNED_IN_FILTER = "numEntriesScannedInFilter"
NUM_ENTRIES_SCANNED_POST_FILTER = "numEntriesScannedPostFilter"
TOTAL_DOCS = "totalDocs"
EXCEPTION_KEY = "Exception"


def _i32(x: int) -> bytes:
    return struct.pack(">i", x)


def _utf8(s: str) -> bytes:
    return s.encode("utf-8")


def java_string_hash(s: str) -> int:
    """String.hashCode over UTF-16 code units, as a signed 32-bit int."""
    h = 0
    for u in struct.unpack(">%dH" % (len(s.encode("utf-16-be")) // 2), s.encode("utf-16-be")):
        h = (31 * h + u) & 0xFFFFFFFF
    return h - (1 << 32) if h >= 1 << 31 else h


def java_hashmap_order(keys: Sequence[str]) -> List[str]:
    """Iteration order of a java.util.HashMap<String, ?> filled by put() in the given order from the default capacity
    (16, load factor 0.75, doubling when size exceeds the threshold): ascending bucket index of the spread hash, entries
    of one bucket in insertion order (a resize splits a bucket's list preserving relative order)."""
    cap = 16
    while len(keys) > cap * 3 // 4:
        cap *= 2

    def bucket(k: str) -> int:
        h = java_string_hash(k) & 0xFFFFFFFF
        return (h ^ (h >> 16)) & (cap - 1)
    return [k for _, _, k in sorted((bucket(k), i, k) for i, k in enumerate(keys))]


# ---------------------------------------------------------------------------------------------------------------------
# DataTableCustomSerDe objects
# ---------------------------------------------------------------------------------------------------------------------
class AvgPair(tuple):
    """AvgAggregationFunction.AvgPair (double sum, long count)."""


class MinMaxRangePair(tuple):
    """MinMaxRangeAggregationFunction.MinMaxRangePair (double min, double max)."""


class HyperLogLogRegs:
    """stream-lib HyperLogLog registers (pinot_amd/hll.py layout)."""

    def __init__(self, regs):
        self.regs = regs


def object_type(v) -> int:
    """DataTableCustomSerDe.getDataTypeOfObject for the intermediates this path produces."""
    if isinstance(v, str):
        return T_STRING
    if isinstance(v, AvgPair):
        return T_AVG_PAIR
    if isinstance(v, MinMaxRangePair):
        return T_MIN_MAX_RANGE
    if isinstance(v, HyperLogLogRegs):
        return T_HLL
    if isinstance(v, QD.QuantileDigest):
        return T_QDIGEST
    if isinstance(v, dict):
        return T_HASHMAP
    if isinstance(v, (set, frozenset)):
        return T_INT_SET
    if isinstance(v, list):
        return T_DOUBLE_ARRAY
    if isinstance(v, float):
        return T_DOUBLE
    raise TypeError("no DataTableCustomSerDe type for %r" % type(v))


def serialize_object(v) -> bytes:
    """DataTableCustomSerDe.serializeObject (core/util/DataTableCustomSerDe.java:164-218)."""
    t = object_type(v)
    if t == T_STRING:
        return _utf8(v)
    if t == T_DOUBLE:
        return struct.pack(">d", v)
    if t == T_AVG_PAIR:
        return struct.pack(">dq", float(v[0]), int(v[1]))
    if t == T_MIN_MAX_RANGE:
        return struct.pack(">dd", float(v[0]), float(v[1]))
    if t == T_DOUBLE_ARRAY:
        return _i32(len(v)) + b"".join(struct.pack(">d", float(x)) for x in v)
    if t == T_INT_SET:
        return _i32(len(v)) + b"".join(_i32(int(x)) for x in sorted(v))
    if t == T_HLL:
        return HLL.to_bytes(v.regs)
    if t == T_QDIGEST:
        return v.serialize()
    # HashMap: size, then (key type, value type) before the first entry, then length-prefixed key / value bytes
    out = [_i32(len(v))]
    keys = java_hashmap_order(list(v.keys())) if all(isinstance(k, str) for k in v) else list(v.keys())
    first = True
    for k in keys:
        val = v[k]
        if first:
            out += [_i32(object_type(k)), _i32(object_type(val))]
            first = False
        kb, vb = serialize_object(k), serialize_object(val)
        out += [_i32(len(kb)), kb, _i32(len(vb)), vb]
    return b"".join(out)


def deserialize_object(b: bytes, t: int):
    """DataTableCustomSerDe.deserializeObject (:102-153)."""
    if t == T_STRING:
        return b.decode("utf-8")
    if t == T_MUTABLE_LONG:
        return struct.unpack(">q", b)[0]
    if t == T_DOUBLE:
        return struct.unpack(">d", b)[0]
    if t == T_AVG_PAIR:
        s, c = struct.unpack(">dq", b)
        return AvgPair((s, c))
    if t == T_MIN_MAX_RANGE:
        return MinMaxRangePair(struct.unpack(">dd", b))
    if t == T_DOUBLE_ARRAY:
        n = struct.unpack_from(">i", b)[0]
        return list(struct.unpack_from(">%dd" % n, b, 4))
    if t == T_INT_SET:
        n = struct.unpack_from(">i", b)[0]
        return set(struct.unpack_from(">%di" % n, b, 4))
    if t == T_HLL:
        return HyperLogLogRegs(HLL.from_bytes(b))
    if t == T_QDIGEST:
        return QD.QuantileDigest.deserialize(b)
    if t == T_HASHMAP:
        if not b:
            return {}
        n = struct.unpack_from(">i", b)[0]
        if n == 0:
            return {}
        kt, vt = struct.unpack_from(">ii", b, 4)
        p, out = 12, {}
        for _ in range(n):
            ln = struct.unpack_from(">i", b, p)[0]
            k = deserialize_object(b[p + 4:p + 4 + ln], kt)
            p += 4 + ln
            ln = struct.unpack_from(">i", b, p)[0]
            out[k] = deserialize_object(b[p + 4:p + 4 + ln], vt)
            p += 4 + ln
        return out
    raise ValueError("DataTable object type %d not supported (Java-serialized objects are not read)" % t)


# ---------------------------------------------------------------------------------------------------------------------
# DataTable
# ---------------------------------------------------------------------------------------------------------------------
class DataTable:
    """common/utils/DataTable.java: rows of fixed-width cells + STRING dictionary + metadata + schema."""

    def __init__(self, columns: Optional[List[str]] = None, types: Optional[List[str]] = None, version: int = V2):
        self.version = version
        self.columns = list(columns or [])
        self.types = list(types or [])
        self.rows: List[list] = []
        self.metadata: Dict[str, str] = {}

    # ---- writing (DataTableBuilder + DataTable.toBytes) ----
    def to_bytes(self) -> bytes:
        offs, row_bytes = [], 0
        for t in self.types:
            offs.append(row_bytes)
            row_bytes += CELL_BYTES[t]
        dictionary: Dict[str, Dict[str, int]] = {}
        fixed, var = bytearray(), bytearray()
        for row in self.rows:
            cell = bytearray(row_bytes)
            for c, (t, v) in enumerate(zip(self.types, row)):
                o = offs[c]
                if t == "LONG":
                    struct.pack_into(">q", cell, o, int(v))
                elif t in ("DOUBLE", "FLOAT"):
                    struct.pack_into(">d", cell, o, float(v))
                elif t == "INT":
                    struct.pack_into(">i", cell, o, int(v))
                elif t == "STRING":
                    ids = dictionary.setdefault(self.columns[c], {})
                    ids.setdefault(v, len(ids))
                    struct.pack_into(">i", cell, o, ids[v])
                elif t == "OBJECT":
                    ob = serialize_object(v)
                    struct.pack_into(">ii", cell, o, len(var), len(ob))
                    if self.version == V2:
                        var += _i32(object_type(v))
                    var += ob
                else:
                    raise ValueError("cell type %s not supported" % t)
            fixed += cell
        # a schema-less (exception-only) table has no dictionary at all: DataTable() leaves it null (serializeDictionary)
        dict_bytes = bytearray(_i32(len(dictionary)) if self.columns else b"")
        for col in java_hashmap_order(list(dictionary)):
            rev = {i: s for s, i in dictionary[col].items()}
            dict_bytes += _i32(len(_utf8(col))) + _utf8(col) + _i32(len(rev))
            for i in sorted(rev):  # HashMap<Integer, String>: Integer keys 0..n-1 iterate ascending below capacity
                vb = _utf8(rev[i])
                dict_bytes += _i32(i) + _i32(len(vb)) + vb
        meta = bytearray(_i32(len(self.metadata)))
        for k in java_hashmap_order(list(self.metadata)):
            kb, vb = _utf8(k), _utf8(self.metadata[k])
            meta += _i32(len(kb)) + kb + _i32(len(vb)) + vb
        schema = bytearray()
        if self.columns:
            schema += _i32(len(self.columns))
            for name in self.columns:
                schema += _i32(len(_utf8(name))) + _utf8(name)
            for t in self.types:
                schema += _i32(len(t)) + t.encode("ascii")
        has_rows = bool(self.columns)
        head = [self.version, len(self.rows), len(self.columns)]
        pos = HEADER_BYTES
        for sect in (dict_bytes, meta, schema):
            head += [pos, len(sect)]
            pos += len(sect)
        head += [pos, len(fixed) if has_rows else 0]
        pos += len(fixed) if has_rows else 0
        head += [pos, len(var) if has_rows else 0]
        return b"".join(_i32(x) for x in head) + bytes(dict_bytes) + bytes(meta) + bytes(schema) + \
            (bytes(fixed) + bytes(var) if has_rows else b"")

    # ---- reading (DataTable(byte[])) ----
    @staticmethod
    def from_bytes(b: bytes) -> "DataTable":
        h = struct.unpack_from(">13i", b, 0)
        version, nrows, ncols = h[0], h[1], h[2]
        if version not in (V1, V2):
            raise ValueError("Illegal value for version %d" % version)
        (ds, dl), (ms, ml), (ss, sl), (fs, fl), (vs, vl) = [(h[3 + 2 * i], h[4 + 2 * i]) for i in range(5)]
        dt = DataTable(version=version)
        rev: Dict[str, Dict[int, str]] = {}
        if dl:
            p = ds
            n = struct.unpack_from(">i", b, p)[0]
            p += 4
            for _ in range(n):
                ln = struct.unpack_from(">i", b, p)[0]
                col = b[p + 4:p + 4 + ln].decode("utf-8")
                p += 4 + ln
                m = struct.unpack_from(">i", b, p)[0]
                p += 4
                ids = rev.setdefault(col, {})
                for _ in range(m):
                    i, ln = struct.unpack_from(">ii", b, p)
                    ids[i] = b[p + 8:p + 8 + ln].decode("utf-8")
                    p += 8 + ln
        if ml:
            p = ms
            n = struct.unpack_from(">i", b, p)[0]
            p += 4
            for _ in range(n):
                ln = struct.unpack_from(">i", b, p)[0]
                k = b[p + 4:p + 4 + ln].decode("utf-8")
                p += 4 + ln
                ln = struct.unpack_from(">i", b, p)[0]
                dt.metadata[k] = b[p + 4:p + 4 + ln].decode("utf-8")
                p += 4 + ln
        if sl:
            p = ss
            n = struct.unpack_from(">i", b, p)[0]
            p += 4
            for _ in range(n):
                ln = struct.unpack_from(">i", b, p)[0]
                dt.columns.append(b[p + 4:p + 4 + ln].decode("utf-8"))
                p += 4 + ln
            for _ in range(n):
                ln = struct.unpack_from(">i", b, p)[0]
                dt.types.append(b[p + 4:p + 4 + ln].decode("ascii"))
                p += 4 + ln
        offs, row_bytes = [], 0
        for t in dt.types:
            offs.append(row_bytes)
            row_bytes += CELL_BYTES[t]
        fixed = b[fs:fs + fl] if fl else b""
        var = b[vs:vs + vl] if vl else b""
        for r in range(nrows):
            row = []
            for c, t in enumerate(dt.types):
                o = r * row_bytes + offs[c]
                if t == "LONG":
                    row.append(struct.unpack_from(">q", fixed, o)[0])
                elif t in ("DOUBLE", "FLOAT"):
                    row.append(struct.unpack_from(">d", fixed, o)[0])
                elif t == "INT":
                    row.append(struct.unpack_from(">i", fixed, o)[0])
                elif t == "STRING":
                    row.append(rev[dt.columns[c]][struct.unpack_from(">i", fixed, o)[0]])
                elif t == "OBJECT":
                    start, ln = struct.unpack_from(">ii", fixed, o)
                    if version == V2:
                        typ = struct.unpack_from(">i", var, start)[0]
                        row.append(deserialize_object(var[start + 4:start + 4 + ln], typ))
                    else:
                        raise ValueError("version-1 DataTables hold Java-serialized objects: not read")
                else:
                    raise ValueError("cell type %s not supported" % t)
            dt.rows.append(row)
        return dt


# ---------------------------------------------------------------------------------------------------------------------
# InstanceResponse <-> DataTable (IntermediateResultsBlock.getDataTable / BrokerReduceService's read)
# ---------------------------------------------------------------------------------------------------------------------
def _base_fn(fn: str) -> str:
    """The function whose intermediate an MV function carries: AggregationFunctionRegistry maps countmv / summv / minmv
    / maxmv / avgmv to the Count / Sum / Min / Max / Avg functions (AggregationFunctionRegistry.java:76-80)."""
    from .broker import base_function
    return base_function(fn)


def _to_object(fn: str, v):
    """The in-process intermediate of one function as the reference's Serializable (query/aggregation/function/*):
    avg (sum, count) -> AvgPair, minmaxrange -> MinMaxRangePair, distinctcount -> IntOpenHashSet, percentile value
    multiset -> DoubleArrayList, HLL registers -> HyperLogLog, count / sum / min / max -> Double."""
    fn = _base_fn(fn)
    if fn == "avg":
        return AvgPair((float(v[0]), int(v[1])))
    if fn == "minmaxrange":
        return MinMaxRangePair((float(v[0]), float(v[1])))
    if fn == "distinctcount":
        return set(int(x) for x in v)
    if fn in ("distinctcounthll", "fasthll"):
        import numpy as np
        return HyperLogLogRegs(HLL.empty() if v is None else np.asarray(v, dtype=np.uint8))  # None: a fresh estimator
    if fn.startswith("percentileest"):
        return v if v is not None else QD.QuantileDigest()
    if fn.startswith("percentile"):
        out = []
        for value, count in v:
            out += [float(value)] * int(count)
        return out
    return float(v)


def _from_object(fn: str, o):
    fn = _base_fn(fn)
    if fn == "avg":
        return (float(o[0]), int(o[1]))
    if fn == "minmaxrange":
        return (float(o[0]), float(o[1]))
    if fn == "distinctcount":
        return set(o)
    if fn in ("distinctcounthll", "fasthll"):
        return o.regs
    if fn.startswith("percentileest"):
        return o
    if fn.startswith("percentile"):
        hist: Dict[float, int] = {}
        for x in o:
            hist[x] = hist.get(x, 0) + 1
        return sorted(hist.items())
    if fn == "count":
        return int(o)
    return float(o)


def response_to_datatable(broker_request: dict, resp) -> bytes:
    """Server side: IntermediateResultsBlock.getDataTable (+ attachMetadataToDataTable); exception-only responses are
    a schema-less table carrying their "Exception<code>" metadata (getExceptionsDataTable)."""
    from .broker import function_name
    aggs = broker_request["aggregations"]
    if resp.aggregation is not None:
        types = ["LONG" if _base_fn(a["fn"]) == "count" else
                 ("DOUBLE" if _base_fn(a["fn"]) in ("sum", "min", "max") else "OBJECT") for a in aggs]
        dt = DataTable([function_name(a) for a in aggs], types)
        dt.rows.append([int(v) if t == "LONG" else (float(v) if t == "DOUBLE" else _to_object(a["fn"], v))
                        for a, t, v in zip(aggs, types, resp.aggregation)])
    elif resp.group_by is not None:
        dt = DataTable(["functionName", "GroupByResultMap"], ["STRING", "OBJECT"])
        for a, m in zip(aggs, resp.group_by):
            dt.rows.append([function_name(a), {k: _to_object(a["fn"], v) for k, v in m.items()}])
    else:
        dt = DataTable()
    # attachMetadataToDataTable runs for exception-only tables too (IntermediateResultsBlock.java:163-178)
    st = list(resp.stats) if resp.stats is not None else [0, 0, 0, 0]
    dt.metadata[NUM_DOCS_SCANNED] = str(int(st[0]))
    dt.metadata[NUM_ENTRIES_SCANNED_IN_FILTER] = str(int(st[1]))
    dt.metadata[NUM_ENTRIES_SCANNED_POST_FILTER] = str(int(st[2]))
    dt.metadata[TOTAL_DOCS] = str(int(st[3]))
    for code, msg in resp.exceptions.items():
        dt.metadata[EXCEPTION_KEY + str(code)] = msg
    return dt.to_bytes()


def datatable_to_response(broker_request: dict, b: bytes):
    """Broker side: the DataTable read back into the InstanceResponse the reduce consumes."""
    from .broker import InstanceResponse
    dt = DataTable.from_bytes(b)
    resp = InstanceResponse()
    for k, v in dt.metadata.items():
        if k.startswith(EXCEPTION_KEY):
            resp.exceptions[int(k[len(EXCEPTION_KEY):])] = v
    resp.stats = [int(dt.metadata.get(k, 0)) for k in (NUM_DOCS_SCANNED, NUM_ENTRIES_SCANNED_IN_FILTER,
                                                       NUM_ENTRIES_SCANNED_POST_FILTER, TOTAL_DOCS)]
    if not dt.columns:
        return resp
    aggs = broker_request["aggregations"]
    if dt.columns == ["functionName", "GroupByResultMap"]:
        resp.group_by = [{k: _from_object(a["fn"], v) for k, v in row[1].items()} for a, row in zip(aggs, dt.rows)]
    else:
        resp.aggregation = [_from_object(a["fn"], v) for a, v in zip(aggs, dt.rows[0])]
    return resp
