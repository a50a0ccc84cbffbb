"""Realtime (mutable) segments, SURVEY §8(f) rank 4: the query side of a consuming segment.

The reference indexes stream rows into a RealtimeSegmentImpl (core/realtime/impl/RealtimeSegmentImpl.java:185-334):
every column is dictionary-encoded by a mutable dictionary that numbers values in arrival order
(realtime/impl/dictionary/MutableDictionaryReader.java:36-41, {Int,Long,Float,Double,String}MutableDictionary), the
forward index holds one int dictId per doc (FixedByteSingleColumnSingleValueReaderWriter), inverted-index columns keep
one growing bitmap per dictId (realtime/impl/invertedIndex/DimensionInvertertedIndex.java), and queries see the docs
indexed so far (docIdSearchableOffset).  Its data source reports isSorted() false and hasInvertedIndex() per the
configured columns (realtime/impl/datasource/RealtimeColumnDataSource.java:140-152), and RANGE predicates are evaluated
by scanning the mutable dictionary (RangeRealtimeDictionaryPredicateEvaluator.java:34-75).

Here :class:`RealtimeSegment` keeps the same host structures (arrival-order dictionaries, per-doc dictIds, per-dictId
doc lists) and stages a snapshot of the docs indexed so far for the GPU path the way RealtimeSegmentConverter turns a
consuming segment into an immutable one: each dictionary sorted, the dictIds remapped, a fixed-bit forward index (never
a sorted one: the realtime data source is unsorted) and the bitmap inverted index of the configured columns.  The
value sets every predicate selects are the realtime evaluators' (``oracle.pinot_oracle`` restates both and the tests
compare them), so a query answers exactly what the reference answers on the consuming segment.  The snapshot is cached
until the next :meth:`RealtimeSegment.index`.
"""
from typing import Dict, List, Sequence, Tuple

import numpy as np

from pinot_amd import segment as S

_NP = {"INT": np.int32, "LONG": np.int64, "FLOAT": np.float32, "DOUBLE": np.float64}


class MutableDictionary:
    """MutableDictionaryReader + the typed mutable dictionaries: ids in first-arrival order, min / max tracked
    (IntMutableDictionary.java:31-97)."""

    def __init__(self, data_type: str):
        self.data_type = data_type
        self.values: List = []
        self._ids: Dict = {}
        self.min = None
        self.max = None

    def _coerce(self, raw):
        if self.data_type == "STRING":
            return str(raw)
        if self.data_type in ("INT", "LONG"):
            v = int(raw) if not isinstance(raw, str) else int(raw.strip())
            if self.data_type == "INT" and not -(1 << 31) <= v < (1 << 31):
                raise ValueError("NumberFormatException: value out of int range: %r" % (raw,))
            return v
        v = float(raw)
        return float(np.float32(v)) if self.data_type == "FLOAT" else v

    def index(self, raw) -> None:
        """index(Object): addToDictionaryBiMap + updateMinMax, for a value or an Object[] of values."""
        for r in (raw if isinstance(raw, (list, tuple, np.ndarray)) else [raw]):
            v = self._coerce(r)
            if v not in self._ids:
                self._ids[v] = len(self.values)
                self.values.append(v)
            if self.min is None or v < self.min:
                self.min = v
            if self.max is None or v > self.max:
                self.max = v

    def index_of(self, raw) -> int:
        """indexOf: the arrival-order id, -1 when absent (getIndexOfFromBiMap)."""
        return self._ids.get(self._coerce(raw), -1)

    def length(self) -> int:
        return len(self.values)


class RealtimeSegment:
    """RealtimeSegmentImpl's indexing and query-visible state.

    ``schema``: {column: (data_type, single_value, field_type)} with field_type DIMENSION / METRIC / TIME.
    ``inverted``: the table's invertedIndexColumns (DIMENSION / METRIC / TIME inverted indexes, :132-157)."""

    def __init__(self, name: str, schema: Dict[str, Tuple[str, bool, str]], capacity: int,
                 inverted: Sequence[str] = ()):
        self.name = name
        self.schema = dict(schema)
        self.capacity = int(capacity)
        self.inverted = set(inverted)
        self.dictionaries = {c: MutableDictionary(t) for c, (t, _, _) in self.schema.items()}
        self._ids: Dict[str, list] = {c: [] for c in self.schema}  # per doc: dictId (SV) or dictId list (MV)
        self.max_mv = {c: 0 for c, (_, sv, _) in self.schema.items() if not sv}
        self.num_docs_indexed = 0
        self.rows_dropped = 0
        self._snap = None

    def index(self, row: Dict) -> bool:
        """index(GenericRow) (:185-334): a row with a null in any column is dropped (counted, still returns true);
        otherwise every value enters its dictionary, the doc gets the next docId, and the return value says whether the
        segment can take more rows (numDocsIndexed < capacity)."""
        if any(row.get(c) is None for c in self.schema):
            self.rows_dropped += 1
            return True
        for c, (_, sv, _) in self.schema.items():
            v = row[c]
            if not sv and len(v) == 0:
                raise ValueError("column %s: a multi-value doc needs at least one value here (the v1 MV forward "
                                 "index this snapshot writes has no empty docs)" % c)
            self.dictionaries[c].index(v)
            if not sv:
                self.max_mv[c] = max(self.max_mv[c], len(v))
        for c, (_, sv, _) in self.schema.items():
            d = self.dictionaries[c]
            self._ids[c].append(d.index_of(row[c]) if sv else [d.index_of(x) for x in row[c]])
        self.num_docs_indexed += 1
        self._snap = None
        return self.num_docs_indexed < self.capacity

    @property
    def num_docs(self) -> int:
        """Docs visible to queries (docIdSearchableOffset + 1)."""
        return self.num_docs_indexed

    def arrival_ids(self, column: str):
        """The forward index as the reference holds it: arrival-order dictIds per doc (a list per doc for MV)."""
        return self._ids[column]

    def snapshot(self) -> S.SegmentData:
        """The docs indexed so far as an immutable v1 segment (RealtimeSegmentConverter's shape): per column the
        dictionary sorted (strings by Java compareTo, padded with '\\0' so padded and raw order agree), dictIds
        remapped, a fixed-bit forward index (unsorted even when the ids happen to ascend), and the inverted index of
        the configured columns."""
        if self._snap is not None:
            return self._snap
        n = self.num_docs_indexed
        if n == 0:
            raise ValueError("realtime segment %s has no docs yet" % self.name)
        cols = []
        for c, (t, sv, ft) in self.schema.items():
            d = self.dictionaries[c]
            ct = {"METRIC": "METRIC", "TIME": "TIME"}.get(ft, "DIMENSION")
            if sv:
                vals = [d.values[i] for i in self._ids[c]]
                raw = np.array(vals, dtype=object) if t == "STRING" else np.asarray(vals, dtype=_NP[t])
                cols.append(S.make_column(c, raw, data_type=t, column_type=ct, inverted=c in self.inverted,
                                          pad=S.DEFAULT_PAD, force_unsorted=True))
            else:
                if t == "STRING":
                    raise ValueError("column %s: multi-value STRING columns are not staged" % c)
                docs = [np.asarray([d.values[i] for i in ids], dtype=_NP[t]) for ids in self._ids[c]]
                cols.append(S.make_mv_column(c, docs, data_type=t, column_type=ct, inverted=c in self.inverted))
        self._snap = S.make_segment(self.name, cols)
        return self._snap

    def device_segment(self, ctx):
        """The snapshot staged into HBM (engine.IndexSegment), restaged only after new rows arrive."""
        from pinot_amd import engine as E
        snap = self.snapshot()
        if getattr(self, "_dev", None) is None or self._dev_for is not snap:
            if getattr(self, "_dev", None) is not None:
                self._dev.destroy()
            self._dev = E.IndexSegment(ctx, snap)
            self._dev_for = snap
        return self._dev
