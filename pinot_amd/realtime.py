"""Realtime (mutable) segments, SURVEY §8(f) rank 4: the query side of a consuming segment.

The reference indexes stream rows into a RealtimeSegmentImpl (core/realtime/impl/RealtimeSegmentImpl.java:185-334):
every column is dictionary-encoded by a mutable dictionary that numbers values in arrival order
(realtime/impl/dictionary/MutableDictionaryReader.java:36-41, {Int,Long,Float,Double,String}MutableDictionary), the
forward index holds one int dictId per doc (FixedByteSingleColumnSingleValueReaderWriter), inverted-index columns keep
one growing bitmap per dictId (realtime/impl/invertedIndex/DimensionInvertertedIndex.java), and queries see the docs
indexed so far (docIdSearchableOffset).  Its data source reports isSorted() false and hasInvertedIndex() per the
configured columns (realtime/impl/datasource/RealtimeColumnDataSource.java:140-152), and RANGE predicates are evaluated
by scanning the mutable dictionary (RangeRealtimeDictionaryPredicateEvaluator.java:34-75).

Here :class:`RealtimeSegment` keeps the same host structures (arrival-order dictionaries, per-doc dictIds) and, for the
GPU path, a native mutable segment (pgx_mutable_*, include/pgx.h): every doc's arrival-order dictIds live in HBM and
only the docs indexed since the last query cross PCIe (O(new rows)); when a dictionary grew, its sorted form and the
arrival -> sorted id map go down (O(cardinality)); the library re-packs the forward indexes on the device into the
shape RealtimeSegmentConverter gives an immutable segment (sorted dictionaries, unsorted fixed-bit forward indexes) and
keeps the configured inverted columns' bitmap-filter semantics, evaluated by scanning.  No host pass over the rows per
query.  The value sets every predicate selects are the realtime evaluators' (``oracle.pinot_oracle`` restates both and
the tests compare them), so a query answers exactly what the reference answers on the consuming segment.
:meth:`RealtimeSegment.snapshot` still builds the whole converter-shaped v1 segment on the host (the CPU tests use it).
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

    def _sorted_dictionary(self, c: str):
        """(sorted v1 dictionary bytes, entry width, arrival -> sorted id map, sorted values) of column c's mutable
        dictionary: SegmentDictionaryCreator's order (numbers ascending; strings by Java compareTo of the '\\0'-padded
        values, so padded and raw order agree)."""
        t = self.schema[c][0]
        vals = self.dictionaries[c].values
        if t == "STRING":
            width = max([1] + [len(v.encode("utf-8")) for v in vals])
            order = sorted(range(len(vals)), key=lambda i: [ord(ch) for ch in vals[i]])
            svals = [vals[i] for i in order]
            data = b"".join(v.encode("utf-8") + S.DEFAULT_PAD.encode() * (width - len(v.encode("utf-8"))) for v in svals)
        else:
            arr = np.asarray(vals, dtype=_NP[t])
            order = np.argsort(arr, kind="stable")
            svals = arr[order]
            data = svals.astype(S._DICT_NP[t]).tobytes()
            width = int(S._DICT_NP[t][-1])
        remap = np.empty(len(vals), dtype=np.int32)
        remap[np.asarray(order, dtype=np.int64)] = np.arange(len(vals), dtype=np.int32)
        return data, width, remap, svals

    def device_segment(self, ctx):
        """The docs indexed so far as a queryable segment in HBM (engine.IndexSegment over pgx_mutable_snapshot).  Only
        the docs indexed since the previous call are sent, and a dictionary only when it grew; the snapshot is re-made
        only when something changed."""
        import ctypes as C

        from pinot_amd import engine as E
        from pinot_amd import native as N
        L = N.lib()
        n = self.num_docs_indexed
        if n == 0:
            raise ValueError("realtime segment %s has no docs yet" % self.name)
        names = list(self.schema)
        if getattr(self, "_mut", None) is None or self._mut_ctx is not ctx:
            self._release_device()
            cols = (N.MutableColumn * len(names))()
            keep = []
            for i, c in enumerate(names):
                t, sv, _ = self.schema[c]
                b = c.encode()
                keep.append(b)
                cols[i].name = b
                cols[i].data_type = {"INT": N.PGX_INT, "LONG": N.PGX_LONG, "FLOAT": N.PGX_FLOAT, "DOUBLE": N.PGX_DOUBLE,
                                     "STRING": N.PGX_STRING}[t]
                cols[i].is_multi_value = int(not sv)
                cols[i].has_inverted = int(c in self.inverted)
            h = C.c_void_p()
            N.check(L.pgx_mutable_create(ctx.handle, self.name.encode(), self.capacity, len(names), cols, C.byref(h)))
            self._mut, self._mut_ctx, self._synced = h, ctx, 0
            self._dict_card = {c: 0 for c in names}
        changed = False
        if self._synced < n:  # the new docs' arrival-order dictIds (and value counts of multi-value columns)
            lo = self._synced
            arrs, counts = [], []
            for c in names:
                ids = self._ids[c][lo:n]
                if self.schema[c][1]:
                    arrs.append(np.asarray(ids, dtype=np.int32))
                    counts.append(None)
                else:
                    arrs.append(np.asarray([x for doc in ids for x in doc], dtype=np.int32))
                    counts.append(np.asarray([len(doc) for doc in ids], dtype=np.int32))
            idp = (C.c_void_p * len(names))(*[a.ctypes.data for a in arrs])
            cnp = (C.c_void_p * len(names))(*[x.ctypes.data if x is not None else None for x in counts])
            N.check(L.pgx_mutable_append(self._mut, n - lo, idp, cnp))
            self.docs_sent = getattr(self, "docs_sent", 0) + (n - lo)  # every doc crosses PCIe once
            self._synced = n
            changed = True
        for i, c in enumerate(names):  # dictionaries that grew: sorted form + arrival -> sorted map
            card = self.dictionaries[c].length()
            if card != self._dict_card[c]:
                data, width, remap, _ = self._sorted_dictionary(c)
                N.check(L.pgx_mutable_set_dictionary(self._mut, i, card, data, len(data), width, 0, remap.ctypes.data))
                self._dict_card[c] = card
                changed = True
        if getattr(self, "_dev", None) is None or changed:
            if getattr(self, "_dev", None) is not None:
                self._dev.destroy()
            h = C.c_void_p()
            N.check(L.pgx_mutable_snapshot(self._mut, C.byref(h)))
            self._dev = E.IndexSegment.from_handle(ctx, self._metadata(), h)
        return self._dev

    def _metadata(self) -> S.SegmentData:
        """Column metadata of the snapshot for the host side of the engine (types, sorted dictionaries for key rendering
        and predicate values); the bytes themselves live in the library."""
        n = self.num_docs_indexed
        seg = S.SegmentData(self.name, n, n)
        for c, (t, sv, ft) in self.schema.items():
            data, width, _, _ = self._sorted_dictionary(c)
            card = self.dictionaries[c].length()
            ct = {"METRIC": "METRIC", "TIME": "TIME"}.get(ft, "DIMENSION")
            col = S.Column(c, t, ct, card, S.num_bits(card), n, n, False, c in self.inverted, data, width, None, None,
                           None, S.DEFAULT_PAD)
            if not sv:
                col.is_mv = True
                col.total_entries = sum(len(x) for x in self._ids[c])
                col.max_mv = self.max_mv[c]
            seg.columns[c] = col
        return seg

    def _release_device(self):
        from pinot_amd import native as N
        if getattr(self, "_dev", None) is not None:
            self._dev.destroy()
            self._dev = None
        if getattr(self, "_mut", None) is not None:
            N.lib().pgx_mutable_release(self._mut)
            self._mut = None

    def __del__(self):
        try:
            self._release_device()
        except Exception:
            pass
