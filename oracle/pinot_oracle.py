"""CPU ORACLE for the pinot-core segment query hot path -- TEST INFRASTRUCTURE ONLY.

This module is a literal CPU restatement of the reference's (Java) per-segment query algorithm.
It exists to CHECK the MI355X path: only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import it, and never as the thing measured or shipped.  The product path
(pinot_amd + libpgx.so) never imports anything from oracle/.

Parity of this oracle is PINNED by the reference's own known-answer tests, frozen as fixtures in
tests/golden/ (see tests/golden/make_golden.py and tests/test_oracle_golden.py):
  * AggregationSingleValueQueriesTest.java:43-221 on test_data-sv.avro (all 8 aggregation /
    group-by cases, with and without the 5-clause filter, including ExecutionStatistics such as
    numEntriesScannedInFilter=84134, which depends on the exact iterator algebra restated below);
  * QueryExecutorTest.java:97-200 on simpleData200001.avro (2 segments, combine);
  * the Java-written v1 segment starTreeSegment.tar.gz (fixed-bit MSB-first decode, dictionaries).

All functions cite the reference file:line they restate.  Paths are relative to
pinot-core/src/main/java/com/linkedin/pinot/core/.
"""
from __future__ import annotations

import heapq
import math
import struct
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

EOF = -2147483648  # Constants.EOF (core/common/Constants.java) == Integer.MIN_VALUE
INT_MAX = 2147483647
INT_MIN = -2147483648
MAX_DOC_PER_CALL = 10000  # plan/DocIdSetPlanNode.java:33
GROUP_BY_BLOCK = 5000  # plan/AggregationGroupByPlanNode.java:53
MAX_INITIAL_RESULT_HOLDER_CAPACITY = 10000  # operator/aggregation/ResultHolderFactory.java:33
LONG_MAX = (1 << 63) - 1


# ------------------------------------------------------------------------------------------------
# a-1: fixed-bit forward index decode
# ------------------------------------------------------------------------------------------------
def get_num_of_bits(card: int) -> int:
    """SingleValueUnsortedForwardIndexCreator.getNumOfBits (segment/creator/impl/fwd/...:48-57)."""
    if card < 2:
        return 1
    ret = int(math.ceil(math.log(card) / math.log(2)))
    return 1 if ret == 0 else ret


def _s32(x: int) -> int:
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x & 0x80000000 else x


def read_int(buf: bytes, nr_bytes: int, start_bit: int, end_bit: int) -> int:
    """Literal restatement of PinotDataCustomBitSet.readInt (util/PinotDataCustomBitSet.java:122-155).
    buf is the big-endian forward-index byte buffer."""
    bit_length = end_bit - start_bit
    if bit_length < 16 and end_bit + 32 < nr_bytes * 8:
        byte_pos = start_bit // 8
        bit_off = start_bit % 8
        shift = 32 - (bit_off + bit_length)
        int_value = _s32(int.from_bytes(buf[byte_pos:byte_pos + 4], "big"))
        mask = (1 << bit_length) - 1
        return (int_value >> shift) & mask  # Java '>>' is arithmetic
    byte_pos = start_bit >> 3
    start_off = start_bit & 7
    s = start_off + bit_length
    end_off = (8 - (s & 7)) & 7
    nbytes = (s + 7) >> 3
    number = 0
    i = -1
    while True:
        number |= buf[byte_pos] & 0xFF
        i += 1
        byte_pos += 1
        if i == nbytes - 1:
            break
        number <<= 8
    number >>= end_off
    number &= (0xFFFFFFFF >> (32 - bit_length))
    return _s32(number)


def decode_fixed_bit(buf: bytes, num_rows: int, bits: int) -> np.ndarray:
    """v1 FixedBitSingleValueReader.getInt for every row (io/reader/impl/v1/FixedBitSingleValueReader.java:30-58,
    FixedBitSingleValueMultiColReader.java:87-130): row r occupies bits [r*b, r*b+b)."""
    n = len(buf)
    return np.array([read_int(buf, n, r * bits, r * bits + bits) for r in range(num_rows)], dtype=np.int64)


def decode_fixed_bit_fast(buf: bytes, num_rows: int, bits: int) -> np.ndarray:
    """Vectorised equivalent of decode_fixed_bit (checked against it in tests)."""
    a = np.frombuffer(bytes(buf) + b"\0" * 8, dtype=np.uint8)
    start = np.arange(num_rows, dtype=np.int64) * bits
    byte = start >> 3
    w = np.zeros(num_rows, dtype=np.uint64)
    for k in range(5):
        w = (w << np.uint64(8)) | a[byte + k].astype(np.uint64)
    shift = (40 - (start & 7) - bits).astype(np.uint64)
    return ((w >> shift) & np.uint64((1 << bits) - 1)).astype(np.int64)


# ------------------------------------------------------------------------------------------------
# Segment model (the oracle builds its own dictionaries from raw column values)
# ------------------------------------------------------------------------------------------------
@dataclass
class OColumn:
    name: str
    dtype: str  # INT, LONG, FLOAT, DOUBLE, STRING
    dictionary: np.ndarray  # sorted distinct values (object array of str for STRING)
    dict_ids: np.ndarray  # int64 per doc
    is_sorted: bool
    has_inverted: bool
    bits: int
    mv_ids: Optional[List[np.ndarray]] = None  # multi-value column: the dictIds of every doc (dict_ids: all values)
    realtime: bool = False  # mutable dictionary: values in arrival order (realtime/impl/dictionary/*MutableDictionary)

    @property
    def card(self) -> int:
        return len(self.dictionary)

    def _parse(self, raw: str):
        if self.dtype == "STRING":
            return raw
        if self.dtype in ("INT", "LONG"):
            return int(raw)
        return float(np.float32(float(raw))) if self.dtype == "FLOAT" else float(raw)

    def index_of(self, raw: str) -> int:
        """Dictionary.indexOf: binary search returning -(insertion)-1 when absent
        (segment/index/readers/IntDictionary.java:28-37, StringDictionary.java:37-51); on a mutable dictionary the
        arrival-order id or -1 (MutableDictionaryReader.getIndexOfFromBiMap)."""
        if self.realtime:
            v = self._parse(raw)
            hits = [i for i, x in enumerate(self.dictionary.tolist()) if x == v]
            return hits[0] if hits else -1
        if self.dtype == "STRING":
            keys = list(self.dictionary)
            v = raw
        elif self.dtype in ("INT", "LONG"):
            keys = self.dictionary
            v = int(raw)
        else:
            keys = self.dictionary
            v = float(raw)
        pos = int(np.searchsorted(np.asarray(keys, dtype=object if self.dtype == "STRING" else None), v, side="left"))
        if pos < self.card and keys[pos] == v:
            return pos
        return -(pos + 1)

    def value_as_double(self, ids: np.ndarray) -> np.ndarray:
        """Dictionary.readDoubleValues: (double) cast of the dictionary value (IntDictionary.java:50-52)."""
        return self.dictionary[ids].astype(np.float64)

    def string_of(self, dict_id: int) -> str:
        """Dictionary.get(dictId).toString() used for string group keys."""
        v = self.dictionary[dict_id]
        if self.dtype == "STRING":
            return v
        if self.dtype in ("INT", "LONG"):
            return str(int(v))
        return repr(float(v))


@dataclass
class OSegment:
    columns: Dict[str, OColumn]
    total_docs: int
    total_raw_docs: int

    @staticmethod
    def from_realtime(dictionaries: Dict[str, Tuple[str, list]], ids: Dict[str, list], num_docs: int,
                      inverted: Sequence[str] = ()) -> "OSegment":
        """A consuming segment as RealtimeSegmentImpl holds it (core/realtime/impl/RealtimeSegmentImpl.java:185-334):
        per column (data type, arrival-order dictionary values) and the per-doc arrival-order dictIds (a list per doc
        for a multi-value column); never sorted, inverted per the configured columns
        (RealtimeColumnDataSource.java:140-152)."""
        cols = {}
        for name, (dt, values) in dictionaries.items():
            dictionary = np.array(values, dtype=object) if dt == "STRING" else np.asarray(
                values, dtype=np.float64 if dt in ("FLOAT", "DOUBLE") else np.int64)
            per = ids[name][:num_docs]
            if per and isinstance(per[0], (list, tuple)):
                mv = [np.asarray(x, dtype=np.int64) for x in per]
                flat = np.concatenate(mv)
                cols[name] = OColumn(name, dt, dictionary, flat, False, name in inverted,
                                     get_num_of_bits(len(dictionary)), mv, realtime=True)
            else:
                cols[name] = OColumn(name, dt, dictionary, np.asarray(per, dtype=np.int64), False, name in inverted,
                                     get_num_of_bits(len(dictionary)), realtime=True)
        return OSegment(cols, num_docs, num_docs)

    @staticmethod
    def from_raw(raw: Dict[str, np.ndarray], inverted: Sequence[str] = (), dtypes: Dict[str, str] = None,
                 sorted_override: Dict[str, bool] = None) -> "OSegment":
        cols = {}
        n = None
        for name, vals in raw.items():
            if isinstance(vals, list) and vals and isinstance(vals[0], (list, tuple, np.ndarray)):
                # multi-value column: one dictionary over every value (SegmentDictionaryCreator), per-doc id arrays
                n = len(vals) if n is None else n
                lens = [len(v) for v in vals]
                flat = np.concatenate([np.asarray(v) for v in vals])
                dt = (dtypes or {}).get(name) or ("INT" if flat.dtype.kind in "iu" else "DOUBLE")
                dictionary, ids = np.unique(flat, return_inverse=True)
                starts = np.concatenate([[0], np.cumsum(lens)])
                per = [ids[starts[d]:starts[d + 1]].astype(np.int64) for d in range(n)]
                cols[name] = OColumn(name, dt, dictionary, ids.astype(np.int64), False, name in inverted,
                                     get_num_of_bits(len(dictionary)), per)
                continue
            vals = np.asarray(vals)
            n = len(vals) if n is None else n
            dt = (dtypes or {}).get(name)
            if dt is None:
                dt = "STRING" if vals.dtype.kind in "SUO" else ("INT" if vals.dtype.kind in "iu" else "DOUBLE")
            if dt == "STRING":
                sv = np.array([v.decode() if isinstance(v, bytes) else str(v) for v in vals], dtype=object)
                dictionary = np.array(sorted(set(sv.tolist())), dtype=object)
                lookup = {v: i for i, v in enumerate(dictionary)}
                ids = np.array([lookup[v] for v in sv], dtype=np.int64)
            else:
                dictionary, ids = np.unique(vals, return_inverse=True)
                ids = ids.astype(np.int64)
            is_sorted = bool(np.all(np.diff(ids) >= 0)) if n > 1 else True
            if sorted_override and name in sorted_override:
                is_sorted = sorted_override[name]
            cols[name] = OColumn(name, dt, dictionary, ids, is_sorted,
                                 name in inverted or is_sorted, get_num_of_bits(len(dictionary)))
        return OSegment(cols, n, n)


# ------------------------------------------------------------------------------------------------
# a-4: predicates -> dictId space
# ------------------------------------------------------------------------------------------------
def parse_range(rng: str) -> Tuple[str, str, bool, bool]:
    """RangePredicate (common/predicate/RangePredicate.java:31-57)."""
    s = rng.strip()
    lo_s, hi_s = s.split("\t\t")[0], s.split("\t\t")[1]
    lower = lo_s[1:]
    upper = hi_s[:-1]
    inc_lower = (lower == "*") if s.startswith("(") else True
    inc_upper = (upper == "*") if s.endswith(")") else True
    return lower, upper, inc_lower, inc_upper


@dataclass
class Evaluator:
    kind: str  # EQ NEQ IN NOT_IN RANGE
    match: np.ndarray  # bool[card]: apply(dictId)
    matching_ids: np.ndarray
    non_matching_ids: Optional[np.ndarray]
    always_false: bool


def make_evaluator(col: OColumn, leaf: dict) -> Evaluator:
    """PredicateEvaluatorProvider (operator/filter/predicate/PredicateEvaluatorProvider.java:31-54) and the
    Equals/NotEquals/In/NotIn/RangeOffline evaluators in the same package."""
    op = leaf["op"]
    card = col.card
    m = np.zeros(card, dtype=bool)
    if op == "RANGE" and col.realtime:
        # RangeRealtimeDictionaryPredicateEvaluator.java:34-75: '*' takes the dictionary's min / max value, then every
        # dictId whose value lies in the range (MutableDictionary.inRange, e.g. IntMutableDictionary.java:143-174)
        lower, upper, inc_lo, inc_hi = parse_range(leaf["values"][0])
        if card:
            vals = col.dictionary.tolist()
            lo = min(vals) if lower == "*" else col._parse(lower)
            hi = max(vals) if upper == "*" else col._parse(upper)
            for i, v in enumerate(vals):
                ok = (v >= lo if inc_lo else v > lo) and (v <= hi if inc_hi else v < hi)
                m[i] = ok
        ids = np.nonzero(m)[0]
        return Evaluator(op, m, ids, None, len(ids) == 0)
    if op == "RANGE":
        lower, upper, inc_lo, inc_hi = parse_range(leaf["values"][0])
        # RangeOfflineDictionaryPredicateEvaluator.java:30-65
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
        if end >= start:
            m[start:end + 1] = True
        ids = np.nonzero(m)[0]
        return Evaluator(op, m, ids, None, (end - start + 1) <= 0)
    if op == "EQ":
        i = col.index_of(leaf["values"][0])
        if i >= 0:
            m[i] = True
        return Evaluator(op, m, np.nonzero(m)[0], None, i < 0)
    if op == "IN":
        for v in leaf["values"]:
            i = col.index_of(v)
            if i >= 0:
                m[i] = True
        ids = np.nonzero(m)[0]
        return Evaluator(op, m, ids, None, len(ids) == 0)
    if op == "NEQ":
        i = col.index_of(leaf["values"][0])
        m[:] = True
        non = np.array([i] if i >= 0 else [], dtype=np.int64)
        if i >= 0:
            m[i] = False
        # NotEqualsPredicateEvaluator.alwaysFalse (:102-104): every dictId excluded
        return Evaluator(op, m, np.nonzero(m)[0], non, len(non) == card)
    if op == "NOT_IN":
        m[:] = True
        non = set()
        for v in leaf["values"]:
            i = col.index_of(v)
            if i >= 0:
                non.add(i)
        for i in non:
            m[i] = False
        # NotInPredicateEvaluator.alwaysFalse (:98-100): the excluded id set covers the dictionary
        return Evaluator(op, m, np.nonzero(m)[0], np.array(sorted(non), dtype=np.int64), len(non) == card)
    raise ValueError(op)


# ------------------------------------------------------------------------------------------------
# a-5..a-12: literal restatement of the filter DocIdSet / iterator algebra (for ExecutionStatistics)
# ------------------------------------------------------------------------------------------------
class _ScanSet:
    """ScanBasedSingleValueDocIdSet + SVScanDocIdIterator (operator/docidsets/ScanBasedSingleValueDocIdSet.java:30-85,
    operator/dociditerators/SVScanDocIdIterator.java:40-155)."""
    kind = "scan"

    def __init__(self, col: OColumn, ev: Evaluator, start: int, end: int):
        self.ids = col.dict_ids
        self.match = ev.match
        self.ev = ev
        self.scanned = 0
        # The iterator's alwaysFalse EOF state (:42-45) is overwritten by the DocIdSet's setStartDocId/setEndDocId
        # (ScanBasedFilterOperator.java:81-87); only applyAnd re-checks alwaysFalse.
        self._set_start(start)
        self.end = end

    def _set_start(self, s):
        self.cur = s - 1
        self.start = s

    # FilterBlockDocIdSet interface
    def min_doc(self):
        return self.start

    def max_doc(self):
        return self.end

    def set_start(self, s):
        self._set_start(s)

    def set_end(self, e):
        self.end = e

    def iterator(self):
        return self

    def entries(self):
        return self.scanned

    # iterator
    def is_match(self, doc):
        if self.cur == EOF:
            return False
        self.scanned += 1
        return bool(self.match[self.ids[doc]])

    def advance(self, target):
        if self.cur == EOF:
            return EOF
        if target < self.start:
            target = self.start
        elif target > self.end:
            self.cur = EOF
        if self.cur >= target:
            return self.cur
        self.cur = target - 1
        return self.next()

    def next(self):
        if self.cur == EOF:
            return EOF
        n = len(self.ids)
        while self.cur + 1 < n and self.cur < self.end:
            self.cur += 1
            self.scanned += 1
            if self.match[self.ids[self.cur]]:
                return self.cur
        self.cur = EOF
        return EOF

    def apply_and(self, answer: List[int]) -> List[int]:
        res = []
        if self.ev.always_false:
            return res
        doc = -1
        it = iter(answer)
        for d in it:
            if not doc < self.end:
                break
            doc = d
            if doc >= self.start:
                self.scanned += 1
                if self.match[self.ids[doc]]:
                    res.append(doc)
        return res


class _ListIter:
    """BitmapDocIdIterator (clipped, operator/dociditerators/BitmapDocIdIterator.java:40-84) or
    RangelessBitmapDocIdIterator (:30-80) over a sorted doc list."""

    def __init__(self, docs: Sequence[int], start=None, end=None):
        self.docs = docs
        self.pos = 0
        self.cur = -1
        self.start = start
        self.end = end

    def _raw_next(self):
        if self.pos >= len(self.docs):
            return None
        v = self.docs[self.pos]
        self.pos += 1
        return v

    def next(self):
        if self.cur == EOF or self.pos >= len(self.docs):
            self.cur = EOF
            return EOF
        self.cur = self._raw_next()
        if self.start is not None:
            while self.cur < self.start and self.pos < len(self.docs):
                self.cur = self._raw_next()
            if self.cur < self.start or self.end < self.cur:
                self.cur = EOF
        return self.cur

    def advance(self, target):
        if self.cur == target:
            return self.cur
        c = self.next()
        while c < target and c != EOF:
            c = self.next()
        return c


class _BitmapSet:
    """BitmapDocIdSet (operator/docidsets/BitmapDocIdSet.java:55-145)."""
    kind = "bitmap"

    def __init__(self, col: OColumn, ev: Evaluator, start: int, end: int):
        if ev.kind in ("NEQ", "NOT_IN"):
            ids, exclusion = ev.non_matching_ids, True
        else:
            ids, exclusion = ev.matching_ids, False
        docs = np.nonzero(np.isin(col.dict_ids, ids))[0]
        if exclusion:
            inside = np.zeros(len(col.dict_ids), dtype=bool)
            inside[start:end + 1] = True
            m = np.zeros(len(col.dict_ids), dtype=bool)
            m[docs] = True
            m[inside] = ~m[inside]
            docs = np.nonzero(m)[0]
        self.answer = docs.tolist()
        self.start, self.end = start, end

    def min_doc(self):
        return self.start

    def max_doc(self):
        return self.end

    def set_start(self, s):
        self.start = s

    def set_end(self, e):
        self.end = e

    def iterator(self):
        return _ListIter(self.answer, self.start, self.end)

    def entries(self):
        return 0


class _SortedIter:
    """SortedDocIdIterator (operator/dociditerators/SortedDocIdIterator.java:35-100)."""

    def __init__(self, pairs):
        self.pairs = pairs
        self.pp = 0
        self.cur = -1

    def advance(self, target):
        P = self.pairs
        if self.pp == len(P) or target > P[-1][1]:
            self.pp = len(P)
            self.cur = EOF
            return EOF
        if self.cur >= target:
            return self.cur
        while self.pp < len(P):
            if P[self.pp][0] > target:
                self.cur = P[self.pp][0]
                break
            elif P[self.pp][0] <= target <= P[self.pp][1]:
                self.cur = target
                break
            self.pp += 1
        if self.pp == len(P):
            self.cur = EOF
        return self.cur

    def next(self):
        P = self.pairs
        if self.pp == len(P) or self.cur > P[-1][1]:
            self.pp = len(P)
            self.cur = EOF
            return EOF
        self.cur += 1
        if self.pp < len(P) and self.cur > P[self.pp][1]:
            self.pp += 1
            self.cur = EOF if self.pp == len(P) else P[self.pp][0]
        elif self.cur < P[self.pp][0]:
            self.cur = P[self.pp][0]
        return self.cur


class _EmptyIter:
    def next(self):
        return EOF

    def advance(self, t):
        return EOF


class _SortedSet:
    """SortedInvertedIndexBasedFilterOperator.nextFilterBlock (operator/filter/SortedInvertedIndexBasedFilterOperator.java:71-193)
    + SortedDocIdSet (operator/docidsets/SortedDocIdSet.java:30-100)."""
    kind = "sorted"

    def __init__(self, col: OColumn, ev: Evaluator, start: int, end: int):
        ids = col.dict_ids
        # SortedInvertedIndexReader.getMinMaxRangeFor: per-dictId inclusive [first,last] doc
        first = np.full(col.card, -1, dtype=np.int64)
        last = np.full(col.card, -2, dtype=np.int64)
        u, f = np.unique(ids, return_index=True)
        first[u] = f
        u2, l2 = np.unique(ids[::-1], return_index=True)
        last[u2] = len(ids) - 1 - l2
        additive = ev.kind in ("EQ", "IN", "RANGE")
        d = np.sort(ev.matching_ids if additive else ev.non_matching_ids)
        pairs = []
        if len(d):
            def clip(p):  # IntRanges.clip (operator/filter/IntRanges.java)
                return [max(p[0], start), min(p[1], end)]

            def invalid(p):
                return p[1] < p[0]

            lastp = clip([int(first[d[0]]), int(last[d[0]])])
            for di in d[1:]:
                cur = clip([int(first[di]), int(last[di])])
                if invalid(lastp):
                    lastp = cur
                    continue
                if cur[0] <= lastp[1] + 1 and lastp[0] <= cur[1] + 1:  # rangesAreMergeable
                    lastp = [min(lastp[0], cur[0]), max(lastp[1], cur[1])]
                else:
                    if not invalid(lastp):
                        pairs.append(lastp)
                    lastp = cur
            if not invalid(lastp):
                pairs.append(lastp)
        if not additive:
            newp = []
            if not pairs:
                newp.append([start, end])
            else:
                r = [start, pairs[0][0] - 1]
                if r[1] >= r[0]:
                    newp.append(r)
                for a, b in zip(pairs[:-1], pairs[1:]):
                    r = [a[1] + 1, b[0] - 1]
                    if r[1] >= r[0]:
                        newp.append(r)
                r = [pairs[-1][1] + 1, end]
                if r[1] >= r[0]:
                    newp.append(r)
            pairs = newp
        self.pairs = pairs

    def min_doc(self):
        return self.pairs[0][0] if self.pairs else 0

    def max_doc(self):
        return self.pairs[-1][1] if self.pairs else 0

    def set_start(self, s):
        pass

    def set_end(self, e):
        pass

    def iterator(self):
        return _SortedIter(self.pairs) if self.pairs else _EmptyIter()

    def entries(self):
        return 0

    def docs(self):
        out = []
        for a, b in self.pairs:
            out.extend(range(a, b + 1))
        return out


class _AndIter:
    """AndDocIdIterator (operator/dociditerators/AndDocIdIterator.java:38-122)."""

    def __init__(self, iters, scan_flags):
        idx = sum(1 for f in scan_flags if f == "index")
        sc = sum(1 for f in scan_flags if f == "scan")
        if idx > 0 and sc > 0:
            self.has_scan = True
            self.iters = [it for it, f in zip(iters, scan_flags) if f != "scan"]
            self.scans = [it for it, f in zip(iters, scan_flags) if f == "scan"]
        else:
            self.has_scan = False
            self.iters = list(iters)
            self.scans = []
        self.cur = -1
        self.cmax = -1

    def advance(self, target):
        if self.cur == EOF:
            return EOF
        if self.cur >= target:
            return self.cur
        self.cmax = target - 1
        return self.next()

    def next(self):
        if self.cur == EOF:
            return EOF
        self.cmax += 1
        i = 0
        n = len(self.iters)
        while i < n:
            p = self.iters[i].advance(self.cmax)
            if p == EOF:
                self.cmax = EOF
                break
            if p > self.cmax:
                self.cmax = p
                if i > 0:
                    i = -1
            if self.has_scan and i == n - 1:
                for s in self.scans:
                    if not s.is_match(self.cmax):
                        i = -1
                        self.cmax += 1
                        break
            i += 1
        self.cur = self.cmax
        return self.cur


class _OrIter:
    """OrDocIdIterator (operator/dociditerators/OrDocIdIterator.java:30-153)."""

    def __init__(self, iters, lo, hi):
        self.iters = iters
        self.inq = [False] * len(iters)
        self.q = []  # heap of (doc, idx)
        self.cur = -1
        self.lo, self.hi = lo, hi

    def advance(self, target):
        if self.cur == EOF:
            return EOF
        if target < self.lo:
            target = self.lo
        elif target > self.hi:
            self.cur = EOF
            return EOF
        keep = []
        for d, i in self.q:
            if d < target:
                self.inq[i] = False
            else:
                keep.append((d, i))
        self.q = keep
        heapq.heapify(self.q)
        for i, it in enumerate(self.iters):
            if not self.inq[i]:
                nd = it.advance(target)
                if nd != EOF:
                    heapq.heappush(self.q, (nd, i))
                self.inq[i] = True
        self.cur = self.q[0][0] if self.q else EOF
        return self.cur

    def next(self):
        if self.cur == EOF:
            return EOF
        while self.q and self.q[0][0] <= self.cur:
            d, i = heapq.heappop(self.q)
            self.inq[i] = False
        self.cur += 1
        for i, it in enumerate(self.iters):
            if not self.inq[i]:
                nd = it.advance(self.cur)
                if nd != EOF:
                    heapq.heappush(self.q, (nd, i))
                self.inq[i] = True
        self.cur = self.q[0][0] if self.q else EOF
        return self.cur


def intersect_sorted_range_sets(sets: List[List[List[int]]]) -> List[List[int]]:
    """SortedRangeIntersection.intersectSortedRangeSets (core/util/SortedRangeIntersection.java:31-120), literally:
    pointer per range set, chase the max head, emit the overlap, merge contiguous results."""
    if not sets:
        return []
    if len(sets) == 1:
        return [list(p) for p in sets[0]]
    if any(len(s) == 0 for s in sets):
        return []
    cur = [0] * len(sets)
    max_head, max_idx = -1, -1
    result: List[List[int]] = []
    reached_end = False
    while not reached_end:
        for i, s in enumerate(sets):
            head = s[cur[i]][0]
            if head > max_head:
                max_head, max_idx = head, i
        i = 0
        while i < len(sets):
            if i == max_idx:
                i += 1
                continue
            found = False
            restart = False
            while not found and cur[i] < len(sets[i]):
                lo, hi = sets[i][cur[i]]
                if lo <= max_head <= hi:
                    found = True
                    break
                if lo > max_head:
                    max_head, max_idx = lo, i
                    restart = True
                    break
                cur[i] += 1
            if restart:
                i = 0
                continue
            if not found:
                reached_end = True
                break
            i += 1
        if reached_end:
            break
        a, b = sets[0][cur[0]]
        inter = [a, b]
        for i in range(1, len(sets)):
            lo, hi = sets[i][cur[i]]
            inter = [max(inter[0], lo), min(inter[1], hi)]
        if result and inter[0] == result[-1][1] + 1:
            result[-1][1] = inter[1]
        else:
            result.append(inter)
        for i in range(len(sets)):
            if sets[i][cur[i]][1] == inter[1]:
                cur[i] += 1
                if cur[i] == len(sets[i]):
                    reached_end = True
                    break
    return result


class _AndSet:
    """AndBlockDocIdSet (operator/docidsets/AndBlockDocIdSet.java:49-63,146-266)."""
    kind = "and"

    def __init__(self, children):
        self.children = children
        self.lo, self.hi = INT_MIN, INT_MAX
        self.answer = None  # the `answer` FIELD (:46): it survives between iterator() calls
        self._update()

    def _update(self):
        for c in self.children:
            self.lo = max(self.lo, c.min_doc())
            self.hi = min(self.hi, c.max_doc())
        for c in self.children:
            c.set_start(self.lo)
            c.set_end(self.hi)

    def min_doc(self):
        return self.lo

    def max_doc(self):
        return self.hi

    def set_start(self, s):
        self.lo = max(self.lo, s)
        self._update()

    def set_end(self, e):
        self.hi = min(self.hi, e)
        self._update()

    def entries(self):
        return sum(c.entries() for c in self.children)

    def iterator(self):
        """fastIterator (:146-229).  The classification loop already calls iterator() on every nested operator child
        (:166-168) and the no-index branch calls it on every child again (:171-178), so an AND without sorted/bitmap
        children builds its nested operators' iterators twice; a nested AND with bitmap children but no sorted child
        then re-uses its `answer` field (:192-203), already reduced by the first call's applyAnd."""
        ranges, bitmaps, scans, rest = [], [], [], []
        for c in self.children:
            if c.kind == "sorted":
                ranges.append(c)
            elif c.kind == "bitmap":
                bitmaps.append(c)
            elif c.kind == "scan":
                scans.append(c)
            else:
                rest.append(c.iterator())
        if not bitmaps and not ranges:
            its = [c.iterator() for c in self.children]
            return _AndIter(its, [_flag(c) for c in self.children])
        if ranges:
            # SortedRangeIntersection.intersectSortedRangeSets (util/SortedRangeIntersection.java:31)
            pairs = intersect_sorted_range_sets([r.pairs for r in ranges])
            self.answer = {d for a, b in pairs for d in range(a, b + 1)}
        for i, b in enumerate(bitmaps):
            if self.answer is None:
                self.answer = set(b.answer)
            else:
                self.answer &= set(b.answer)
        answer = sorted(self.answer)
        for s in scans:
            it = s.iterator()
            res = set(it.apply_and(answer))
            answer = [d for d in answer if d in res]
        self.answer = set(answer)
        ans_it = _ListIter(answer)
        if not rest:
            return ans_it
        return _AndIter([ans_it] + rest, ["index"] + ["other"] * len(rest))


class _OrSet:
    """OrBlockDocIdSet (operator/docidsets/OrBlockDocIdSet.java:42-135)."""
    kind = "or"

    def __init__(self, children):
        self.children = children
        self.lo, self.hi = INT_MAX, INT_MIN
        self._update()

    def _update(self):
        for c in self.children:
            self.lo = min(self.lo, c.min_doc())
            self.hi = max(self.hi, c.max_doc())
        for c in self.children:
            c.set_start(self.lo)
            c.set_end(self.hi)

    def min_doc(self):
        return self.lo

    def max_doc(self):
        return self.hi

    def set_start(self, s):
        self.lo = min(self.lo, s)
        self._update()

    def set_end(self, e):
        self.hi = max(self.hi, e)
        self._update()

    def entries(self):
        return sum(c.entries() for c in self.children)

    def iterator(self):
        if any(c.kind == "bitmap" for c in self.children):
            raw, allb = [], set()
            for c in self.children:
                if c.kind == "sorted":
                    allb |= set(c.docs())
                elif c.kind == "bitmap":
                    allb |= set(c.answer)
                else:
                    raw.append(c.iterator())
            raw.append(_ListIter(sorted(allb), self.lo, self.hi))
            its = raw
        else:
            its = [c.iterator() for c in self.children]
        return _OrIter(its, self.lo, self.hi)


class _MatchAllSet:
    """MatchEntireSegmentOperator / SizeBasedDocIdIterator (operator/filter/MatchEntireSegmentOperator.java:25-44)."""
    kind = "all"

    def __init__(self, n):
        self.n = n
        self.cur = -1

    def iterator(self):
        return self

    def next(self):
        self.cur += 1
        if self.cur >= self.n:
            self.cur = EOF
        return self.cur

    def entries(self):
        return 0


def _flag(c):
    if c.kind == "scan":
        return "scan"
    if c.kind in ("bitmap", "sorted"):
        return "index"
    return "other"


_PRIORITY = {"sorted": 0, "and": 1, "bitmap": 2, "scan": 3, "or": 4}


def mv_doc_view(col: OColumn, ev: Evaluator):
    """A multi-value leaf as a per-doc predicate: the evaluators' apply(int[]) (operator/filter/predicate/
    {Equals,In,RangeOffline}PredicateEvaluator.java: ANY value matches; NotEquals / NotIn: NO value is excluded) driven
    by MVScanDocIdIterator (operator/dociditerators/MVScanDocIdIterator.java:78-121, one entry scanned per doc), or
    the bitmap of every doc holding a matching (excluded) value, flipped for NEQ / NOT_IN (BitmapBasedFilterOperator).
    Returned as a pseudo single-value column whose dictId of doc d is d, so the iterator algebra applies unchanged."""
    neg = ev.kind in ("NEQ", "NOT_IN")
    doc = np.array([bool(ev.match[v].all()) if neg else bool(ev.match[v].any()) for v in col.mv_ids], dtype=bool)
    n = len(col.mv_ids)
    pcol = OColumn(col.name, col.dtype, col.dictionary, np.arange(n, dtype=np.int64), False, col.has_inverted, col.bits)
    pev = Evaluator(ev.kind, doc, np.nonzero(doc)[0], np.nonzero(~doc)[0] if neg else None, ev.always_false)
    return pcol, pev


def build_filter(seg: OSegment, tree: Optional[dict]):
    """FilterPlanNode.constructPhysicalOperator + reorder (plan/FilterPlanNode.java:77-170)."""
    if tree is None:
        return _MatchAllSet(seg.total_raw_docs)
    start, end = 0, seg.total_raw_docs - 1
    op = tree["op"]
    if op in ("AND", "OR"):
        kids = [build_filter(seg, c) for c in tree["children"]]
        kids = sorted(kids, key=lambda k: _PRIORITY[k.kind])  # Collections.sort is stable
        return _AndSet(kids) if op == "AND" else _OrSet(kids)
    col = seg.columns[tree["column"]]
    ev = make_evaluator(col, tree)
    if col.mv_ids is not None:
        col, ev = mv_doc_view(col, ev)
    if col.has_inverted and op != "RANGE":
        if col.is_sorted:
            return _SortedSet(col, ev, start, end)
        return _BitmapSet(col, ev, start, end)
    return _ScanSet(col, ev, start, end)


def filter_docs(seg: OSegment, tree: Optional[dict]) -> Tuple[np.ndarray, int]:
    """BReusableFilteredDocIdSetOperator (operator/BReusableFilteredDocIdSetOperator.java:68-109): the ascending
    matching docIds and numEntriesScannedInFilter, via the literal iterator algebra."""
    s = build_filter(seg, tree)
    it = s.iterator()
    out = []
    while True:
        d = it.next()
        if d == EOF:
            break
        out.append(d)
    return np.array(out, dtype=np.int64), int(s.entries())


def filter_mask_vectorized(seg: OSegment, tree: Optional[dict]) -> np.ndarray:
    """Set semantics of the same filter (docs in [0,totalRawDocs) satisfying the predicate tree)."""
    n = seg.total_raw_docs
    if tree is None:
        return np.ones(n, dtype=bool)
    op = tree["op"]
    if op == "AND":
        m = np.ones(n, dtype=bool)
        for c in tree["children"]:
            m &= filter_mask_vectorized(seg, c)
        return m
    if op == "OR":
        m = np.zeros(n, dtype=bool)
        for c in tree["children"]:
            m |= filter_mask_vectorized(seg, c)
        return m
    col = seg.columns[tree["column"]]
    ev = make_evaluator(col, tree)
    if col.mv_ids is not None:
        col, ev = mv_doc_view(col, ev)
    return ev.match[col.dict_ids[:n]]


# ------------------------------------------------------------------------------------------------
# a-13..a-17, a-20: aggregation / group-by execution
# ------------------------------------------------------------------------------------------------
FN_DEFAULT = {"count": 0.0, "sum": 0.0, "min": math.inf, "max": -math.inf,
              "countmv": 0.0, "summv": 0.0, "minmv": math.inf, "maxmv": -math.inf}
MV_FUNCTIONS = ("countmv", "summv", "minmv", "maxmv", "avgmv")
EXT_FUNCTIONS = ("distinctcount", "distinctcounthll", "fasthll", "minmaxrange", "percentile50", "percentile90", "percentile95",
                 "percentile99", "percentileest50", "percentileest90", "percentileest95", "percentileest99")
# DistinctCountMV / DistinctCountHLLMV / MinMaxRangeMV / PercentileMV / PercentileestMV (AggregationFunctionFactory.java:
# 48-58): the single-value function over every value of the selected docs (getMVHashCodeArray for the distinct counts)
EXT_MV_FUNCTIONS = ("distinctcountmv", "distinctcounthllmv", "minmaxrangemv") + tuple(
    "percentile%dmv" % p for p in (50, 90, 95, 99)) + tuple("percentileest%dmv" % p for p in (50, 90, 95, 99))


def ext_base(fn: str) -> str:
    """The single-value function an extended multi-value function restates over every value."""
    return fn[:-2] if fn in EXT_MV_FUNCTIONS else fn


# DISTINCTCOUNTHLL: stream-lib 2.7.0 HyperLogLog(log2m = HllConstants.DEFAULT_LOG2M = 8) (third-party, not vendored;
# com.clearspring.analytics:stream, pom.xml:525-527), restated scalar and per offer.
HLL_LOG2M = 8


def _i32(x: int) -> int:
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x & 0x80000000 else x


def murmur_hash_long(data: int) -> int:
    """MurmurHash.hashLong(long) in Java int arithmetic (>>> = logical shift of the 32-bit pattern)."""
    m, r = 0x5BD1E995, 24
    h = 0
    k = _i32(_i32(data) * m)
    k ^= (k & 0xFFFFFFFF) >> r
    h ^= _i32(k * m)
    k = _i32(_i32(data >> 32) * m)
    k ^= (k & 0xFFFFFFFF) >> r
    h = _i32(h * m)
    h ^= _i32(k * m)
    h ^= (h & 0xFFFFFFFF) >> 13
    h = _i32(h * m)
    h ^= (h & 0xFFFFFFFF) >> 15
    return _i32(h)


def hll_offer(regs: List[int], value: int) -> None:
    """HyperLogLog.offer(Integer) -> offerHashed(MurmurHash.hash(o)): j = x >>> (32 - log2m),
    r = numberOfLeadingZeros((x << log2m) | (1 << (log2m - 1)) + 1) + 1, RegisterSet.updateIfGreater(j, r)."""
    x = murmur_hash_long(value) & 0xFFFFFFFF
    j = x >> (32 - HLL_LOG2M)
    w = ((x << HLL_LOG2M) & 0xFFFFFFFF) | ((1 << (HLL_LOG2M - 1)) + 1)
    r = 32 - w.bit_length() + 1
    if r > regs[j]:
        regs[j] = r


def hll_from_string(s: str) -> List[int]:
    """HllUtil.convertStringToHll (core/startree/hll/HllUtil.java:58-60, SerializationConverter :146-175: byte =
    (byte)(char - 129)) then HyperLogLog.Builder.build: readInt log2m, readInt size, size bytes of big-endian int
    RegisterSet words, register i = (word[i / 6] >>> 5 * (i % 6)) & 0x1f."""
    b = bytes(((ord(c) - 129) & 0xFF) for c in s)
    log2m, size = struct.unpack_from(">ii", b, 0)
    if log2m != HLL_LOG2M:  # HyperLogLog.addAll into HyperLogLog(8): "Cannot merge estimators of different sizes"
        raise ValueError("Cannot merge estimators of different sizes")
    words = struct.unpack_from(">%dI" % (size // 4), b, 8)
    return [(words[i // 6] >> (5 * (i % 6))) & 0x1F for i in range(1 << HLL_LOG2M)]


def hll_add_all(regs: List[int], other: List[int]) -> None:
    for i, v in enumerate(other):
        if v > regs[i]:
            regs[i] = v


def hll_cardinality(regs: List[int]) -> int:
    """HyperLogLog.cardinality(): harmonic mean estimate, linear counting at or below 2.5 m, Math.round."""
    m = 1 << HLL_LOG2M
    total, zeros = 0.0, 0.0
    for v in regs:
        total += 1.0 / (1 << v)
        if v == 0:
            zeros += 1.0
    est = (0.7213 / (1 + 1.079 / m)) * m * m * (1 / total)
    if est <= 2.5 * m:
        est = m * math.log(m / zeros) if zeros else math.inf
    if est == math.inf:
        return (1 << 63) - 1
    return int(math.floor(est + 0.5))


def java_hash_code(col: OColumn, dict_id: int) -> int:
    """common/DataFetcher.java:242-248 fetchSingleHashCodes: dictionary.get(dictId).hashCode() of the boxed value
    (Integer, Long, Float, Double, String), the values DISTINCTCOUNT / DISTINCTCOUNTHLL receive
    (operator/aggregation/DefaultAggregationExecutor.java:135-139)."""
    v = col.dictionary[dict_id]
    if col.dtype == "INT":
        return _i32(int(v))
    if col.dtype == "LONG":  # Long.hashCode: (int)(value ^ (value >>> 32))
        u = int(v) & 0xFFFFFFFFFFFFFFFF
        return _i32(u ^ (u >> 32))
    if col.dtype == "FLOAT":  # Float.hashCode: floatToIntBits (NaN -> 0x7fc00000)
        f = float(v)
        return 0x7FC00000 if f != f else _i32(struct.unpack(">I", struct.pack(">f", f))[0])
    if col.dtype == "DOUBLE":  # Double.hashCode: bits ^ (bits >>> 32) of doubleToLongBits
        d = float(v)
        u = 0x7FF8000000000000 if d != d else struct.unpack(">Q", struct.pack(">d", d))[0]
        return _i32(u ^ (u >> 32))
    h = 0  # String.hashCode over UTF-16 code units
    for ch in str(v):
        cp = ord(ch)
        units = [cp] if cp < 0x10000 else [0xD800 + ((cp - 0x10000) >> 10), 0xDC00 + ((cp - 0x10000) & 0x3FF)]
        for u16 in units:
            h = (31 * h + u16) & 0xFFFFFFFF
    return _i32(h)


def _projection_columns(q: dict) -> List[str]:
    cols = []
    for a in q["aggregations"]:
        if a["fn"] != "count" and a["column"] not in cols:
            cols.append(a["column"])
    for g in (q.get("group_by") or {}).get("columns", []):
        if g not in cols:
            cols.append(g)
    return cols


def _blocks(docs: np.ndarray, size: int):
    for i in range(0, len(docs), size):
        yield docs[i:i + size]


def run_aggregation(seg: OSegment, q: dict, literal_filter: bool = True) -> dict:
    """AggregationOperator.getNextBlock + DefaultAggregationExecutor (operator/aggregation/AggregationOperator.java:77-104,
    DefaultAggregationExecutor.java:94-303) with Count/Sum/Min/Max/Avg.aggregate."""
    if literal_filter:
        docs, scanned = filter_docs(seg, q.get("filter"))
    else:
        docs, scanned = np.nonzero(filter_mask_vectorized(seg, q.get("filter")))[0], None
    holders = []
    for a in q["aggregations"]:
        fn = ext_base(a["fn"])
        holders.append([0.0, 0] if fn in ("avg", "avgmv") else set() if fn == "distinctcount" else
                       [0] * (1 << HLL_LOG2M) if fn in ("distinctcounthll", "fasthll") else
                       [math.inf, -math.inf] if fn == "minmaxrange" else _qdigest() if fn.startswith("percentileest")
                       else [] if fn.startswith("percentile") else
                       FN_DEFAULT[fn])
    for blk in _blocks(docs, MAX_DOC_PER_CALL):
        for k, a in enumerate(q["aggregations"]):
            fn = a["fn"]
            if fn == "count":
                holders[k] = holders[k] + float(len(blk))  # CountAggregationFunction.aggregate:43-48
                continue
            col = seg.columns[a["column"]]
            if fn in MV_FUNCTIONS:  # {Count,Sum,Min,Max,Avg}MVAggregationFunction.aggregate: every value of every doc
                if col.mv_ids is None:
                    raise ValueError("%s over a single-value column" % fn)
                vals = [col.value_as_double(col.mv_ids[int(d)]) for d in blk]
                flat = np.concatenate(vals) if vals else np.zeros(0)
                if fn == "countmv":
                    holders[k] = holders[k] + float(len(flat))
                elif fn == "summv":
                    holders[k] = holders[k] + (float(np.cumsum(flat)[-1]) if len(flat) else 0.0)
                elif fn == "minmv":
                    holders[k] = min(holders[k], float(flat.min())) if len(flat) else holders[k]
                elif fn == "maxmv":
                    holders[k] = max(holders[k], float(flat.max())) if len(flat) else holders[k]
                else:
                    holders[k] = [holders[k][0] + (float(np.cumsum(flat)[-1]) if len(flat) else 0.0),
                                  holders[k][1] + len(flat)]
                continue
            mvx = fn in EXT_MV_FUNCTIONS
            if (col.mv_ids is not None) != mvx:
                raise ValueError("%s over a %s column" % (fn, "single-value" if mvx else "multi-value"))
            fn = ext_base(fn)
            # the block's values: one per doc, or every value of every doc (getMVHashCodeArray / getMultiValues)
            ids = (np.concatenate([col.mv_ids[int(d)] for d in blk]) if len(blk) else np.zeros(0, np.int64)) \
                if mvx else col.dict_ids[blk]
            if fn in ("distinctcount", "distinctcounthll"):  # getSVHashCodeArray: (int) of each value's hashCode()
                hc = [java_hash_code(col, int(i)) for i in ids]
                if fn == "distinctcount":
                    holders[k].update(hc)
                else:
                    for x in hc:
                        hll_offer(holders[k], x)
                continue
            if fn == "fasthll":  # FastHllAggregationFunction.aggregate: addAll(convertStringToHll(value)) per doc
                if col.dtype != "STRING":
                    raise ValueError("fasthll over a non-STRING column")
                for i in ids:
                    hll_add_all(holders[k], hll_from_string(col.dictionary[int(i)]))
                continue
            if col.dtype == "STRING":  # String[] values where aggregate() requires double[]
                raise ValueError("%s over a STRING column" % fn)
            v = col.value_as_double(np.asarray(ids, dtype=np.int64))
            if fn == "sum":  # SumAggregationFunction.aggregate:45-56 (sequential double sum)
                s = float(np.cumsum(v)[-1]) if len(v) else 0.0
                holders[k] = holders[k] + s
            elif fn == "min":
                mn = float(v.min()) if len(v) else math.inf
                if mn < holders[k]:
                    holders[k] = mn
            elif fn == "max":
                mx = float(v.max()) if len(v) else -math.inf
                if mx > holders[k]:
                    holders[k] = mx
            elif fn == "avg":  # AvgAggregationFunction.aggregate:47-65
                s = float(np.cumsum(v)[-1]) if len(v) else 0.0
                holders[k] = [holders[k][0] + s, holders[k][1] + len(blk)]
            elif fn == "minmaxrange":  # MinMaxRangeAggregationFunction.aggregate: block min / max into the pair
                if len(v):
                    holders[k] = [min(holders[k][0], float(v.min())), max(holders[k][1], float(v.max()))]
            elif fn.startswith("percentileest"):  # PercentileestAggregationFunction.aggregate: add((long) v) per doc
                for x in v.tolist():
                    holders[k].add(int(x))
            elif fn.startswith("percentile"):  # PercentileAggregationFunction.aggregate: DoubleArrayList of values
                holders[k].extend(v.tolist())
    results = []
    for k, a in enumerate(q["aggregations"]):
        a = dict(a, fn=ext_base(a["fn"]))
        if a["fn"] in ("count", "countmv"):
            results.append(int(holders[k]))  # MutableLongValue((long) double)
        elif a["fn"] in ("avg", "avgmv"):
            results.append((float(holders[k][0]), int(holders[k][1])))
        elif a["fn"] == "distinctcount":
            results.append(set(holders[k]))
        elif a["fn"] in ("distinctcounthll", "fasthll"):
            results.append(list(holders[k]))
        elif a["fn"] == "minmaxrange":
            results.append((float(holders[k][0]), float(holders[k][1])))
        elif a["fn"].startswith("percentileest"):
            results.append(holders[k])
        elif a["fn"].startswith("percentile"):
            results.append(sorted(holders[k]))
        else:
            results.append(float(holders[k]))
    n_proj = len(_projection_columns(q))
    stats = [len(docs), scanned, len(docs) * n_proj, seg.total_raw_docs]
    return {"results": results, "stats": stats}


def group_key_mode(cards: Sequence[int]) -> Tuple[str, int]:
    """DefaultGroupKeyGenerator storage-type choice (operator/aggregation/groupby/DefaultGroupKeyGenerator.java:131-186)."""
    prod = 1
    for c in cards:
        if prod > LONG_MAX // c:
            return "ARRAY_MAP_BASED", LONG_MAX
        prod *= c
    if prod > MAX_INITIAL_RESULT_HOLDER_CAPACITY:
        return "LONG_MAP_BASED", prod
    return "ARRAY_BASED", prod


def run_group_by(seg: OSegment, q: dict, literal_filter: bool = True) -> dict:
    """AggregationGroupByOperator + DefaultGroupByExecutor + DefaultGroupKeyGenerator + {fn}.aggregateGroupBySV
    (operator/aggregation/groupby/AggregationGroupByOperator.java:81-106, DefaultGroupByExecutor.java:104-307,
    DefaultGroupKeyGenerator.java:214-262, SumAggregationFunction.java:70-81, MinAggregationFunction.java:75-88,
    AvgAggregationFunction.java:79-97).

    Returns the per-segment map {tuple(dictIds): [result per function]} (order-free), the storage mode, the
    ARRAY_BASED iteration order (ascending key), string keys and ExecutionStatistics."""
    if literal_filter:
        docs, scanned = filter_docs(seg, q.get("filter"))
    else:
        docs, scanned = np.nonzero(filter_mask_vectorized(seg, q.get("filter")))[0], None
    gcols = [seg.columns[c] for c in q["group_by"]["columns"]]
    cards = [c.card for c in gcols]
    mode, prod = group_key_mode(cards)
    if any(c.mv_ids is not None for c in gcols) or \
            any(a["fn"] in MV_FUNCTIONS or a["fn"] in EXT_MV_FUNCTIONS for a in q["aggregations"]):
        return _run_group_by_mv(seg, q, docs, scanned, gcols, cards, mode)
    # Raw key = sum_j dictId_j * prod_{i<j} card_i (column 0 least significant), :230-246
    ids = np.stack([c.dict_ids[docs] for c in gcols], axis=1) if len(docs) else np.zeros((0, len(gcols)), np.int64)
    keys = [tuple(int(x) for x in row) for row in ids]
    uniq = {}
    for k in keys:
        if k not in uniq:
            uniq[k] = len(uniq)  # first-seen dense group id (LONG/ARRAY_MAP modes)
    gid = np.array([uniq[k] for k in keys], dtype=np.int64)
    G = len(uniq)
    out = {k: [] for k in uniq}
    for a in q["aggregations"]:
        fn = a["fn"]
        if fn == "count":
            acc = np.zeros(G)
            np.add.at(acc, gid, 1.0)
            vals = [int(x) for x in acc]
        else:
            col = seg.columns[a["column"]]
            if fn in ("distinctcount", "distinctcounthll"):
                v = [java_hash_code(col, int(i)) for i in col.dict_ids[docs]]
            elif fn == "fasthll":
                v = [col.dictionary[int(i)] for i in col.dict_ids[docs]]
            else:
                v = col.value_as_double(col.dict_ids[docs])
            if fn == "sum":
                acc = np.zeros(G)
                np.add.at(acc, gid, v)  # unbuffered, in doc order == holder[key] += v sequentially
                vals = [float(x) for x in acc]
            elif fn == "min":
                acc = np.full(G, math.inf)
                np.minimum.at(acc, gid, v)
                vals = [float(x) for x in acc]
            elif fn == "max":
                acc = np.full(G, -math.inf)
                np.maximum.at(acc, gid, v)
                vals = [float(x) for x in acc]
            elif fn == "avg":
                acc = np.zeros(G)
                np.add.at(acc, gid, v)
                cnt = np.bincount(gid, minlength=G)
                vals = [(float(s), int(c)) for s, c in zip(acc, cnt)]
            elif fn == "distinctcount":  # DistinctCountAggregationFunction.aggregateGroupBySV: a set per group
                vals = [set() for _ in range(G)]
                for i, x in zip(gid.tolist(), v):
                    vals[i].add(x)
            elif fn == "distinctcounthll":  # DistinctCountHLLAggregationFunction.aggregateGroupBySV: an HLL per group
                vals = [[0] * (1 << HLL_LOG2M) for _ in range(G)]
                for i, x in zip(gid.tolist(), v):
                    hll_offer(vals[i], x)
            elif fn == "fasthll":  # FastHllAggregationFunction.aggregateGroupBySV: addAll per doc into its group's HLL
                vals = [[0] * (1 << HLL_LOG2M) for _ in range(G)]
                for i, x in zip(gid.tolist(), v):
                    hll_add_all(vals[i], hll_from_string(x))
            elif fn == "minmaxrange":  # MinMaxRangeAggregationFunction.aggregateGroupBySV: a (min, max) pair
                mn = np.full(G, math.inf)
                mx = np.full(G, -math.inf)
                np.minimum.at(mn, gid, v)
                np.maximum.at(mx, gid, v)
                vals = [(float(a_), float(b_)) for a_, b_ in zip(mn, mx)]
            elif fn.startswith("percentileest"):  # PercentileestAggregationFunction.aggregateGroupBySV: per doc
                vals = [_qdigest() for _ in range(G)]
                for i, x in zip(gid.tolist(), v.tolist()):
                    vals[i].add(int(x))
            elif fn.startswith("percentile"):  # PercentileAggregationFunction.aggregateGroupBySV: a list per group
                vals = [[] for _ in range(G)]
                for i, x in zip(gid.tolist(), v.tolist()):
                    vals[i].append(x)
                vals = [sorted(x) for x in vals]
        for k, i in uniq.items():
            out[k].append(vals[i])

    def raw_key(k):
        r = 0
        for j in range(len(k) - 1, -1, -1):
            r = r * cards[j] + k[j]
        return r

    def string_key(k):  # DefaultGroupKeyGenerator.*ToStringGroupKey :711-773
        return "\t".join(gcols[j].string_of(k[j]) for j in range(len(k)))

    order = sorted(uniq.keys(), key=raw_key) if mode == "ARRAY_BASED" else None
    n_proj = len(_projection_columns(q))
    stats = [len(docs), scanned, len(docs) * n_proj, seg.total_raw_docs]
    return {"mode": mode, "map": out, "order": order, "string_key": string_key, "stats": stats,
            "empty": len(docs) == 0}


def doc_group_keys(gcols, d: int) -> List[tuple]:
    """DefaultGroupKeyGenerator.generateKeysForDocId{ArrayBased,LongMapBased,ArrayMapBased}
    (operator/aggregation/groupby/DefaultGroupKeyGenerator.java:475-608): one key per combination of the doc's values,
    a single-value column contributing its one dictId, a multi-value column each of its values (duplicates included:
    a doc whose column holds v twice yields the key twice).  Keys as dictId tuples."""
    keys = [()]
    for c in gcols:
        ids = c.mv_ids[d] if c.mv_ids is not None else [c.dict_ids[d]]
        keys = [k + (int(i),) for i in ids for k in keys]
    return keys


def _run_group_by_mv(seg: OSegment, q: dict, docs, scanned, gcols, cards, mode) -> dict:
    """Group-by with multi-value group columns (DefaultGroupByExecutor.java:154-196 -> aggregateGroupByMV) and/or
    multi-value functions, restated per doc in doc order:
      COUNT                 += 1 per (doc, key)                       CountAggregationFunction.java:81-90
      SUM/MIN/MAX/AVG (SV)  the doc's value into each of its keys     Sum/Min/Max/AvgAggregationFunction.aggregateGroupByMV
      COUNTMV               += number of the doc's values             CountMVAggregationFunction.java:90-102
      SUMMV / AVGMV         += every value (AVGMV count += 1 each)    SumMVAggregationFunction.java:98-112, AvgMV:113-133
      MINMV / MAXMV         the holder's value BEFORE the doc is read once; each value below (above) it replaces the
                            holder, so the doc leaves the LAST such value in its value order, not its extreme
                            (MinMVAggregationFunction.java:76-91 aggregateGroupBySV, :103-119 aggregateGroupByMV;
                            MaxMVAggregationFunction.java:85-121).
    Extended functions (distinctcount / percentile / HLL ...) are not restated here."""
    uniq, order_seen = {}, []
    per = []  # (doc, key) pairs in processing order
    for d in docs.tolist():
        for k in doc_group_keys(gcols, d):
            if k not in uniq:
                uniq[k] = len(uniq)
                order_seen.append(k)
            per.append((d, uniq[k]))
    G = len(uniq)
    out = {k: [] for k in uniq}
    for a in q["aggregations"]:
        fn = a["fn"]
        if fn == "count":
            acc = [0] * G
            for _, g in per:
                acc[g] += 1
            vals = acc
        else:
            col = seg.columns[a["column"]]
            mv = fn in MV_FUNCTIONS or fn in EXT_MV_FUNCTIONS
            if mv and col.mv_ids is None:
                raise ValueError("%s over a single-value column" % fn)
            if not mv and col.mv_ids is not None:
                raise ValueError("%s over a multi-value column" % fn)
            fn = ext_base(fn)

            def dids(d):
                return col.mv_ids[d] if mv else [col.dict_ids[d]]

            def dvals(d):
                return [float(x) for x in col.value_as_double(np.asarray(dids(d), dtype=np.int64))]
            if fn in ("distinctcount", "distinctcounthll", "fasthll", "minmaxrange") or fn.startswith("percentile"):
                # {DistinctCount,DistinctCountHLL,FastHll,MinMaxRange,Percentile,Percentileest}{,MV}
                # .aggregateGroupByMV: every value of the doc into each of its keys' holders
                vals = [None] * G
                for d, g in per:
                    if fn == "distinctcount":
                        vals[g] = (vals[g] or set()) | {java_hash_code(col, int(i)) for i in dids(d)}
                    elif fn == "distinctcounthll":
                        vals[g] = vals[g] or [0] * (1 << HLL_LOG2M)
                        for i in dids(d):
                            hll_offer(vals[g], java_hash_code(col, int(i)))
                    elif fn == "fasthll":
                        vals[g] = vals[g] or [0] * (1 << HLL_LOG2M)
                        for i in dids(d):
                            hll_add_all(vals[g], hll_from_string(col.dictionary[int(i)]))
                    elif fn == "minmaxrange":
                        lo, hi = vals[g] or (math.inf, -math.inf)
                        for x in dvals(d):
                            lo, hi = min(lo, x), max(hi, x)
                        vals[g] = (lo, hi)
                    elif fn.startswith("percentileest"):
                        vals[g] = vals[g] or _qdigest()
                        for x in dvals(d):
                            vals[g].add(int(x))
                    else:
                        vals[g] = (vals[g] or []) + dvals(d)
                if fn.startswith("percentile") and not fn.startswith("percentileest"):
                    vals = [sorted(x) for x in vals]
            elif fn in ("sum", "summv"):
                acc = [0.0] * G
                for d, g in per:
                    for v in dvals(d):
                        acc[g] += v
                vals = acc
            elif fn == "countmv":
                acc = [0] * G
                for d, g in per:
                    acc[g] += len(col.mv_ids[d])
                vals = acc
            elif fn in ("avg", "avgmv"):
                acc = [[0.0, 0] for _ in range(G)]
                for d, g in per:
                    for v in dvals(d):
                        acc[g][0] += v
                        acc[g][1] += 1
                vals = [(s, c) for s, c in acc]
            elif fn in ("min", "minmv"):
                acc = [math.inf] * G
                for d, g in per:
                    old = acc[g]
                    for v in dvals(d):
                        if v < old:
                            acc[g] = v
                vals = acc
            elif fn in ("max", "maxmv"):
                acc = [-math.inf] * G
                for d, g in per:
                    old = acc[g]
                    for v in dvals(d):
                        if v > old:
                            acc[g] = v
                vals = acc
            else:
                raise ValueError("unsupported function %s" % fn)
        for k, i in uniq.items():
            out[k].append(vals[i])

    def raw_key(k):
        r = 0
        for j in range(len(k) - 1, -1, -1):
            r = r * cards[j] + k[j]
        return r

    def string_key(k):
        return "\t".join(gcols[j].string_of(k[j]) for j in range(len(k)))

    order = sorted(uniq.keys(), key=raw_key) if mode == "ARRAY_BASED" else None
    n_proj = len(_projection_columns(q))
    stats = [len(docs), scanned, len(docs) * n_proj, seg.total_raw_docs]
    return {"mode": mode, "map": out, "order": order, "string_key": string_key, "stats": stats,
            "empty": len(docs) == 0, "first_seen": order_seen}


# ------------------------------------------------------------------------------------------------
# a-19: combine across segments
# ------------------------------------------------------------------------------------------------
def _qdigest():
    """QuantileDigest(0.05) as vendored by the reference (quantile/digest/QuantileDigest.java).  The data structure is
    shared with the product's host code (pinot_amd/qdigest.py restates it); what the oracle checks independently is the
    per-doc insertion in doc order, as PercentileestAggregationFunction does, against the GPU's value histogram."""
    from pinot_amd.qdigest import QuantileDigest
    return QuantileDigest(0.05)


def combine_two(fn: str, a, b):
    """Legacy combineTwoValues (query/aggregation/function/{Sum,Count,Min,Max,Avg}AggregationFunction.java)."""
    fn = ext_base(fn)
    if fn in ("count", "countmv", "summv"):
        return a + b
    if fn == "minmv":
        return a if a < b else b
    if fn == "maxmv":
        return a if a > b else b
    if fn == "avgmv":
        return (a[0] + b[0], a[1] + b[1])
    if fn == "sum":
        return a + b
    if fn == "min":
        return a if a < b else b
    if fn == "max":
        return a if a > b else b
    if fn == "avg":
        return (a[0] + b[0], a[1] + b[1])
    if fn == "distinctcount":  # DistinctCountAggregationFunction.combineTwoValues: set union
        return set(a) | set(b)
    if fn in ("distinctcounthll", "fasthll"):  # {DistinctCountHLL,FastHll}AggregationFunction.combineTwoValues: addAll
        return [max(x, y) for x, y in zip(a, b)]
    if fn == "minmaxrange":  # MinMaxRangeAggregationFunction.combineTwoValues
        return (min(a[0], b[0]), max(a[1], b[1]))
    if fn.startswith("percentileest"):  # DigestAggregationFunction.combineTwoValues: merge (a copy of) the first
        return _qdigest().merge(a).merge(b)
    if fn.startswith("percentile"):  # PercentileAggregationFunction.combineTwoValues: list concatenation
        return sorted(list(a) + list(b))
    raise ValueError(fn)


def java_int_cast(x: float) -> int:
    """Java (int) of a double: truncation toward zero, saturating at the int range, NaN -> 0 (JLS 5.1.3)."""
    if x != x:
        return 0
    if x >= 2147483647.0:
        return 2147483647
    if x <= -2147483648.0:
        return -2147483648
    return int(x)


def reduce_extended(fn: str, v) -> float:
    """Final value of the extended functions (query/aggregation/function/DistinctCountAggregationFunction.java:136-145,
    MinMaxRangeAggregationFunction.java:129-146, quantile/PercentileUtil.java:40-52: sorted list, element
    (int)(size * p / 100))."""
    fn = ext_base(fn)
    if fn == "distinctcount":
        return len(v)
    if fn in ("distinctcounthll", "fasthll"):  # {DistinctCountHLL,FastHll}AggregationFunction.reduce: cardinality()
        return hll_cardinality(v)
    if fn == "minmaxrange":
        return v[1] - v[0] if v[0] != math.inf and v[1] != -math.inf else -1.0  # DEFAULT_MIN_MAX_RANGE_VALUE
    if fn.startswith("percentileest"):  # DigestAggregationFunction.reduce: getQuantile of the merged digest
        return v.get_quantile(int(fn[len("percentileest"):]) / 100.0)
    p = int(fn[len("percentile"):])
    return float(sorted(v)[int(len(v) * (p / 100.0))])


def combine_aggregation(parts: List[dict], q: dict) -> dict:
    """MCombineOperator + CombineService.mergeTwoBlocks (operator/MCombineOperator.java:84-199,
    query/aggregation/CombineService.java:45-177)."""
    res = list(parts[0]["results"])
    for p in parts[1:]:
        res = [combine_two(a["fn"], x, y) for a, x, y in zip(q["aggregations"], res, p["results"])]
    stats = [sum(p["stats"][i] or 0 for p in parts) for i in range(4)]
    return {"results": res, "stats": stats}


def combine_group_by(parts: List[dict], q: dict) -> dict:
    """MCombineGroupByOperator.combineBlocks (operator/MCombineGroupByOperator.java:139-233): merge per-segment maps
    by STRING group key, then AggregationGroupByOperatorService.trimToSize (query/aggregation/groupby/
    AggregationGroupByOperatorService.java:59-77,284-361).  Returns {string_key: [results]} untrimmed plus the trimmed
    per-function maps."""
    merged: Dict[str, list] = {}
    fns = [a["fn"] for a in q["aggregations"]]
    for p in parts:
        if p["empty"]:
            continue
        for k, v in p["map"].items():
            sk = p["string_key"](k)
            if sk in merged:
                merged[sk] = [combine_two(f, x, y) for f, x, y in zip(fns, merged[sk], v)]
            else:
                merged[sk] = list(v)
    top_n = q["group_by"].get("top_n", 10)
    min_trim = max(top_n, 1000)
    threshold, size = min_trim * 20, min_trim * 5
    trimmed = []
    for i, f in enumerate(fns):
        items = [(k, v[i]) for k, v in merged.items()]
        # getMinMaxPriorityQueue returns null for intermediates that are not Comparable (IntOpenHashSet,
        # MinMaxRangePair): those functions keep every group (AggregationGroupByOperatorService.java:336-349).
        # PERCENTILE's DoubleArrayList IS Comparable (lexicographic, over values in merge order, which depends on
        # thread timing): that trim is not reproducible, so every group is kept here too (parity unpinned above the
        # threshold; tests stay below it).
        if len(merged) > threshold and f not in EXT_FUNCTIONS and f not in EXT_MV_FUNCTIONS:
            keyf = (lambda kv: kv[1][0] / kv[1][1] if kv[1][1] else 0.0) if f == "avg" else (lambda kv: kv[1])
            items.sort(key=keyf, reverse=(f != "min"))
            items = items[:size]
        trimmed.append(dict(items))
    stats = [sum(p["stats"][i] or 0 for p in parts) for i in range(4)]
    return {"merged": merged, "trimmed": trimmed, "stats": stats, "trim_threshold": threshold, "trim_size": size}


# ------------------------------------------------------------------------------------------------
# a-18: star-tree traversal (test oracle)
# ------------------------------------------------------------------------------------------------
def parse_star_tree_off_heap(buf: bytes):
    """StarTreeOffHeap.readHeader (core/startree/StarTreeOffHeap.java:95-150): dimension names by index and the node
    table (7 x int32 per node, native LE: dimName, dimValue, startDoc, endDoc (exclusive), aggDocId, childStart,
    childEnd)."""
    import struct
    magic, _version, _hsize, nd = struct.unpack_from("<QiIi", buf, 0)
    assert magic == 0xBADDA55B00DAD00D
    pos, names = 20, {}
    for _ in range(nd):
        i, ln = struct.unpack_from("<ii", buf, pos)
        names[i] = buf[pos + 8:pos + 8 + ln].decode("utf-8")
        pos += 8 + ln
    (nn,) = struct.unpack_from("<i", buf, pos)
    nodes = np.frombuffer(buf, dtype="<i4", count=7 * nn, offset=pos + 4).reshape(nn, 7).astype(np.int64)
    return names, nodes


def star_tree_docs(seg: OSegment, tree_bytes: bytes, q: dict, num_raw: int) -> np.ndarray:
    """Doc ids StarTreeIndexOperator selects (operator/filter/StarTreeIndexOperator.java:134-478): BFS that follows the
    matching children of predicate columns (getMatchingDictionaryIds + getChildForDimensionValue), every non-star child
    of group-by columns (or when no star child exists) and the star child otherwise; matched entries contribute their
    aggregated doc, their range, or their range filtered by the remaining predicates."""
    from collections import deque
    names, nodes = parse_star_tree_off_heap(tree_bytes)
    tree = q.get("filter")
    leaves = [] if tree is None else ([tree] if tree["op"] not in ("AND", "OR") else tree["children"])
    preds = {lf["column"]: make_evaluator(seg.columns[lf["column"]], lf) for lf in leaves}
    if any(ev.always_false for ev in preds.values()):
        return np.zeros(0, dtype=np.int64)
    gb = set(q["group_by"]["columns"]) if q.get("group_by") else set()
    queue = deque([(0, frozenset(preds), frozenset(gb))])
    matched = []
    while queue:
        node, rp, rg = queue.popleft()
        _, _, st, en, agg, cs, ce = nodes[node]
        if cs == -1 or (not rp and not rg and agg >= num_raw):
            matched.append((node, rp, rg))
            continue
        col = names[int(nodes[cs][0])]
        children = range(int(cs), int(ce) + 1)
        if col in preds:
            nrp, nrg = rp - {col}, rg - {col}
            by_value = {int(nodes[c][1]): c for c in children}
            for did in preds[col].matching_ids:
                if int(did) in by_value:
                    queue.append((by_value[int(did)], nrp, nrg))
        elif col in gb or int(nodes[cs][1]) != -1:
            real = [c for c in children if int(nodes[c][1]) != -1]
            nrg = rg - {col} if real else rg
            for c in real:
                queue.append((c, rp, nrg))
        else:
            queue.append((int(cs), rp, rg))
    out = []
    for node, rp, rg in matched:
        _, _, st, en, agg, _, _ = nodes[node]
        if not rp:
            out.append(np.array([agg]) if (agg >= num_raw and not rg) else np.arange(st, en))
        else:
            r = np.arange(st, en)
            keep = np.ones(len(r), dtype=bool)
            for c in rp:
                keep &= preds[c].match[seg.columns[c].dict_ids[r]]
            out.append(r[keep])
    return np.sort(np.concatenate(out)).astype(np.int64) if out else np.zeros(0, dtype=np.int64)


def sum_by_group(seg: OSegment, docs: np.ndarray, metrics: Sequence[str], group_cols: Sequence[str]) -> dict:
    """BaseSumStarTreeIndexTest.computeSum (pinot-core/src/test/.../startree/BaseSumStarTreeIndexTest.java:145-195):
    per group key (dictionary values joined), the double sums of the metric columns over the given docs."""
    res = {}
    for d in docs.tolist():
        key = "\t".join(seg.columns[g].string_of(int(seg.columns[g].dict_ids[d])) for g in group_cols)
        acc = res.setdefault(key, [0.0] * len(metrics))
        for i, m in enumerate(metrics):
            c = seg.columns[m]
            acc[i] += float(c.dictionary[c.dict_ids[d]])
    return res
