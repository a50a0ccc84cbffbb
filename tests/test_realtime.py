"""Realtime (consuming) segments on the CPU: RealtimeSegment's indexing semantics (RealtimeSegmentImpl.index), its
snapshot (sorted dictionaries, remapped ids, unsorted forward index, inverted indexes), and the property the GPU path
rests on: on every predicate the realtime evaluators (arrival-order mutable dictionary, RangeRealtimeDictionary-
PredicateEvaluator) select exactly the docs the offline evaluators select on the snapshot, so aggregations and groups
agree too.  Both sides are the oracle's restatements (oracle/pinot_oracle.py make_evaluator, OSegment.from_realtime)."""
import numpy as np
import pytest

from oracle import pinot_oracle as O
from pinot_amd import pql
from pinot_amd import segment as S
from pinot_amd.realtime import RealtimeSegment

SCHEMA = {"dim": ("INT", True, "DIMENSION"), "name": ("STRING", True, "DIMENSION"),
          "lng": ("LONG", True, "DIMENSION"), "tags": ("INT", False, "DIMENSION"),
          "met": ("INT", True, "METRIC"), "dbl": ("DOUBLE", True, "METRIC"), "ts": ("LONG", True, "TIME")}


def _rows(rng, n):
    names = ["a", "ab", "abc", "b", "ba", "z", "zz", "m"]
    out = []
    for i in range(n):
        out.append({"dim": int(rng.integers(-50, 50)), "name": names[int(rng.integers(0, len(names)))],
                    "lng": int(rng.integers(-(1 << 40), 1 << 40)) if rng.random() < 0.3 else int(rng.integers(0, 9)),
                    "tags": [int(x) for x in rng.integers(0, 12, size=int(rng.integers(1, 4)))],
                    "met": int(rng.integers(0, 1000)), "dbl": float(rng.integers(-300, 300)) / 4.0,
                    "ts": 1_600_000_000 + i})
    return out


@pytest.fixture(scope="module")
def rt():
    rng = np.random.default_rng(11)
    seg = RealtimeSegment("rt_0", SCHEMA, capacity=5000, inverted=["dim", "tags"])
    for r in _rows(rng, 3000):
        assert seg.index(r)
    return seg


def _oracle_realtime(seg):
    dicts = {c: (t, list(seg.dictionaries[c].values)) for c, (t, _, _) in seg.schema.items()}
    ids = {c: seg.arrival_ids(c) for c in seg.schema}
    return O.OSegment.from_realtime(dicts, ids, seg.num_docs, inverted=sorted(seg.inverted))


def _oracle_offline(snap):
    cols = {}
    for name, c in snap.columns.items():
        d = np.asarray(c.dictionary_values(), dtype=object if c.data_type == "STRING" else None)
        if c.is_mv:
            per = [x.astype(np.int64) for x in c.mv_dict_ids()]
            cols[name] = O.OColumn(name, c.data_type, d, np.concatenate(per), False, c.has_inverted, c.bits, per)
        else:
            cols[name] = O.OColumn(name, c.data_type, d, c.dict_ids().astype(np.int64), c.is_sorted, c.has_inverted,
                                   c.bits)
    return O.OSegment(cols, snap.total_docs, snap.total_raw_docs)


def test_index_semantics():
    seg = RealtimeSegment("rt_cap", {"a": ("INT", True, "DIMENSION"), "m": ("LONG", True, "METRIC")}, capacity=3)
    assert seg.index({"a": 7, "m": 1})
    assert seg.index({"a": None, "m": 2})  # dropped, still accepting
    assert seg.rows_dropped == 1 and seg.num_docs == 1
    assert seg.index({"a": 3, "m": 2})
    assert not seg.index({"a": 7, "m": 5})  # capacity reached: numDocsIndexed < capacity is false
    d = seg.dictionaries["a"]
    assert d.values == [7, 3] and d.index_of("3") == 1 and d.index_of(4) == -1
    assert (d.min, d.max) == (3, 7)
    assert seg.arrival_ids("a") == [0, 1, 0]


def test_snapshot_layout(rt):
    snap = rt.snapshot()
    assert snap.total_docs == rt.num_docs
    for name, (t, sv, _) in rt.schema.items():
        c = snap.columns[name]
        d = rt.dictionaries[name]
        vals = c.dictionary_values()
        assert list(vals) == sorted(d.values, key=lambda v: [ord(ch) for ch in v] if t == "STRING" else v)
        assert not c.is_sorted and c.has_inverted == (name in rt.inverted)
        if sv:
            got = [vals[i] for i in c.dict_ids()]
            assert got == [d.values[i] for i in rt.arrival_ids(name)]
        else:
            got = [[int(vals[i]) for i in x] for x in c.mv_dict_ids()]
            assert got == [[d.values[i] for i in x] for x in rt.arrival_ids(name)]
    # ts ascends with the doc id: still an unsorted (fixed-bit) forward index, as the realtime data source reports
    assert snap.columns["ts"].fwd_bytes is not None and snap.columns["ts"].sorted_bytes is None
    assert rt.snapshot() is snap  # cached until the next index()


LEAVES = [
    ("dim", "EQ", ["7"]), ("dim", "EQ", ["1000"]), ("dim", "IN", ["-3", "4", "99", "17"]), ("dim", "NEQ", ["0"]),
    ("dim", "NOT_IN", ["1", "2", "3"]), ("dim", "RANGE", ["[-10\t\t10]"]), ("dim", "RANGE", ["(-10\t\t10)"]),
    ("dim", "RANGE", ["(*\t\t5)"]), ("dim", "RANGE", ["[5\t\t*)"]), ("dim", "RANGE", ["(60\t\t*)"]),
    ("name", "RANGE", ["[ab\t\tb]"]), ("name", "RANGE", ["(a\t\tba)"]), ("name", "EQ", ["zz"]), ("name", "IN", ["m", "q"]),
    ("lng", "RANGE", ["[0\t\t4]"]), ("lng", "RANGE", ["(*\t\t0)"]), ("met", "RANGE", ["[100\t\t900)"]),
    ("dbl", "RANGE", ["(-10.5\t\t20.25]"]), ("dbl", "EQ", ["-0.25"]), ("tags", "IN", ["3", "5"]),
    ("tags", "RANGE", ["[2\t\t4]"]), ("tags", "NEQ", ["0"]),
]


@pytest.mark.parametrize("leaf", LEAVES, ids=[" ".join([c, op] + v) for c, op, v in LEAVES])
def test_realtime_evaluator_selects_what_the_snapshot_selects(rt, leaf):
    col, op, vals = leaf
    tree = {"op": op, "column": col, "values": vals}
    ort = _oracle_realtime(rt)
    off = _oracle_offline(rt.snapshot())
    a = np.nonzero(O.filter_mask_vectorized(ort, tree))[0]
    b = np.nonzero(O.filter_mask_vectorized(off, tree))[0]
    assert np.array_equal(a, b)
    # and the realtime evaluator by its own definition: the docs whose value lies in the range
    ev = O.make_evaluator(ort.columns[col], tree)
    assert ev.always_false == (len(ev.matching_ids) == 0)


QUERIES = [
    "SELECT COUNT(*), SUM(met), MIN(dbl), MAX(lng), AVG(met) FROM rt WHERE dim BETWEEN -20 AND 20",
    "SELECT SUM(met), MAX(dbl) FROM rt WHERE name > 'ab' AND dim <> 3 GROUP BY name",
    "SELECT COUNT(*), MIN(met) FROM rt WHERE tags IN (1, 2) OR lng < 5 GROUP BY dim, name",
    "SELECT SUM(dbl) FROM rt WHERE met >= 500 GROUP BY tags",
]


@pytest.mark.parametrize("text", QUERIES)
def test_realtime_answers_equal_snapshot_answers(rt, text):
    q = pql.compile(text)
    ort = _oracle_realtime(rt)
    off = _oracle_offline(rt.snapshot())
    if q.get("group_by"):
        a, b = O.run_group_by(ort, q), O.run_group_by(off, q)
        ma = {a["string_key"](k): v for k, v in a["map"].items()}
        mb = {b["string_key"](k): v for k, v in b["map"].items()}
        assert ma == mb and len(ma) > 0
    else:
        a, b = O.run_aggregation(ort, q), O.run_aggregation(off, q)
        assert a["results"] == b["results"]
    assert list(a["stats"]) == list(b["stats"])
