"""CPU checks of the oracle's multi-value group-by restatement (oracle/pinot_oracle.py _run_group_by_mv): key expansion
per doc (DefaultGroupKeyGenerator.generateKeysForDocId*: one key per value combination, duplicates included) and the
*MV functions' group-by folds, including MINMV / MAXMV's read-once holder (MinMVAggregationFunction.java:103-119: a doc
leaves the LAST value below the holder's old value, not its minimum)."""
from oracle import pinot_oracle as O
from pinot_amd import pql


def _seg():
    # doc 0: g {1, 2} v [5, 3, 4]; doc 1: g {2} v [9, 1]; doc 2: g {1, 1} v [2]
    return O.OSegment.from_raw({"g": [[1, 2], [2], [1, 1]], "v": [[5, 3, 4], [9, 1], [2]],
                                "m": __import__("numpy").array([10, 20, 30], dtype="int32")})


def _run(text):
    o = O.run_group_by(_seg(), pql.compile(text), literal_filter=True)
    return {o["string_key"](k): v for k, v in o["map"].items()}


def test_keys_per_value_and_duplicates():
    m = _run("SELECT COUNT(*), SUM(m) FROM t GROUP BY g")
    # g=1: doc 0 once, doc 2 twice (duplicate value) -> 3 pairs; g=2: docs 0, 1
    assert m["1"] == [3, 10.0 + 30.0 + 30.0]
    assert m["2"] == [2, 30.0]


def test_mv_functions_fold_per_doc():
    m = _run("SELECT COUNTMV(v), SUMMV(v), AVGMV(v) FROM t GROUP BY g")
    assert m["1"] == [3 + 1 + 1, 12.0 + 2.0 + 2.0, (16.0, 5)]
    assert m["2"] == [3 + 2, 12.0 + 10.0, (22.0, 5)]


def test_minmv_maxmv_read_the_holder_once_per_doc():
    m = _run("SELECT MINMV(v), MAXMV(v) FROM t GROUP BY g")
    # g=2: doc 0 from +inf keeps the last value below +inf = 4 (not 3); doc 1: values below 4 -> 1
    # MAXMV g=2: doc 0 from -inf -> 4 (last value above -inf); doc 1: 9 > 4 -> 9, 1 not -> 9
    assert m["2"] == [1.0, 9.0]
    # g=1: doc 0 -> 4 (MIN) / 4 (MAX); doc 2 twice: 2 < 4 -> 2, then 2 < 2 no -> 2; MAX: 2 > 4 no -> 4
    assert m["1"] == [2.0, 4.0]
