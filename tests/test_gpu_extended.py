"""GPU parity of DISTINCTCOUNT / MINMAXRANGE / PERCENTILEnn (pinot_amd/extended.py): aggregation-only
requests decomposed into GPU sub-queries (MIN/MAX in the base query, a GROUP BY <column> histogram) against the CPU
oracle's literal restatement of the reference functions (IntOpenHashSet of (int) values, Pair of extremes,
DoubleArrayList + PercentileUtil), over several segments with different dictionaries."""
import numpy as np
import pytest

from oracle import pinot_oracle as O
from pinot_amd import pql
from tests import helpers as H

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    from pinot_amd import engine as E
    ctx = E.Context(0)
    rng = np.random.default_rng(17)
    gsegs, osegs = [], []
    for i in range(3):
        n = 40000 + 9000 * i
        raw = {"d": rng.integers(0, 50 + 10 * i, n).astype(np.int32),
               "v": rng.integers(-(1 << 20), 1 << 20, n).astype(np.int32) // (i + 1),
               "w": (rng.integers(0, 3000, n) * 0.37 - 300.0).astype(np.float32),
               "m": rng.integers(0, 5000, n).astype(np.int32)}
        s, o = H.build_pair("ext%d" % i, raw, types={"w": "FLOAT"})
        gsegs.append(E.IndexSegment(ctx, s))
        osegs.append(o)
    yield ctx, gsegs, osegs
    ctx.close()


QUERIES = [
    "SELECT DISTINCTCOUNT(d), MINMAXRANGE(v), PERCENTILE50(v), PERCENTILE90(m), COUNT(*) FROM t",
    "SELECT SUM(m), DISTINCTCOUNT(w), PERCENTILE95(w), PERCENTILE99(w), MINMAXRANGE(w) FROM t WHERE d < 20",
    "SELECT MINMAXRANGE(m), DISTINCTCOUNT(v), AVG(m), PERCENTILE50(d) FROM t WHERE v > 1000 AND m IN (1, 2, 3, 4000)",
    "SELECT COUNT(*), MINMAXRANGE(m), DISTINCTCOUNT(d) FROM t WHERE d = 123456",
    "SELECT DISTINCTCOUNTHLL(v), DISTINCTCOUNT(v), DISTINCTCOUNTHLL(w), DISTINCTCOUNTHLL(d) FROM t WHERE m < 4000",
    "SELECT DISTINCTCOUNTHLL(m), COUNT(*) FROM t WHERE d = 123456",
    "SELECT PERCENTILEEST50(v), PERCENTILEEST90(m), PERCENTILEEST99(w), COUNT(*) FROM t WHERE d < 40",
]


@pytest.mark.parametrize("text", QUERIES)
def test_extended_functions_match_oracle(env, text):
    from pinot_amd import engine as E
    from pinot_amd import extended as X
    ctx, gsegs, osegs = env
    q = pql.compile(text)
    blk = E.InstancePlanMakerImplV2(ctx).make_inter_segment_plan(gsegs, q).execute()
    got = blk.get_aggregation_result()
    parts = [O.run_aggregation(s, q, literal_filter=False) for s in osegs]
    exp = O.combine_aggregation(parts, q)
    fns = [a["fn"] for a in q["aggregations"]]
    for fn, g, e in zip(fns, got, exp["results"]):
        if fn == "distinctcount":
            assert g == e
        elif fn == "distinctcounthll":  # HyperLogLog registers bit-exact, then the same cardinality()
            assert list(g) == list(e)
            assert X.reduce_value(fn, g) == O.reduce_extended(fn, e)
        elif fn == "minmaxrange":
            assert tuple(g) == tuple(e)
            assert X.reduce_value(fn, g) == O.reduce_extended(fn, e)
        elif fn.startswith("percentileest"):  # both digests answer within the rank-error guarantee
            _assert_qdigest_bound(fn, X.reduce_value(fn, g), O.reduce_extended(fn, e), _selected(osegs, q, fn, fns))
        elif fn.startswith("percentile"):
            vals, cnts = np.unique(np.asarray(e, dtype=np.float64), return_counts=True)
            assert g == [(float(x), int(c)) for x, c in zip(vals, cnts)]
            if e:
                assert X.reduce_value(fn, g) == O.reduce_extended(fn, e)
        else:
            H.assert_values_equal([g], [e], [fn])
    st = blk.stats.as_list()
    assert st[0] == exp["stats"][0] and st[2] == exp["stats"][2] and st[3] == exp["stats"][3]
    assert st[1] == H.literal_entries(osegs, q)


def _selected(osegs, q, fn, fns):
    """The (long) values PERCENTILEEST offers: the column's selected values over every segment."""
    col = q["aggregations"][fns.index(fn)]["column"]
    out = []
    for s in osegs:
        m = O.filter_mask_vectorized(s, q.get("filter"))
        c = s.columns[col]
        out += [int(x) for x in c.dictionary[c.dict_ids[np.nonzero(m)[0]]].astype(np.float64)]
    return np.sort(np.array(out, dtype=np.int64))


def _assert_qdigest_bound(fn, got, exp, values):
    """QuantileDigest(maxError = 0.05): the answer's rank lies within maxError * N of q * N (getQuantile contract)."""
    qq = int(fn[len("percentileest"):]) / 100.0
    n = len(values)
    for x in (got, exp):
        lo, hi = np.searchsorted(values, x, side="left"), np.searchsorted(values, x, side="right")
        assert lo - 0.05 * n - 1 <= qq * n <= hi + 0.05 * n + 1, (fn, x, qq, n)


GROUPED = [
    "SELECT DISTINCTCOUNT(v), MINMAXRANGE(m), SUM(m), PERCENTILE50(m), COUNT(*) FROM t GROUP BY d",
    "SELECT PERCENTILE90(w), DISTINCTCOUNT(w), MAX(v) FROM t WHERE m < 2500 GROUP BY d TOP 5",
    "SELECT MINMAXRANGE(v), AVG(m), DISTINCTCOUNT(m) FROM t WHERE d IN (1, 2, 3) GROUP BY d, m",
    "SELECT DISTINCTCOUNTHLL(v), SUM(m), DISTINCTCOUNTHLL(w) FROM t WHERE m > 100 GROUP BY d",
    "SELECT PERCENTILEEST90(m), SUM(m) FROM t WHERE d < 10 GROUP BY d",
]


def _group_values(osegs, q, key, fn, fns):
    col = q["aggregations"][fns.index(fn)]["column"]
    gcols = q["group_by"]["columns"]
    out = []
    for s in osegs:
        m = O.filter_mask_vectorized(s, q.get("filter"))
        for d in np.nonzero(m)[0]:
            if "\t".join(s.columns[g].string_of(int(s.columns[g].dict_ids[d])) for g in gcols) == key:
                c = s.columns[col]
                out.append(float(c.dictionary[c.dict_ids[d]]))
    return out


@pytest.mark.parametrize("text", GROUPED)
def test_extended_functions_group_by_match_oracle(env, text):
    from pinot_amd import engine as E
    ctx, gsegs, osegs = env
    q = pql.compile(text)
    blk = E.InstancePlanMakerImplV2(ctx).make_inter_segment_plan(gsegs, q).execute()
    got = blk.get_aggregation_group_by_result().as_map()
    exp = O.combine_group_by([O.run_group_by(s, q, literal_filter=False) for s in osegs], q)
    fns = [a["fn"] for a in q["aggregations"]]
    assert set(got) == set(exp["merged"])
    for k, e in exp["merged"].items():
        for fn, g, x in zip(fns, got[k], e):
            if fn == "distinctcount":
                assert g == x
            elif fn == "distinctcounthll":
                assert list(g) == list(x)
            elif fn == "minmaxrange":
                assert tuple(g) == tuple(x)
            elif fn.startswith("percentileest"):  # same multiset offered: same count, quantiles within the bound
                assert g.count == x.count
                vals = np.sort(np.array([int(v) for v in _group_values(osegs, q, k, fn, fns)], dtype=np.int64))
                _assert_qdigest_bound(fn, g.get_quantile(int(fn[13:]) / 100.0), x.get_quantile(int(fn[13:]) / 100.0),
                                      vals)
            elif fn.startswith("percentile"):
                vals, cnts = np.unique(np.asarray(x, dtype=np.float64), return_counts=True)
                assert g == [(float(a), int(c)) for a, c in zip(vals, cnts)]
            else:
                H.assert_values_equal([g], [x], [fn])
    for i, fn in enumerate(fns):  # combine output: every group for the extended functions, trimmed maps otherwise
        assert set(blk.trimmed[i]) == set(exp["trimmed"][i])
    st = blk.stats.as_list()
    assert st[0] == exp["stats"][0] and st[2] == exp["stats"][2] and st[3] == exp["stats"][3]
    assert st[1] == H.literal_entries(osegs, q)


def test_extended_over_string_column(env):
    """DISTINCTCOUNT / DISTINCTCOUNTHLL take String.hashCode() of STRING values (getSVHashCodeArray); PERCENTILE gets
    String[] where its aggregate() requires double[], which the reference rejects."""
    from pinot_amd import engine as E
    from pinot_amd import native as N
    ctx, _, _ = env
    words = np.array(["a", "b", "c", "a", "hello", "Aa", "BB", "\u00e9t\u00e9", "x\ty"])  # "Aa"/"BB" share a hash
    raw = {"s": words, "m": np.arange(len(words), dtype=np.int32)}
    seg, o = H.build_pair("strx", raw)
    g = E.IndexSegment(ctx, seg)
    pm = E.InstancePlanMakerImplV2(ctx)
    for text in ("SELECT DISTINCTCOUNT(s), DISTINCTCOUNTHLL(s) FROM t WHERE m < 8",
                 "SELECT DISTINCTCOUNT(s), DISTINCTCOUNTHLL(s) FROM t GROUP BY m"):
        q = pql.compile(text)
        blk = pm.make_inter_segment_plan([g], q).execute()
        if q.get("group_by"):
            got = blk.get_aggregation_group_by_result().as_map()
            exp = O.combine_group_by([O.run_group_by(o, q, literal_filter=False)], q)["merged"]
            assert set(got) == set(exp)
            for k in exp:
                assert got[k][0] == exp[k][0] and list(got[k][1]) == list(exp[k][1])
        else:
            got = blk.get_aggregation_result()
            exp = O.combine_aggregation([O.run_aggregation(o, q, literal_filter=False)], q)["results"]
            assert got[0] == exp[0] and list(got[1]) == list(exp[1])
            assert len(got[0]) == 6  # a b c hello Aa|BB ete
    with pytest.raises(N.PgxError) as ei:
        pm.make_inter_segment_plan([g], pql.compile("SELECT PERCENTILE50(s) FROM t")).execute()
    assert ei.value.status == N.PGX_ERR_UNSUPPORTED


def test_fasthll_over_serialized_hll_column(env):
    """FASTHLL over a STRING column of serialized HyperLogLogs (the star-tree HLL derived field: HllUtil
    .convertHllToString, char = byte + 129): addAll of every selected doc's estimator, aggregation-only and group-by,
    registers bit-exact against the oracle's per-doc restatement; FASTHLL over a numeric column is rejected."""
    from pinot_amd import engine as E
    from pinot_amd import hll
    from pinot_amd import native as N
    ctx, _, _ = env
    rng = np.random.default_rng(23)
    pool = [hll.to_string(hll.from_ints(rng.integers(0, 1 << 20, int(rng.integers(1, 400))).tolist()))
            for _ in range(60)]
    gsegs, osegs = [], []
    for i in range(2):
        n = 3000 + 500 * i
        raw = {"h": np.array([pool[j] for j in rng.integers(0, len(pool), n)], dtype=object),
               "d": rng.integers(0, 12, n).astype(np.int32)}
        s, o = H.build_pair("fhll%d" % i, raw)
        gsegs.append(E.IndexSegment(ctx, s))
        osegs.append(o)
    pm = E.InstancePlanMakerImplV2(ctx)
    q = pql.compile("SELECT FASTHLL(h), COUNT(*) FROM t WHERE d < 7")
    got = pm.make_inter_segment_plan(gsegs, q).execute().get_aggregation_result()
    exp = O.combine_aggregation([O.run_aggregation(o, q, literal_filter=False) for o in osegs], q)["results"]
    assert list(got[0]) == list(exp[0]) and int(got[1]) == int(exp[1])
    assert hll.cardinality(got[0]) == O.reduce_extended("fasthll", exp[0])
    q = pql.compile("SELECT FASTHLL(h) FROM t GROUP BY d")
    got = pm.make_inter_segment_plan(gsegs, q).execute().get_aggregation_group_by_result().as_map()
    exp = O.combine_group_by([O.run_group_by(o, q, literal_filter=False) for o in osegs], q)["merged"]
    assert set(got) == set(exp)
    for k in exp:
        assert list(got[k][0]) == list(exp[k][0])
    with pytest.raises(N.PgxError) as ei:
        pm.make_inter_segment_plan(gsegs, pql.compile("SELECT FASTHLL(d) FROM t")).execute()
    assert ei.value.status == N.PGX_ERR_UNSUPPORTED


def test_histogram_group_key_with_tab_in_leading_string(env):
    """A leading STRING group value holding a tab: the histogram sub-query's groups are folded per leading key from
    the result's per-column key parts, not by re-splitting the joined string (DefaultGroupKeyGenerator joins with tab,
    so the joined key alone is ambiguous)."""
    from pinot_amd import engine as E
    ctx, _, _ = env
    g0 = np.array(["a\tb", "a", "a\tb", "c", "a", "a\tb", "c", "c\t"] * 50)
    raw = {"g": g0, "v": (np.arange(len(g0)) % 7).astype(np.int32), "m": np.arange(len(g0), dtype=np.int32)}
    seg, o = H.build_pair("tabkey", raw)
    gs = E.IndexSegment(ctx, seg)
    pm = E.InstancePlanMakerImplV2(ctx)
    for text in ("SELECT DISTINCTCOUNT(v), PERCENTILE50(v), COUNT(*) FROM t GROUP BY g",
                 "SELECT DISTINCTCOUNT(v) FROM t WHERE m < 300 GROUP BY g"):
        q = pql.compile(text)
        got = pm.make_inter_segment_plan([gs], q).execute().get_aggregation_group_by_result().as_map()
        exp = O.combine_group_by([O.run_group_by(o, q, literal_filter=False)], q)["merged"]
        assert set(got) == set(exp)
        for k in exp:
            assert got[k][0] == exp[k][0], k
            if len(exp[k]) > 1:
                vals, cnts = np.unique(np.asarray(exp[k][1], dtype=np.float64), return_counts=True)
                assert got[k][1] == [(float(a), int(c)) for a, c in zip(vals, cnts)]
                assert got[k][2] == exp[k][2]
