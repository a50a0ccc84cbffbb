"""Realtime (consuming) segments on the GPU: queries over RealtimeSegment.device_segment against the oracle's
restatement of the consuming segment itself (arrival-order mutable dictionaries, RangeRealtimeDictionaryPredicate-
Evaluator, OSegment.from_realtime) -- results, groups and execution statistics; again after more rows arrive; and a
consuming segment queried beside an immutable one (one combine)."""
import numpy as np
import pytest

from pinot_amd import pql
from pinot_amd.realtime import RealtimeSegment
from tests import helpers as H
from tests.test_realtime import SCHEMA, _oracle_realtime, _rows

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from pinot_amd import engine as E
    c = E.Context(0)
    yield c
    c.close()


QUERIES = [
    "SELECT COUNT(*), SUM(met), MIN(dbl), MAX(lng), AVG(met) FROM rt",
    "SELECT COUNT(*), SUM(met), MIN(dbl), MAX(lng), AVG(met) FROM rt WHERE dim BETWEEN -20 AND 20",
    "SELECT SUM(met), MAX(dbl) FROM rt WHERE name > 'ab' AND dim <> 3 GROUP BY name",
    "SELECT COUNT(*), MIN(met) FROM rt WHERE tags IN (1, 2) OR lng < 5 GROUP BY dim, name",
    "SELECT SUM(dbl), COUNT(*) FROM rt WHERE met >= 500 GROUP BY tags",
    "SELECT COUNT(*), SUM(met) FROM rt WHERE dim IN (3, 4, 5) AND name NOT IN ('z', 'zz') GROUP BY ts",
    "SELECT SUMMV(tags), MAXMV(tags) FROM rt WHERE dbl < 0",
]


def _run_inner(ctx, seg, q):
    from pinot_amd import engine as E
    op = E.InstancePlanMakerImplV2(ctx).make_inner_segment_plan(seg, q).run()
    blk = op.next_block()
    return blk, op.get_execution_statistics()


def _check(ctx, rt, text, nonempty=True):
    q = pql.compile(text)
    blk, st = _run_inner(ctx, rt.device_segment(ctx), q)
    o = H.oracle_answer([_oracle_realtime(rt)], q, literal=True)
    fns = [a["fn"] for a in q["aggregations"]]
    assert st.as_list() == list(o["stats"])
    if q.get("group_by"):
        gr = blk.get_aggregation_group_by_result()
        m = gr.as_map() if gr is not None else {}  # no selected doc: no group-by result
        assert set(m) == set(o["map"]) and (len(m) > 0 or not nonempty)
        for k, v in o["map"].items():
            H.assert_values_equal(m[k], v, fns)
    else:
        H.assert_values_equal(blk.get_aggregation_result(), o["results"], fns)


@pytest.mark.parametrize("text", QUERIES)
def test_consuming_segment_matches_oracle(ctx, text):
    rng = np.random.default_rng(5)
    rt = RealtimeSegment("rt_g", SCHEMA, capacity=100000, inverted=["dim", "tags"])
    for r in _rows(rng, 20000):
        rt.index(r)
    _check(ctx, rt, text)


def test_queries_follow_ingestion(ctx):
    """Rows arriving between queries: every query sees exactly the docs indexed so far (docIdSearchableOffset)."""
    rng = np.random.default_rng(9)
    rt = RealtimeSegment("rt_i", SCHEMA, capacity=100000, inverted=["name"])
    rows = _rows(rng, 9000)
    seen = []
    for stop in (1, 700, 4096, 9000):
        for r in rows[len(seen):stop]:
            rt.index(r)
            seen.append(r)
        for text in QUERIES[1:4]:
            _check(ctx, rt, text, nonempty=stop > 1)
        q = pql.compile("SELECT COUNT(*), SUM(met) FROM rt")
        blk, _ = _run_inner(ctx, rt.device_segment(ctx), q)
        res = blk.get_aggregation_result()
        assert int(res[0]) == stop and int(res[1]) == sum(r["met"] for r in seen)
        # in place: each doc's dictIds crossed to the device once, at the first query after it arrived (pgx_mutable)
        assert rt.docs_sent == stop


def test_consuming_beside_immutable(ctx):
    """A server holding an immutable segment and a consuming one answers one combined query (MCombineOperator /
    MCombineGroupByOperator over both), equal to the oracle's combine of the two restatements."""
    from pinot_amd import engine as E
    rng = np.random.default_rng(21)
    rt = RealtimeSegment("rt_c", SCHEMA, capacity=100000, inverted=["dim"])
    rows = _rows(rng, 6000)
    for r in rows[3000:]:
        rt.index(r)
    raw = {c: np.array([r[c] for r in rows[:3000]], dtype=object if t == "STRING" else None)
           for c, (t, sv, _) in SCHEMA.items() if sv}
    raw["lng"] = raw["lng"].astype(np.int64)
    raw["ts"] = raw["ts"].astype(np.int64)
    seg, oseg = H.build_pair("off_c", raw, inverted=["dim"], types={"lng": "LONG", "ts": "LONG", "name": "STRING"})
    gsegs = [E.IndexSegment(ctx, seg), rt.device_segment(ctx)]
    for text in ["SELECT COUNT(*), SUM(met), MAX(dbl) FROM rt WHERE dim > 0",
                 "SELECT SUM(met), MIN(lng) FROM rt WHERE name IN ('a', 'm', 'zz') GROUP BY name, dim"]:
        q = pql.compile(text)
        r = E.InstancePlanMakerImplV2(ctx).make_inter_segment_plan(gsegs, q).execute()
        o = H.oracle_answer([oseg, _oracle_realtime(rt)], q, literal=True)
        fns = [a["fn"] for a in q["aggregations"]]
        if q.get("group_by"):
            m = r.get_aggregation_group_by_result().as_map()
            assert set(m) == set(o["map"])
            for k, v in o["map"].items():
                H.assert_values_equal(m[k], v, fns)
        else:
            H.assert_values_equal(r.get_aggregation_result(), o["results"], fns)


def test_rejected_append_changes_nothing(ctx):
    """pgx_mutable_append validates every column before touching any state.  A batch whose multi-value
    column (tags, index 3) is valid but whose later column (met, index 4) holds a negative dictId is rejected, and the
    consuming segment afterwards answers exactly as if the batch had never been offered."""
    import ctypes as C

    from pinot_amd import native as N
    rng = np.random.default_rng(33)
    rt = RealtimeSegment("rt_bad", SCHEMA, capacity=100000, inverted=["dim"])
    rows = _rows(rng, 3000)
    for r in rows[:2000]:
        rt.index(r)
    rt.device_segment(ctx)  # the first 2000 docs are in HBM
    L = N.lib()
    k = 5
    arrs = []
    for c in SCHEMA:
        if c == "tags":
            arrs.append((np.zeros(2 * k, dtype=np.int32), np.full(k, 2, dtype=np.int32)))
        elif c == "met":
            arrs.append((np.full(k, -1, dtype=np.int32), None))
        else:
            arrs.append((np.zeros(k, dtype=np.int32), None))
    idp = (C.c_void_p * len(arrs))(*[a.ctypes.data for a, _ in arrs])
    cnp = (C.c_void_p * len(arrs))(*[x.ctypes.data if x is not None else None for _, x in arrs])
    assert L.pgx_mutable_append(rt._mut, k, idp, cnp) == N.PGX_ERR_INVALID_ARG
    nd = C.c_int32()
    N.check(L.pgx_mutable_num_docs(rt._mut, C.byref(nd)))
    assert nd.value == 2000
    for r in rows[2000:]:  # the valid rows that follow land right after the first 2000
        rt.index(r)
    for text in QUERIES:
        _check(ctx, rt, text)
