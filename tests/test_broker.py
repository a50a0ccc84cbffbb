"""Server response + broker reduce (pinot_amd/broker.py), pinned by BrokerReduceServiceTest
(pinot-core/src/test/java/com/linkedin/pinot/query/executor/BrokerReduceServiceTest.java:163,287,397-413): two segments
of simpleData200001.avro per server, 2 and 10 servers answering the same instance request.

CPU tests: the server responses come from the CPU oracle (the checker).  GPU test: they come from the GPU server path
(ServerQueryExecutor over staged segments)."""
import numpy as np
import pytest

from oracle import pinot_oracle as O
from pinot_amd import broker as B
from pinot_amd import datatable as D
from pinot_amd import pql
from tests import helpers as H

MULTI = ("SELECT COUNT(*), SUM(met), MAX(met), MIN(met), AVG(met), DISTINCTCOUNT(dim0), DISTINCTCOUNT(dim1) "
         "FROM midas")
BASIC = "SELECT COUNT(*), SUM(met), MAX(met), MIN(met), AVG(met) FROM midas"
GROUPED = "SELECT SUM(met), COUNT(*), MIN(met), AVG(met) FROM midas GROUP BY dim0 TOP 4"


def _oracle_response(q, osegs):
    a = H.oracle_answer(osegs, q)
    if q.get("group_by"):
        return B.InstanceResponse(group_by=[{k: v[i] for k, v in a["map"].items()} for i in range(len(q["aggregations"]))],
                                  stats=a["stats"])
    res = []
    for agg, v in zip(q["aggregations"], a["results"]):
        if agg["fn"].startswith("percentile") and not agg["fn"].startswith("percentileest"):  # the oracle's DoubleArrayList -> the (value, count) multiset
            vals, cnts = np.unique(np.asarray(v, dtype=np.float64), return_counts=True)
            v = [(float(x), int(c)) for x, c in zip(vals, cnts)]
        res.append(v)
    return B.InstanceResponse(aggregation=res, stats=a["stats"])


@pytest.fixture(scope="module")
def osegs():
    raw = dict(np.load(H.GOLD + "/simple_data_200001.npz"))
    return [O.OSegment.from_raw(raw, inverted=list(raw)) for _ in range(2)]


def _by_fn(resp):
    return {r.function: r.value for r in resp.aggregation_results}


def test_two_and_ten_servers_match_reference_goldens(osegs):
    exp = H.load_expected()["broker_reduce"]
    q = pql.compile(MULTI)
    one = _oracle_response(q, osegs)
    svc = B.BrokerReduceService()
    for n, key in ((2, "servers_2"), (10, "servers_10")):
        resp = svc.reduce_on_data_table(q, {"localhost:%d" % (1111 * i): one for i in range(n)})
        got = _by_fn(resp)
        for fn, v in exp[key].items():  # checkAggregationResult: Double.valueOf(value) == expected
            assert float(got[fn]) == float(v), (fn, got[fn], v)
        assert got["count_star"] == str(exp[key]["count_star"])  # long -> toString
        assert got["sum_met"] == B.java_format_5f(float(got["sum_met"]))  # doubles -> %1.5f
        assert resp.num_docs_scanned == n * 400002 and resp.total_docs == n * 400002
        assert not resp.processing_exceptions


def test_group_by_reduce_top_n_and_rendering(osegs):
    q = pql.compile(GROUPED)
    resp = _oracle_response(q, osegs)
    red = B.BrokerReduceService().reduce_on_data_table(q, {"a": resp, "b": resp, "c": resp})
    full = H.oracle_answer(osegs * 3, q)["map"]
    fns = [a["fn"] for a in q["aggregations"]]
    assert [r.function for r in red.aggregation_results] == ["sum_met", "count_star", "min_met", "avg_met"]
    for i, (r, fn) in enumerate(zip(red.aggregation_results, fns)):
        assert r.group_by_columns == ["dim0"] and len(r.group_by_result) == min(4, len(full))
        vals = {k: B._reduce(fn, [v[i]]) for k, v in full.items()}
        order = sorted(vals.values(), reverse=fn != "min")[:4]
        assert [row.value for row in r.group_by_result] == [B._format(fn, v) for v in order]
        for row in r.group_by_result:
            assert B._format(fn, vals[row.group[0]]) == row.value


def test_exception_responses_and_stats():
    q = pql.compile(BASIC)
    ok = B.InstanceResponse(aggregation=[3, 6.0, 3.0, 1.0, (6.0, 3)], stats=[3, 1, 12, 10])
    bad = B.InstanceResponse(exceptions={B.QUERY_EXECUTION_ERROR_CODE: "segment failed"})
    resp = B.BrokerReduceService().reduce_on_data_table(q, {"s1": ok, "s2": bad, "s3": None})
    assert [(e.error_code, e.message) for e in resp.processing_exceptions] == [(200, "segment failed")]
    assert _by_fn(resp) == {"count_star": "3", "sum_met": "6.00000", "max_met": "3.00000", "min_met": "1.00000",
                            "avg_met": "2.00000"}
    assert (resp.num_docs_scanned, resp.num_entries_scanned_in_filter, resp.num_entries_scanned_post_filter,
            resp.total_docs) == (3, 1, 12, 10)
    empty = B.BrokerReduceService().reduce_on_data_table(q, {"s": B.InstanceResponse(aggregation=[0, 0.0, -np.inf,
                                                                                                   np.inf, (0.0, 0)])})
    assert _by_fn(empty) == {"count_star": "0", "sum_met": "0.00000", "max_met": "-Infinity", "min_met": "Infinity",
                             "avg_met": "0.00000"}
    assert B.BrokerReduceService().reduce_on_data_table(q, {}).aggregation_results == []


def test_java_format_rounds_shortest_decimal_half_up():
    assert B.java_format_5f(0.000015) == "0.00002"  # Java: HALF_UP of "1.5E-5"; printf would give 0.00001
    assert B.java_format_5f(2.5) == "2.50000"
    assert B.java_format_5f(-1.234565) == "-1.23457"
    assert B.java_format_5f(1e20) == "100000000000000000000.00000"


@pytest.mark.gpu
def test_gpu_servers_match_reference_goldens():
    from pinot_amd import engine as E
    raw = dict(np.load(H.GOLD + "/simple_data_200001.npz"))
    ctx = E.Context(0)
    try:
        segs = []
        for i in range(2):
            seg, _ = H.build_pair("midas_%d" % i, raw, inverted=list(raw), column_types={"met": "METRIC"})
            segs.append(E.IndexSegment(ctx, seg))
        server = B.ServerQueryExecutor(ctx)
        exp = H.load_expected()["broker_reduce"]
        q = pql.compile(MULTI)
        for n, key in ((2, "servers_2"), (10, "servers_10")):
            # odd servers answer over the wire (DataTable bytes, pinot_amd/datatable.py), even ones in process
            resps = {"localhost:%d" % i: (D.response_to_datatable(q, server.process_query(q, segs)) if i % 2
                                          else server.process_query(q, segs)) for i in range(n)}
            got = _by_fn(B.BrokerReduceService().reduce_on_data_table(q, resps))
            for fn, v in exp[key].items():
                assert float(got[fn]) == float(v), (fn, got[fn], v)
        osegs = [O.OSegment.from_raw(raw, inverted=list(raw)) for _ in range(2)]
        qg = pql.compile(GROUPED)
        gpu = B.BrokerReduceService().reduce_on_data_table(qg, {"a": server.process_query(qg, segs),
                                                                "b": server.process_query(qg, segs)})
        cpu = B.BrokerReduceService().reduce_on_data_table(qg, {"a": _oracle_response(qg, osegs),
                                                                "b": _oracle_response(qg, osegs)})
        assert gpu == cpu
    finally:
        ctx.close()


def test_hll_functions_reduce_and_render(osegs):
    """DISTINCTCOUNTHLL across servers: HyperLogLog.addAll of the server estimators, cardinality() rendered as a long
    (query/aggregation/function/DistinctCountHLLAggregationFunction.java combine / reduce / getFunctionName), equal to
    the estimate over all servers' distinct hash codes."""
    from pinot_amd import hll
    q = pql.compile("SELECT DISTINCTCOUNTHLL(dim0), DISTINCTCOUNT(dim0) FROM midas")
    one = _oracle_response(q, osegs)
    resp = B.BrokerReduceService().reduce_on_data_table(q, {"s1": one, "s2": one, "s3": one})
    got = _by_fn(resp)
    assert set(got) == {"distinctCountHLL_dim0", "distinctCount_dim0"}
    regs = np.array(one.aggregation[0], dtype=np.uint8)
    assert got["distinctCountHLL_dim0"] == str(hll.cardinality(regs))
    assert list(hll.from_ints(one.aggregation[1])) == list(regs)  # registers are a function of the hash-code set
    empty = B.BrokerReduceService().reduce_on_data_table(pql.compile("SELECT FASTHLL(dim0) FROM midas"),
                                                          {"s": B.InstanceResponse(aggregation=[None])})
    assert _by_fn(empty) == {"fasthll_dim0": "0"}
