"""CPU tests of the request slicing past one library query's shape limits (engine.agg_slices) and of the operator's
merge of the slices' blocks (_GpuOperator._run_slices), with a stand-in for the library query: every function's value
is a pure function of (function, column, group key), so the merged block must equal the unsliced one."""
import pytest

from pinot_amd import engine as E
from pinot_amd import pql


def test_fits_one_query_is_one_slice():
    assert E.agg_slices(pql.compile("SELECT SUM(m), MIN(m), MAX(m) FROM t GROUP BY g1, g2")) == [[0, 1, 2]]


def test_more_than_eight_functions():
    aggs = ", ".join("SUM(c%d)" % i for i in range(11))
    assert E.agg_slices(pql.compile("SELECT %s FROM t" % aggs)) == [list(range(8)), [8, 9, 10]]
    aggs = ", ".join(["COUNT(*)"] * 17)
    assert E.agg_slices(pql.compile("SELECT %s FROM t" % aggs)) == [list(range(8)), list(range(8, 16)), [16]]


def test_column_limit():
    flt = " AND ".join("f%d > 0" % i for i in range(12))  # 12 filter columns + 2 group columns = 14 fixed
    q = pql.compile("SELECT SUM(a), SUM(b), MIN(a), SUM(c), MAX(d) FROM t WHERE %s GROUP BY g1, g2" % flt)
    assert E.agg_slices(q) == [[0, 1, 2], [3, 4]]  # a, b (16 columns) + a again; c starts a new slice


def test_extended_base_slots():
    # MINMAXRANGE takes two base slots (MIN + MAX) beside the base COUNT(*); DISTINCTCOUNT none
    q = pql.compile("SELECT MINMAXRANGE(a), MINMAXRANGE(b), MINMAXRANGE(c), MINMAXRANGE(d), DISTINCTCOUNT(e), SUM(f) "
                    "FROM t")
    assert E.agg_slices(q) == [[0, 1, 2], [3, 4, 5]]  # 1 + 3 x 2 slots, then 1 + 2 + 0 + 1


def test_avgmv_value_count_plane():
    aggs = ", ".join(["AVGMV(v)"] * 5)
    assert E.agg_slices(pql.compile("SELECT %s FROM t" % aggs)) == [[0, 1, 2, 3], [4]]


def test_avgmv_beside_an_extended_function():
    # an extended slice keeps AVGMV in its base query, whose value-count plane is a slot too:
    # DISTINCTCOUNT + 7 x AVGMV needs 1 (base COUNT(*)) + 0 + 7 x 2 slots, so no slice may hold more than 3 AVGMV
    aggs = ", ".join(["DISTINCTCOUNT(d)"] + ["AVGMV(v)"] * 7)
    sl = E.agg_slices(pql.compile("SELECT %s FROM t GROUP BY g" % aggs))
    assert sl == [[0, 1, 2, 3], [4, 5, 6, 7]]  # 1 + 0 + 3 x 2 = 7, then 4 x 2 = 8


def _value(a, key):
    return (len(a["fn"]) * 1000 + sum(map(ord, a["column"]))) * (1 + sum(map(ord, key)))


class _FakeOp(E._GpuOperator):
    """One library query's worth: refuses a request past the limits, else renders deterministic values."""

    def next_block(self):
        if len(E.agg_slices(self.request)) > 1:
            return super().next_block()
        aggs = self.request["aggregations"]
        assert len(aggs) <= E.MAX_AGGS
        st = E.ExecutionStatistics(100, 7, 100 * 3, 1000)
        if not self.request.get("group_by"):
            return E.IntermediateResultsBlock(aggregation_result=[_value(a, "") for a in aggs], stats=st)
        keys = ["k%d\tx" % i for i in range(5)]
        if self.request.get("filter") and not self.combine:
            return E.IntermediateResultsBlock(stats=st)  # no group selected (inner segment plan)
        order = keys if len(aggs) % 2 else keys[::-1]  # the slices find the groups in different orders
        gb = E.AggregationGroupByResult(order, [[_value(a, k) for a in aggs] for k in order], [a["fn"] for a in aggs],
                                        "ARRAY_BASED")
        blk = E.IntermediateResultsBlock(aggregation_group_by_result=gb, stats=st)
        if self.combine:
            blk.trimmed = [{k: _value(a, k) for k in order[:3]} for a in aggs]
        return blk


@pytest.mark.parametrize("group", [False, True])
def test_slices_merge(group):
    aggs = ", ".join("%s(c%d)" % (f, i) for i, f in enumerate(["SUM", "MIN", "MAX", "AVG"] * 3))
    q = pql.compile("SELECT %s FROM t%s" % (aggs, " GROUP BY g1, g2" if group else ""))
    blk = _FakeOp(None, q, [], combine=True).next_block()
    # numEntriesScannedPostFilter: docs x the request's projected columns (12 aggregated + the 2 group columns)
    assert blk.stats.as_list() == [100, 7, 100 * (14 if group else 12), 1000]
    if not group:
        assert blk.get_aggregation_result() == [_value(a, "") for a in q["aggregations"]]
        return
    m = blk.get_aggregation_group_by_result().as_map()
    assert m == {k: [_value(a, k) for a in q["aggregations"]] for k in ["k%d\tx" % i for i in range(5)]}
    assert len(blk.trimmed) == 12 and all(len(t) == 3 for t in blk.trimmed)
    assert blk.trimmed[9] == {k: _value(q["aggregations"][9], k) for k in blk.trimmed[9]}


def test_slices_no_group_selected():
    aggs = ", ".join("SUM(c%d)" % i for i in range(10))
    q = pql.compile("SELECT %s FROM t WHERE f > 3 GROUP BY g" % aggs)
    blk = _FakeOp(None, q, [], combine=False).next_block()
    assert blk.get_aggregation_group_by_result() is None


class _StarOp(_FakeOp):
    """Slices whose functions all qualify for the star-tree scan fewer docs unless useStarTree=false (with
    `empty`, a filter matching nothing: both scan 0 docs, but only the raw docs count entries scanned in filter)."""
    runs = []
    empty = False

    def next_block(self):
        if len(E.agg_slices(self.request)) > 1:
            return E._GpuOperator.next_block(self)
        star = str((self.request.get("debug_options") or {}).get("useStarTree", "true")) != "false"
        qualifies = all(a["fn"] == "sum" for a in self.request["aggregations"])
        on_tree = star and qualifies
        docs = 0 if _StarOp.empty else (10 if on_tree else 100)
        entries = 0 if on_tree else 1000
        _StarOp.runs.append(docs if not _StarOp.empty else entries)
        return E.IntermediateResultsBlock(aggregation_result=[docs] * len(self.request["aggregations"]),
                                          stats=E.ExecutionStatistics(docs, entries, 0, 1000))


def test_slices_rerun_on_raw_docs_when_star_tree_disagrees():
    # the first slice qualifies for the star-tree, the second does not: the request runs on the raw docs throughout
    aggs = ", ".join(["SUM(m)"] * 8 + ["MIN(m)"])
    q = pql.compile("SELECT %s FROM t" % aggs)
    _StarOp.runs = []
    blk = _StarOp(None, q, [], combine=True).next_block()
    assert _StarOp.runs == [10, 100, 100, 100]
    assert blk.get_aggregation_result() == [100] * 9 and blk.stats.num_docs_scanned == 100
    # every slice qualifies: no re-run
    _StarOp.runs = []
    q = pql.compile("SELECT %s FROM t" % ", ".join(["SUM(m)"] * 10))
    blk = _StarOp(None, q, [], combine=True).next_block()
    assert _StarOp.runs == [10, 10] and blk.stats.num_docs_scanned == 10


def test_slices_rerun_when_only_entries_scanned_differ():
    # a filter that matches nothing scans 0 docs on the tree and on the raw docs; the entries scanned in
    # filter still tell the star-tree slice from the raw one, and the request re-runs on the raw docs
    aggs = ", ".join(["SUM(m)"] * 8 + ["MIN(m)"])
    q = pql.compile("SELECT %s FROM t WHERE d = 3" % aggs)
    _StarOp.runs, _StarOp.empty = [], True
    try:
        blk = _StarOp(None, q, [], combine=True).next_block()
    finally:
        _StarOp.empty = False
    assert _StarOp.runs == [0, 1000, 1000, 1000]
    assert blk.stats.num_entries_scanned_in_filter == 1000
