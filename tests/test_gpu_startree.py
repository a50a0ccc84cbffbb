"""GPU parity of star-tree queries: the host traverses the segment's OFF_HEAP star tree
(StarTreeIndexOperator) and the generated kernel scans the selected node ranges / aggregated docs with the remaining
predicates.  Checked against BaseSumStarTreeIndexTest's property (star-tree sums == raw-doc sums), against the same
query with the debug option useStarTree=false (raw scan on the GPU), and against the oracle's restated traversal
(numDocsScanned = docs the reference's StarTreeIndexOperator would return)."""
import copy

import numpy as np
import pytest

from oracle import pinot_oracle as O
from pinot_amd import pql
from pinot_amd import startree as ST
from tests.test_startree import METRICS, QUERIES, make_raw, oseg_of

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from pinot_amd import engine as E
    c = E.Context(0)
    yield c
    c.close()


@pytest.fixture(scope="module", params=[500, 100000])
def staged(ctx, request):
    from pinot_amd import engine as E
    dims, mets = make_raw(60000, seed=9)
    seg = ST.make_star_tree_segment("st%d" % request.param, dims, mets, max_leaf_records=request.param,
                                    inverted=("d3",))
    return E.IndexSegment(ctx, seg), seg, oseg_of(seg)


def _run(ctx, gseg, q):
    from pinot_amd import engine as E
    op = E.InstancePlanMakerImplV2(ctx).make_inner_segment_plan(gseg, q).run()
    blk = op.next_block()
    return blk, op.get_execution_statistics().as_list()


def _as_map(blk, q):
    if q.get("group_by"):
        g = blk.get_aggregation_group_by_result()
        return g.as_map() if g is not None else {}
    return {"": blk.get_aggregation_result()}


@pytest.mark.parametrize("text", QUERIES + ["select sum(m1), sum(m2) from T where d3 = 4 and d4 in (1, 5, 9) group by d1"])
def test_star_tree_query(ctx, staged, text):
    gseg, seg, os_ = staged
    q = pql.compile(text.replace("sum(m1) from", "sum(m1), sum(m2) from") if "sum(m2)" not in text else text)
    raw_q = copy.deepcopy(q)
    raw_q["debug_options"] = {"useStarTree": "false"}
    blk, st = _run(ctx, gseg, q)
    blk_raw, st_raw = _run(ctx, gseg, raw_q)
    gcols = q["group_by"]["columns"] if q.get("group_by") else []
    # the reference property: star-tree sums == raw sums (integer metrics: exact)
    star_map, raw_map = _as_map(blk, q), _as_map(blk_raw, q)
    assert star_map == raw_map
    # raw GPU result == oracle over the raw docs
    raw_docs = np.nonzero(O.filter_mask_vectorized(os_, q.get("filter")))[0]
    exp = O.sum_by_group(os_, raw_docs, METRICS, gcols)
    assert {k: [float(x) for x in v] for k, v in raw_map.items()} == exp
    # docs the star tree selects (StarTreeIndexOperator restated) -> numDocsScanned
    docs = O.star_tree_docs(os_, seg.star_tree, q, seg.total_raw_docs)
    assert st[0] == len(docs)
    assert st_raw[0] == len(raw_docs)
    assert st[3] == st_raw[3] == seg.total_raw_docs


@pytest.fixture(scope="module")
def staged_skip(ctx):
    """d4 skipped for materialization (OffHeapStarTreeBuilder: cardinality above the threshold): the star-node rows and
    every aggregated doc hold the star value for it, so RequestUtils.isFitForStarTreeIndex (:149-163, :195-198)
    sends a query grouping or filtering on d4 to the raw docs."""
    from pinot_amd import engine as E
    dims, mets = make_raw(30000, seed=11)
    seg = ST.make_star_tree_segment("stskip", dims, mets, max_leaf_records=300, skip_cardinality=20)
    assert seg.metadata[ST.SKIP_KEY] == "d4"
    return E.IndexSegment(ctx, seg), seg, oseg_of(seg)


@pytest.mark.parametrize("text", [
    "select sum(m1), sum(m2) from T group by d4",
    "select sum(m1), sum(m2) from T where d4 in (3, 7, 11) group by d1",
    "select sum(m1), sum(m2) from T where d4 = 5",
    "select sum(m1), sum(m2) from T where d1 = 2 group by d2",  # fits: served from the star tree
])
def test_star_tree_skipped_dimension(ctx, staged_skip, text):
    gseg, seg, os_ = staged_skip
    q = pql.compile(text)
    blk, st = _run(ctx, gseg, q)
    gcols = q["group_by"]["columns"] if q.get("group_by") else []
    raw_docs = np.nonzero(O.filter_mask_vectorized(os_, q.get("filter")))[0]
    exp = O.sum_by_group(os_, raw_docs, METRICS, gcols)
    assert {k: [float(x) for x in v] for k, v in _as_map(blk, q).items()} == exp
    uses_d4 = "d4" in text
    if uses_d4:
        assert st[0] == len(raw_docs)  # raw scan
    else:
        assert st[0] == len(O.star_tree_docs(os_, seg.star_tree, q, seg.total_raw_docs))
