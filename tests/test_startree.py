"""Star-tree index, CPU side: the builder (pinot_amd/startree.py, restating
OffHeapStarTreeBuilder + StarTreeSerDe OFF_HEAP) and the oracle's restatement of StarTreeIndexOperator, checked with
the reference's own property (pinot-core/src/test/java/com/linkedin/pinot/core/startree/BaseSumStarTreeIndexTest.java):
for every hard-coded query, sums over the docs the star tree selects equal sums over the raw docs."""
import numpy as np
import pytest

from oracle import pinot_oracle as O
from pinot_amd import pql
from pinot_amd import startree as ST

# BaseSumStarTreeIndexTest._hardCodedQueries (:50-65) on INT dimensions (d<k>-v<i> -> i)
QUERIES = [
    "select sum(m1) from T",
    "select sum(m1) from T where d1 = 1",
    "select sum(m1) from T where d1 <> 1",
    "select sum(m1) from T where d1 between 1 and 3",
    "select sum(m1) from T where d1 in (1, 2)",
    "select sum(m1) from T where d1 in (1, 2) and d2 not in (1)",
    "select sum(m1) from T group by d1",
    "select sum(m1) from T group by d1, d2",
    "select sum(m1) from T where d1 = 2 group by d1",
    "select sum(m1) from T where d1 between 1 and 3 group by d2",
    "select sum(m1) from T where d1 = 2 group by d2, d3",
    "select sum(m1) from T where d1 <> 1 group by d2",
    "select sum(m1) from T where d1 in (1, 2) group by d2",
    "select sum(m1) from T where d1 in (1, 2) and d2 not in (1) group by d3",
    "select sum(m1) from T where d1 in (1, 2) and d2 not in (1) group by d3, d4",
]
METRICS = ["m1", "m2"]


def make_raw(n, seed=4):
    rng = np.random.default_rng(seed)
    dims = {"d1": rng.integers(0, 4, n), "d2": rng.integers(0, 6, n), "d3": rng.integers(0, 10, n),
            "d4": rng.integers(0, 40, n)}
    mets = {"m1": rng.integers(0, 1 << 16, n), "m2": rng.integers(0, 1000, n)}
    return dims, mets


def oseg_of(seg):
    """The oracle's view of a v1 segment: dictionaries and per-doc dictIds of every doc (raw + aggregated)."""
    cols = {}
    for name, c in seg.columns.items():
        d = np.asarray(c.dictionary_values()).astype(np.int64)
        cols[name] = O.OColumn(name, c.data_type, d, c.dict_ids().astype(np.int64), c.is_sorted, c.has_inverted, c.bits)
    return O.OSegment(cols, seg.total_docs, seg.total_raw_docs)


@pytest.fixture(scope="module")
def star_seg():
    dims, mets = make_raw(20000)
    seg = ST.make_star_tree_segment("st", dims, mets, max_leaf_records=500)
    return seg, oseg_of(seg), dims, mets


def test_off_heap_bytes_round_trip(star_seg):
    seg, _, _, _ = star_seg
    names, nodes = ST.parse(seg.star_tree)
    assert names == {0: "d1", 1: "d2", 2: "d3", 3: "d4"}
    n2, nodes2 = O.parse_star_tree_off_heap(seg.star_tree)
    assert n2 == names and np.array_equal(nodes, nodes2)
    assert nodes[0][0] == -1 and nodes[0][1] == -1  # root: ALL / ALL
    # BFS layout: children ranges are contiguous and sorted by value, ALL (-1) first
    for x in nodes:
        if x[5] != -1:
            vals = nodes[x[5]:x[6] + 1, 1]
            assert np.all(np.diff(vals) > 0)
    assert seg.total_docs > seg.total_raw_docs == 20000


def test_aggregated_docs_equal_raw_sums(star_seg):
    """Every node's aggregated doc holds the sums of the raw docs under its path (createAggDocForAllNodes), as the
    Java-written fixture starTreeSegment.tar.gz shows for (d1-v0, ALL, ALL)."""
    seg, os_, dims, mets = star_seg
    names, nodes = ST.parse(seg.star_tree)
    d_ids = {k: os_.columns[k].dict_ids for k in dims}
    raw = seg.total_raw_docs

    def path_of(i):  # walk up via the BFS parent relation
        parent = {c: p for p, x in enumerate(nodes) if x[5] != -1 for c in range(x[5], x[6] + 1)}
        path = {}
        while i:
            if nodes[i][1] != -1:
                path[names[int(nodes[i][0])]] = int(nodes[i][1])
            i = parent[i]
        return path

    rng = np.random.default_rng(0)
    for i in [0] + list(rng.choice(len(nodes), size=min(40, len(nodes) - 1), replace=False)):
        path = path_of(int(i))
        sel = np.ones(raw, dtype=bool)
        for k, v in path.items():
            sel &= d_ids[k][:raw] == v
        agg = int(nodes[i][4])
        assert agg >= raw
        for m in METRICS:
            col = os_.columns[m]
            assert int(col.dictionary[col.dict_ids[agg]]) == int(col.dictionary[col.dict_ids[:raw][sel]].sum())


@pytest.mark.parametrize("text", QUERIES)
def test_star_tree_docs_sum_equals_raw_scan(star_seg, text):
    seg, os_, _, _ = star_seg
    q = pql.compile(text)
    gcols = q["group_by"]["columns"] if q.get("group_by") else []
    raw_docs = np.nonzero(O.filter_mask_vectorized(os_, q.get("filter")))[0]
    exp = O.sum_by_group(os_, raw_docs, METRICS, gcols)
    docs = O.star_tree_docs(os_, seg.star_tree, q, seg.total_raw_docs)
    got = O.sum_by_group(os_, docs, METRICS, gcols)
    assert got == exp
    if not q.get("filter") and not gcols:
        assert len(docs) == 1  # the root's aggregated doc


def test_skip_materialization_dimension():
    """OffHeapStarTreeBuilder skipMaterializationForDimensions (:308-322, :738-745): a dimension above the cardinality
    threshold leaves the split order and holds ALL in every star-node row and aggregated doc."""
    dims, mets = make_raw(6000, seed=5)
    seg = ST.make_star_tree_segment("sk", dims, mets, max_leaf_records=100, skip_cardinality=20)
    assert seg.metadata[ST.SKIP_KEY] == "d4"
    assert "d4" not in seg.metadata["startree.split.order"].split(",")
    names, nodes = ST.parse(seg.star_tree)
    assert all(names[int(x[0])] != "d4" for x in nodes[1:])
    d4 = seg.columns["d4"]
    ids = d4.dict_ids()
    assert np.all(ids[seg.total_raw_docs:] == 0)  # dictId 0 = Integer.MIN_VALUE, the star value
    # star-tree sums still equal raw sums for queries that do not touch d4
    os_ = oseg_of(seg)
    for text in QUERIES[:6]:
        q = pql.compile(text)
        raw_docs = np.nonzero(O.filter_mask_vectorized(os_, q.get("filter")))[0]
        docs = O.star_tree_docs(os_, seg.star_tree, q, seg.total_raw_docs)
        assert O.sum_by_group(os_, docs, METRICS, []) == O.sum_by_group(os_, raw_docs, METRICS, [])


@pytest.mark.parametrize("leaf", [500, 60])
def test_dense_combination_count_equals_sort_path(leaf):
    """The builder's dense-table unique combinations (a range whose key span is small) give the segment the sort +
    reduceat path gives: the same OFF_HEAP tree bytes, and every column's dictionary and dictIds."""
    dims, mets = make_raw(20000)
    a = ST.make_star_tree_segment("st", dims, mets, max_leaf_records=leaf)
    b = ST.make_star_tree_segment("st", dims, mets, max_leaf_records=leaf, dense_limit=0)
    assert a.star_tree == b.star_tree and a.total_docs == b.total_docs
    for name in a.columns:
        assert np.array_equal(np.asarray(a.columns[name].dictionary_values()),
                              np.asarray(b.columns[name].dictionary_values()))
        assert np.array_equal(a.columns[name].dict_ids(), b.columns[name].dict_ids())
