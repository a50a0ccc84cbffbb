"""GPU parity on segments the reference itself wrote, and on legacy '%'-padded string dictionaries.

* starTreeSegment.tar.gz (Java-written v1 segment): its star-tree.bin is the Java-serialised ON_HEAP format, which the
  library does not read, so queries scan the raw docs; results must equal the oracle over the same decoded columns
  (raw sum(m1) = 1634).
* Two segments whose STRING column is padded with '%' to different widths: the cross-segment key identity cuts values
  at the padding char (StringDictionary.get, StringDictionary.java:53-66), so equal values merge into one group.
"""
import os
import tarfile

import numpy as np
import pytest

from oracle import pinot_oracle as O
from pinot_amd import pql
from pinot_amd import segment as S
from tests import helpers as H

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from pinot_amd import engine as E
    c = E.Context(0)
    yield c
    c.close()


def oseg_of(seg):
    """The oracle's view of a loaded v1 segment (decoded dictionaries and dictIds of every doc)."""
    cols = {}
    for name, c in seg.columns.items():
        v = c.dictionary_values()
        d = np.array(v, dtype=object) if c.data_type == "STRING" else np.asarray(v).astype(
            np.int64 if c.data_type in ("INT", "LONG") else np.float64)
        cols[name] = O.OColumn(name, c.data_type, d, c.dict_ids().astype(np.int64), c.is_sorted,
                               c.is_sorted or c.inv_bytes is not None, c.bits)  # an index only when its file exists
    return O.OSegment(cols, seg.total_docs, seg.total_raw_docs)


@pytest.fixture(scope="module")
def java_seg(ctx, tmp_path_factory):
    from pinot_amd import engine as E
    d = tmp_path_factory.mktemp("jst")
    with tarfile.open(os.path.join(H.GOLD, "starTreeSegment.tar.gz")) as t:
        t.extractall(d, filter="data")
    seg = S.load_segment(os.path.join(str(d), "starTreeSegment"))
    return E.IndexSegment(ctx, seg), seg, oseg_of(seg)


JAVA_QUERIES = [
    "SELECT SUM(m1), COUNT(*), MIN(m2), MAX(m2) FROM t",
    "SELECT SUM(m1), SUM(m2) FROM t GROUP BY d1",
    "SELECT SUM(m1), AVG(m2) FROM t WHERE d2 = 'd2-v1' GROUP BY d1, d3",
    "SELECT COUNT(*), SUM(m1) FROM t WHERE d1 IN ('d1-v0', 'd1-v2') AND d3 <> 'd3-v0'",
    "SELECT SUM(m2) FROM t WHERE m1 > 0 GROUP BY d2",
]


@pytest.mark.parametrize("text", JAVA_QUERIES)
def test_java_written_segment(ctx, java_seg, text):
    from pinot_amd import engine as E
    gseg, seg, os_ = java_seg
    q = pql.compile(text)
    op = E.InstancePlanMakerImplV2(ctx).make_inner_segment_plan(gseg, q).run()
    blk = op.next_block()
    st = op.get_execution_statistics().as_list()
    o = H.oracle_answer([os_], q, literal=True)
    assert st == list(o["stats"])
    fns = [a["fn"] for a in q["aggregations"]]
    if q.get("group_by"):
        m = blk.get_aggregation_group_by_result().as_map()
        assert set(m) == set(o["map"])
        for k, v in o["map"].items():
            H.assert_values_equal(m[k], v, fns)
    else:
        got = blk.get_aggregation_result()
        H.assert_values_equal(got, o["results"], fns)
        if text == JAVA_QUERIES[0]:
            assert got[0] == 1634.0 and got[1] == 1000


def test_percent_padding_across_segments(ctx):
    """values of a '%'-padded column compare equal across segments of different dictionary widths."""
    from pinot_amd import engine as E
    rng = np.random.default_rng(5)
    vocab = [["ab", "abc", "x"], ["ab", "x", "xyzw"]]
    gsegs, osegs = [], []
    for i, words in enumerate(vocab):
        n = 5000
        raw = {"s": np.array(words, dtype=object)[rng.integers(0, len(words), n)].astype(str),
               "m": rng.integers(0, 1000, n).astype(np.int32)}
        col = S.make_column("s", raw["s"], pad="%")
        seg = S.make_segment("pad%d" % i, [col, S.make_column("m", raw["m"])])
        seg = S.load_segment(S.write_segment(seg, "/tmp/pgx_pad_test"))  # metadata round trip: pad char '%'
        assert seg.columns["s"].pad_char == "%"
        gsegs.append(E.IndexSegment(ctx, seg))
        osegs.append(O.OSegment.from_raw(raw))
    q = pql.compile("SELECT SUM(m), COUNT(*) FROM t GROUP BY s")
    blk = E.InstancePlanMakerImplV2(ctx).make_inter_segment_plan(gsegs, q).execute()
    got = blk.get_aggregation_group_by_result().as_map()
    exp = H.oracle_answer(osegs, q)["map"]
    assert set(got) == {"ab", "abc", "x", "xyzw"} == set(exp)
    for k, v in exp.items():
        H.assert_values_equal(got[k], v, ["sum", "count"])
