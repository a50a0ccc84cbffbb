"""GPU parity of the batched plan/launch pipeline (pgx_host.cpp run_batched): a long segment list is planned and
launched in batches on one stream (the host plans batch k + 1 while the GPU runs batch k); every batch decodes group
keys against global dictionaries over the WHOLE list and accumulates into one dense table and one output block.
PGX_BATCH_SEGS=2 batches a 7-segment list (4 batches, the last one short) whose segments all hold DIFFERENT
dictionaries, so the per-batch remap tables must agree with the whole-list key space.  Checked against the oracle's
combine over all segments, statistics included, and against the unbatched path (PGX_BATCH_SEGS=0)."""
import numpy as np
import pytest

from pinot_amd import pql
from tests import helpers as H
from tests.test_gpu_parity import _rand_segment

pytestmark = pytest.mark.gpu

NSEG = 7


@pytest.fixture(scope="module")
def ctx():
    from pinot_amd import engine as E
    c = E.Context(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def segs(ctx):
    from pinot_amd import engine as E
    gsegs, osegs, fmt = [], [], None
    for i in range(NSEG):
        rng = np.random.default_rng(100 + i)
        n = 65536 + 8192 * i + 97 * i
        raw = _rand_segment(rng, n, {"a": 3000, "b": 40, "c": 700, "s": 6, "g1": 13, "m": 5000}, "b%d" % i,
                            sorted_col="s")
        raw["b"] = (raw["b"] % 50).astype(np.int32)   # shared value domain (so IN lists hit every segment) ...
        raw["g1"] = (raw["g1"] % 11).astype(np.int32)  # ... but each segment's dictionary is its own
        seg, oseg = H.build_pair("b%d" % i, raw, inverted=("b", "c"))
        gsegs.append(E.IndexSegment(ctx, seg))
        osegs.append(oseg)
    return gsegs, osegs


QUERIES = [
    "SELECT COUNT(*), SUM(m), MIN(m), MAX(m) FROM t WHERE a > 0",
    "SELECT COUNT(*), SUM(m) FROM t WHERE b IN (1, 2, 3, 4, 5, 6, 7, 8, 9, 10) AND b <> 4",
    "SELECT SUM(m), COUNT(*) FROM t WHERE b IN (3, 9, 27) OR c > 0 GROUP BY g1",
    "SELECT SUM(m), MAX(m) FROM t GROUP BY g1, b",
    "SELECT COUNT(*), MIN(m) FROM t WHERE (b = 7 OR a < 0) AND s > -100000000 GROUP BY b",
]


def _answer(ctx, gsegs, q):
    from pinot_amd import engine as E
    blk = E.InstancePlanMakerImplV2(ctx).make_inter_segment_plan(gsegs, q).execute()
    if q.get("group_by"):
        g = blk.get_aggregation_group_by_result()
        return (g.as_map() if g is not None else {}), blk.stats.as_list()
    return blk.get_aggregation_result(), blk.stats.as_list()


@pytest.mark.parametrize("text", QUERIES)
def test_batched_equals_oracle_and_unbatched(ctx, segs, text, monkeypatch):
    gsegs, osegs = segs
    q = pql.compile(text)
    fns = [a["fn"] for a in q["aggregations"]]
    monkeypatch.setenv("PGX_BATCH_SEGS", "2")
    got, st = _answer(ctx, gsegs, q)
    monkeypatch.setenv("PGX_BATCH_SEGS", "0")
    ref, st_ref = _answer(ctx, gsegs, q)
    o = H.oracle_answer(osegs, q, literal=True)
    assert st == st_ref == list(o["stats"])
    if q.get("group_by"):
        assert set(got) == set(o["map"]) == set(ref)
        for k, v in o["map"].items():
            H.assert_values_equal(got[k], v, fns)
        assert got == ref
    else:
        H.assert_values_equal(got, o["results"], fns)
        assert got == ref


@pytest.mark.parametrize("rchunk", ["0", "1"])
@pytest.mark.parametrize("text", QUERIES)
def test_compacted_selected_rows_equal_oracle(ctx, segs, text, rchunk, monkeypatch):
    """Bitmap programs evaluated in the query kernel (PGX_RCHUNK=1, which also packs each sub-step's selected rows into
    consecutive lanes -- wave prefix + LDS staging -- before the value gathers / image lookups, group-key remaps and
    table atomics) or by the separate pass (PGX_RCHUNK=0).  The segments' dictionaries differ, so remapped group keys are
    gathered in the packed domain too."""
    gsegs, osegs = segs
    q = pql.compile(text)
    fns = [a["fn"] for a in q["aggregations"]]
    monkeypatch.setenv("PGX_RCHUNK", rchunk)
    got, st = _answer(ctx, gsegs, q)
    o = H.oracle_answer(osegs, q, literal=True)
    assert st == list(o["stats"])
    if q.get("group_by"):
        assert set(got) == set(o["map"])
        for k, v in o["map"].items():
            H.assert_values_equal(got[k], v, fns)
    else:
        H.assert_values_equal(got, o["results"], fns)
