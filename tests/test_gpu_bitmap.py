"""GPU parity of the bitmap inverted-index path: leaves on inverted columns are expanded from the
segment's RoaringBitmap bytes on the device (pgx_roaring_expand) into per-segment doc masks the query kernel reads.

Segments span several 65,536-doc roaring chunks and hold both container kinds (bitmap containers for the
low-cardinality column, array containers for the high-cardinality one).  Every query is checked against the CPU
oracle, and against the same segment without inverted indexes (the scan path), bit-exactly."""
import numpy as np
import pytest

from pinot_amd import pql
from tests import helpers as H

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from pinot_amd import engine as E
    c = E.Context(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def segs(ctx):
    from pinot_amd import engine as E
    rng = np.random.default_rng(11)
    n = 3 * 65536 + 4321  # four roaring chunks, the last one partial
    raw = {"x": rng.integers(0, 5, n).astype(np.int32),        # ~13k docs / value / chunk -> bitmap containers
           "y": rng.integers(0, 300, n).astype(np.int32),      # ~220 docs / value / chunk -> array containers
           "z": rng.integers(-50, 50, n).astype(np.int32),
           "g": rng.integers(0, 17, n).astype(np.int32),
           "m": rng.integers(0, 1 << 20, n).astype(np.int32)}
    inv_seg, oseg = H.build_pair("inv", raw, inverted=("x", "y", "g"))
    scan_seg, _ = H.build_pair("scan", raw)
    assert inv_seg.columns["x"].inv_bytes is not None
    return E.IndexSegment(ctx, inv_seg), E.IndexSegment(ctx, scan_seg), oseg


QUERIES = [
    "SELECT COUNT(*), SUM(m) FROM t WHERE x = 3",
    "SELECT COUNT(*), SUM(m) FROM t WHERE x <> 3",
    "SELECT COUNT(*), SUM(m), MIN(m), MAX(m) FROM t WHERE x IN (0, 2, 4)",
    "SELECT COUNT(*), SUM(m) FROM t WHERE y NOT IN (1, 7, 299)",
    "SELECT COUNT(*), SUM(m) FROM t WHERE y IN (5, 6, 7, 8, 100, 250)",
    "SELECT COUNT(*), SUM(m) FROM t WHERE (x = 1 OR y IN (3, 4, 5)) AND z > 10",
    "SELECT COUNT(*), SUM(m) FROM t WHERE x <> 0 AND y <> 5 AND g = 3",
    "SELECT SUM(m), COUNT(*) FROM t WHERE (x IN (1, 2) OR y = 9) AND x <> 2 GROUP BY g",
    "SELECT SUM(m) FROM t WHERE y = 123456 GROUP BY g",
    # all-bitmap filters: one combined doc mask per segment (pgx_roaring_program), incl. empty and flipped leaves
    "SELECT COUNT(*), SUM(m) FROM t WHERE x = 1 OR y IN (3, 4, 5)",
    "SELECT COUNT(*), SUM(m) FROM t WHERE (y = 123456 OR x = 2) AND x <> 7",
    "SELECT COUNT(*), MIN(m), MAX(m) FROM t WHERE (x IN (0, 4) OR y IN (10, 20, 30)) AND y NOT IN (20, 21) AND g <> 5",
    "SELECT SUM(m), COUNT(*) FROM t WHERE (x = 3 OR g IN (1, 2)) AND (y <> 8 OR x = 0) GROUP BY g",
]


@pytest.mark.parametrize("text", QUERIES)
def test_bitmap_leaves_match_oracle_and_scan(ctx, segs, text):
    from pinot_amd import engine as E
    inv, scan, oseg = segs
    q = pql.compile(text)
    pm = E.InstancePlanMakerImplV2(ctx)
    op = pm.make_inner_segment_plan(inv, q).run()
    blk = op.next_block()
    st = op.get_execution_statistics().as_list()
    blk_scan = pm.make_inner_segment_plan(scan, q).run().next_block()
    o = H.oracle_answer([oseg], q, literal=True)
    fns = [a["fn"] for a in q["aggregations"]]
    assert st == list(o["stats"])  # incl. numEntriesScannedInFilter (literal iterator algebra)
    if q.get("group_by"):
        m = blk.get_aggregation_group_by_result()
        m = m.as_map() if m is not None else {}
        assert set(m) == set(o["map"])
        for k, v in o["map"].items():
            H.assert_values_equal(m[k], v, fns)
        ms = blk_scan.get_aggregation_group_by_result()
        assert m == (ms.as_map() if ms is not None else {})
    else:
        H.assert_values_equal(blk.get_aggregation_result(), o["results"], fns)
        assert blk.get_aggregation_result() == blk_scan.get_aggregation_result()


@pytest.mark.parametrize("order", ["isi", "si", "ssi"])
@pytest.mark.parametrize("text", QUERIES)
def test_mixed_bitmap_and_scan_segments_in_one_query(ctx, segs, text, order):
    """One launch over an inverted segment (combined bitmap program or per-leaf masks) and a scan-only segment: the
    combine over both equals the oracle's combine of the identical segments.  The orders put a scan-only segment first
    too ("si", "ssi"), so a leaf planned for a scan segment must not be reused for an inverted one that shares its
    dictionary and binding (EQ / IN / NEQ / NOT_IN single leaves included)."""
    from pinot_amd import engine as E
    inv, scan, oseg = segs
    q = pql.compile(text)
    pm = E.InstancePlanMakerImplV2(ctx)
    blk = pm.make_inter_segment_plan([inv if c == "i" else scan for c in order], q).execute()
    o = H.oracle_answer([oseg] * len(order), q, literal=True)
    fns = [a["fn"] for a in q["aggregations"]]
    if q.get("group_by"):
        m = blk.get_aggregation_group_by_result()
        m = m.as_map() if m is not None else {}
        assert set(m) == set(o["map"])
        for k, v in o["map"].items():
            H.assert_values_equal(m[k], v, fns)
    else:
        H.assert_values_equal(blk.get_aggregation_result(), o["results"], fns)


# all-bitmap filter whose program ORs more than 64 bitmaps: past the wave kernel's one-bitmap-per-lane limit, so the
# normal heuristic picks the per-segment walk (pgx_roaring_program_seg)
WIDE_IN = "SELECT COUNT(*), SUM(m) FROM t WHERE y IN (%s) AND x <> 1" % ", ".join(str(3 * i + 1) for i in range(70))


@pytest.mark.parametrize("mode", ["0wave", "0", "0chunk", "0narrow", "1"])
@pytest.mark.parametrize("text", QUERIES[9:] + [WIDE_IN])
def test_bitmap_program_in_kernel_vs_separate_pass(ctx, segs, text, mode, monkeypatch):
    """All-bitmap filter sub-trees evaluated per 65536-doc chunk inside the query kernel (LEAF_RCHUNK, PGX_RCHUNK=1)
    or by the separate expansion pass (PGX_RCHUNK=0): the wave-per-chunk kernel ("0wave", the default for programs of
    at most 64 bitmaps and 3 mask slots), one workgroup per segment walking every bitmap's containers in key order
    ("0", PGX_RPROG=seg), one workgroup per (segment, chunk) with a container search ("0chunk", PGX_RPROG=chunk),
    or the stack kernel ("0narrow", PGX_RPROG=stack).  All equal the oracle, statistics included, alone and in a
    multi-segment launch whose workgroups start mid-chunk."""
    from pinot_amd import engine as E
    monkeypatch.setenv("PGX_RCHUNK", mode[0])
    monkeypatch.setenv("PGX_RPROG", {"0wave": "wave", "0": "seg", "0chunk": "chunk", "0narrow": "stack", "1": "wave"}[mode])
    inv, scan, oseg = segs
    q = pql.compile(text)
    pm = E.InstancePlanMakerImplV2(ctx)
    op = pm.make_inner_segment_plan(inv, q).run()
    blk = op.next_block()
    o = H.oracle_answer([oseg], q, literal=True)
    fns = [a["fn"] for a in q["aggregations"]]
    assert op.get_execution_statistics().as_list() == list(o["stats"])
    blk3 = pm.make_inter_segment_plan([inv, scan, inv], q).execute()
    o3 = H.oracle_answer([oseg, oseg, oseg], q, literal=True)
    if q.get("group_by"):
        m = blk.get_aggregation_group_by_result()
        m = m.as_map() if m is not None else {}
        assert set(m) == set(o["map"])
        for k, v in o["map"].items():
            H.assert_values_equal(m[k], v, fns)
        m3 = blk3.get_aggregation_group_by_result()
        m3 = m3.as_map() if m3 is not None else {}
        assert set(m3) == set(o3["map"])
        for k, v in o3["map"].items():
            H.assert_values_equal(m3[k], v, fns)
    else:
        H.assert_values_equal(blk.get_aggregation_result(), o["results"], fns)
        H.assert_values_equal(blk3.get_aggregation_result(), o3["results"], fns)
