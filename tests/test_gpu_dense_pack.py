"""GPU parity of the packed dense group-by update (count and value offset in ONE 64-bit LDS add, flushed per segment
as count and offset sum + count x that segment's vbase; pgx_jit.cpp `pack`, whenever the fields fit).  Semantics: DefaultGroupByExecutor.aggregateColumn -> SumAggregationFunction.aggregateGroupBySV /
AvgAggregationFunction.aggregateGroupBySV.

Cases the default C5 plan does not reach:
* negative values (vbase < 0: the flush adds count x vbase in wrapping u64 arithmetic),
* the field boundary: the host packs only when bits(rows + 1) + bits(rows x (range + 1)) <= 64, so with a 2^32 - 1 value
  range a 60,000-row segment packs and a 70,000-row one falls back to two adds.
Every answer is compared with the CPU oracle, bit-exactly (all sums are integers below 2^53)."""
import glob
import os

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


def _raw(n, seed):
    rng = np.random.default_rng(seed)
    # 30,000 distinct values over the whole INT range: an IMG_U32 image (card x 4 B <= 144 KiB), range 2^32 - 1
    dom = np.unique(rng.integers(-(1 << 31), (1 << 31) - 1, 30000, dtype=np.int64))
    dom[0], dom[-1] = -(1 << 31), (1 << 31) - 1
    m = dom[rng.integers(0, len(dom), n)]
    m[0], m[1] = dom[0], dom[-1]  # both extremes present: the segment's value range is exactly 2^32 - 1
    return {"d": rng.integers(0, 200, n).astype(np.int32),
            "g": rng.integers(0, 17, n).astype(np.int32),
            "m": m.astype(np.int32)}


@pytest.fixture(scope="module")
def segs(ctx):
    from pinot_amd import engine as E
    out = {}
    for n, seed in ((60000, 1), (70000, 2)):
        seg, oseg = H.build_pair("pk%d" % n, _raw(n, seed))
        out[n] = (E.IndexSegment(ctx, seg), oseg)
    return out


QUERIES = [
    "SELECT SUM(m) FROM t GROUP BY g",
    "SELECT AVG(m) FROM t WHERE d < 100 GROUP BY g",
    "SELECT SUM(m) FROM t WHERE d BETWEEN 20 AND 29 GROUP BY g",
]


def _pack_bits(rows, vrange):
    cb = int(rows + 1).bit_length()
    sb = int(rows * (vrange + 1)).bit_length()
    return cb + sb


@pytest.mark.parametrize("variant", ["pack"])
@pytest.mark.parametrize("rows", [60000, 70000])
@pytest.mark.parametrize("text", QUERIES)
def test_dense_pack_matches_oracle(ctx, segs, text, rows, variant, monkeypatch, tmp_path):
    from pinot_amd import engine as E
    one = tmp_path / "one"
    one.mkdir()
    monkeypatch.setenv("PGX_JIT_DUMP", str(one))
    seg, oseg = segs[rows]
    q = pql.compile(text)
    pm = E.InstancePlanMakerImplV2(ctx)
    op = pm.make_inner_segment_plan(seg, q).run()
    m = op.next_block().get_aggregation_group_by_result().as_map()
    o = H.oracle_answer([oseg], q, literal=True)
    fns = [a["fn"] for a in q["aggregations"]]
    assert op.get_execution_statistics().as_list() == list(o["stats"])
    assert set(m) == set(o["map"])
    for k, v in o["map"].items():
        H.assert_values_equal(m[k], v, fns)
    srcs = [open(f).read() for f in glob.glob(os.path.join(str(one), "*.hip"))]
    # both segments: one launch whose members differ in size (the pack decision covers the largest member)
    monkeypatch.delenv("PGX_JIT_DUMP")
    blk = pm.make_inter_segment_plan([segs[60000][0], segs[70000][0]], q).execute()
    o2 = H.oracle_answer([segs[60000][1], segs[70000][1]], q, literal=True)
    m2 = blk.get_aggregation_group_by_result().as_map()
    assert set(m2) == set(o2["map"])
    for k, v in o2["map"].items():
        H.assert_values_equal(m2[k], v, fns)
    # the packed form is generated exactly when the fields fit (checked when this test compiled the one-segment kernel
    # itself: a kernel compiled earlier in the process is not dumped again)
    fits = _pack_bits(rows, (1 << 32) - 1) <= 64
    assert fits == (rows == 60000)
    if variant == "pack" and srcs:
        assert any("atomicAdd(&tab[key], (1ull << " in x for x in srcs) == fits
