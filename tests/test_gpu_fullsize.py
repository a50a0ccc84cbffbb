"""Full-size checks (BASELINE.json sizes) through size-independent properties and oracle spot checks.

* the device synthetic generator is bit-identical to the oracle's C generator (first 1M rows of a 125M-row column);
* C2 (1B rows, 8 x 125M): the GPU result of every segment equals the sum of per-segment GPU results (combine
  linearity) and two whole segments are recomputed by the oracle's C twin (exact COUNT and integer SUM);
* filter complement: count(dA in [64,191]) + count(dA outside) == total rows.
"""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def c2():
    from pinot_amd import engine as E
    from pinot_amd import synth
    ctx = E.Context(0)
    data = synth.DeviceSegments(ctx, synth.WORKLOADS["c2"], list(range(8)))
    yield ctx, data
    data.free()
    ctx.close()


def _query(ctx, segs, text):
    from pinot_amd import engine as E
    from pinot_amd import pql
    return E.InstancePlanMakerImplV2(ctx).make_inter_segment_plan(segs, pql.compile(text)).execute()


def test_synth_matches_oracle_generator(c2):
    from oracle import c_oracle
    from pinot_amd import native as N
    from pinot_amd import synth
    ctx, data = c2
    wl = data.wl
    n = 1 << 20
    for ci, c in enumerate(wl.columns):
        ref = c_oracle.synth_fwd(synth.column_seed(wl.seed, 0, ci), n, c.bits, c.card)[: n * c.bits // 8]
        dev = np.zeros(n * c.bits // 8, dtype=np.uint8)
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")
        ptr = data.buffers[ci].value
        assert hip.hipMemcpy(ctypes.c_void_p(dev.ctypes.data), ctypes.c_void_p(ptr), ctypes.c_size_t(len(dev)), 2) == 0
        assert np.array_equal(dev, ref), c.name


def test_c2_full_size_linearity_and_spot_checks(c2):
    from oracle import c_oracle
    from pinot_amd import synth
    ctx, data = c2
    wl = data.wl
    whole = _query(ctx, data.segments, wl.query).get_aggregation_result()
    per = [_query(ctx, [s], wl.query).get_aggregation_result() for s in data.segments]
    assert whole[0] == sum(p[0] for p in per)
    assert whole[1] == sum(p[1] for p in per)
    comp = _query(ctx, data.segments, "SELECT COUNT(*) FROM T WHERE dA NOT IN (%s)" %
                  ",".join(str(v) for v in range(64, 192))).get_aggregation_result()
    assert whole[0] + comp[0] == wl.rows * wl.segments
    # the oracle's C twin on whole 125M-row segments
    dicts = {c.name: synth.make_dictionary(c.dict_kind, c.card).astype(np.float64) for c in wl.columns}
    for s in (0, 7):
        cols = {c.name: (c_oracle.synth_fwd(synth.column_seed(wl.seed, s, ci), wl.rows, c.bits, c.card), c.bits,
                         dicts[c.name], c.card) for ci, c in enumerate(wl.columns)}
        o = c_oracle.run([c_oracle.Segment(wl.rows, cols)], filter_col="dA", lo=64, hi=191, metric="m")[0]
        assert per[s][0] == o["count"]
        assert per[s][1] == o["sum"]
