"""GPU tests of the boundary's multi-device and asynchronous entry points (include/pgx.h).

* pgx_execute_multi over two contexts (on device 0: the box has one GPU; the code path is the same as for two devices,
  with hipMemcpyPeerAsync copying within one device): segments staged on different contexts, interleaved in the
  segment list, with per-segment dictionaries (the union key space is built over ALL segments).  The merged result
  must equal one pgx_execute over the same segments on one context and the oracle's combine, for aggregation-only,
  dense group-by (dense tables reduced plane by plane), sparse group-by through the partitioned path (device-resident
  groups merged by pgx_group_merge) and through the global hash table (host merge by key).
* pgx_execute_async + pgx_result_wait: several queries in flight on one context equal their synchronous runs; an
  execution error surfaces from pgx_result_wait and from every accessor.
* pgx_result_device_groups + pgx_result_merge_groups (the per-rank step of the cross-process sparse merge): two
  executions over halves of the segments, their groups concatenated in device memory and merged, equal one execution
  over all segments, including the device trim.
"""
import ctypes as C

import numpy as np
import pytest

from pinot_amd import pql
from tests import helpers as H
from tests.test_gpu_parity import _rand_segment

pytestmark = pytest.mark.gpu

AGGS = "SELECT COUNT(*), SUM(m), MIN(m), MAX(m), AVG(m) FROM t"


@pytest.fixture(scope="module")
def ctxs():
    from pinot_amd import engine as E
    cs = [E.Context(0), E.Context(0), E.Context(0)]
    yield cs
    for c in cs:
        c.close()


@pytest.fixture(scope="module")
def diff_segs(ctxs):
    """Four segments with their own dictionaries: 0 and 2 on context A, 1 and 3 on context B; all four again on
    context C for the single-context reference."""
    from pinot_amd import engine as E
    rng = np.random.default_rng(77)
    pairs = []
    for i in range(4):
        raw = _rand_segment(rng, 9000 + 2500 * i, {"a": 3000, "b": 40, "g1": 13, "g2": 900, "m": 5000}, "d%d" % i)
        pairs.append(H.build_pair("d%d" % i, raw, inverted=("b",)))
    multi = [E.IndexSegment(ctxs[i % 2], s) for i, (s, _) in enumerate(pairs)]
    single = [E.IndexSegment(ctxs[2], s) for s, _ in pairs]
    b_vals = np.unique(np.concatenate([p[1].columns["b"].dictionary for p in pairs]))
    return multi, single, [o for _, o in pairs], {"b0": int(b_vals[3]), "b1": int(b_vals[17])}


def _decode(ctx, q, r, segs):
    from pinot_amd import engine as E
    from pinot_amd import native as N
    try:
        return E.decode_result(q, r, segs)
    finally:
        N.lib().pgx_result_release(r)


def _compare(blk_a, blk_b, fns):
    assert blk_a.stats.as_list() == blk_b.stats.as_list()
    ga, gb = blk_a.get_aggregation_group_by_result(), blk_b.get_aggregation_group_by_result()
    if ga is None:
        H.assert_values_equal(blk_a.get_aggregation_result(), blk_b.get_aggregation_result(), fns, rel=1e-12)
        return
    ma, mb = ga.as_map(), gb.as_map()
    assert set(ma) == set(mb)
    for k, v in mb.items():
        H.assert_values_equal(ma[k], v, fns, rel=1e-12)
    assert ga.storage_mode == gb.storage_mode


MULTI_QUERIES = [
    AGGS,
    AGGS + " WHERE a > 0 OR b = %(b0)s",
    AGGS + " WHERE b IN (%(b0)s, %(b1)s) GROUP BY g1",
    AGGS + " GROUP BY g1, b",
    AGGS + " WHERE a < 100000000 GROUP BY g2, a",
    "SELECT MAX(m), COUNT(*) FROM t WHERE b <> %(b1)s GROUP BY a, g1",
]


@pytest.mark.parametrize("text", MULTI_QUERIES)
@pytest.mark.parametrize("flags", [0, "NO_PARTITION"])
def test_execute_multi_equals_single_context(ctxs, diff_segs, text, flags):
    from pinot_amd import engine as E
    from pinot_amd import native as N
    multi, single, osegs, fmt = diff_segs
    q = pql.compile(text % fmt)
    fl = N.PGX_X_NO_PARTITION if flags == "NO_PARTITION" else 0
    fns = [a["fn"] for a in q["aggregations"]]
    qm = E._Query(ctxs[0], q)
    got = _decode(ctxs[0], qm, qm.execute_multi(multi, contexts=ctxs[:2], flags=fl), multi)
    qs = E._Query(ctxs[2], q)
    ref = _decode(ctxs[2], qs, qs.execute(single, flags=fl), single)
    _compare(got, ref, fns)
    o = H.oracle_answer(osegs, q)
    if q.get("group_by"):
        m = got.get_aggregation_group_by_result().as_map()
        assert set(m) == set(o["map"])
        for k, v in o["map"].items():
            H.assert_values_equal(m[k], v, fns)
    else:
        H.assert_values_equal(got.get_aggregation_result(), o["results"], fns)


def test_execute_multi_rejects_foreign_segment(ctxs, diff_segs):
    from pinot_amd import engine as E
    from pinot_amd import native as N
    multi, single, _, _ = diff_segs
    qm = E._Query(ctxs[0], pql.compile(AGGS))
    with pytest.raises(N.PgxError) as e:
        qm.execute_multi([multi[0], single[1]], contexts=ctxs[:2])
    assert e.value.status == 1


def _pairs_raw(n, card, seed):
    rng = np.random.default_rng(seed)
    raw = {"ga": rng.integers(0, card, size=n).astype(np.int32),
           "gb": rng.integers(0, card, size=n).astype(np.int32) * 3,
           "m": rng.integers(-5000, 5000, size=n).astype(np.int32)}
    raw["ga"][:card] = np.arange(card)  # every segment holds the full dictionaries: one key space everywhere (9M keys:
    # beyond the 2^22-slot dense limit, so the sparse partitioned path runs)
    raw["gb"][:card] = np.arange(card) * 3
    raw["m"][:10000] = np.arange(-5000, 5000)  # one metric dictionary in every segment (one value base)
    return raw


@pytest.fixture(scope="module")
def pair_segs(ctxs):
    from pinot_amd import engine as E
    built = [H.build_pair("pq%d" % i, _pairs_raw(150000 + 10000 * i, 3000, 90 + i))[0] for i in range(4)]
    multi = [E.IndexSegment(ctxs[i % 2], s) for i, s in enumerate(built)]
    single = [E.IndexSegment(ctxs[2], s) for s in built]
    return multi, single


PAIRS_Q = "SELECT COUNT(*), SUM(m), MIN(m), MAX(m), AVG(m) FROM t WHERE m > -4000 GROUP BY ga, gb"


def _trimmed_values(q, r, segs):
    from pinot_amd import engine as E
    return [sorted(v[0] / v[1] if isinstance(v, tuple) else v for v in m.values())  # AVG compares by sum / count
            for m in E.trimmed_maps(q, r, segs)]


def test_execute_multi_device_resident_merge(ctxs, pair_segs):
    """Sparse keys through the partitioned path on both contexts: the device-resident groups merge on the device,
    and the device trim of the merged result keeps the same values as the single-context trim."""
    from pinot_amd import engine as E
    from pinot_amd import native as N
    multi, single = pair_segs
    q = pql.compile(PAIRS_Q)
    fns = [a["fn"] for a in q["aggregations"]]
    qm, qs = E._Query(ctxs[0], q), E._Query(ctxs[2], q)
    rm, rs = qm.execute_multi(multi, contexts=ctxs[:2]), qs.execute(single)
    try:
        n = C.c_int64()
        N.check(N.lib().pgx_result_device_groups(rm, C.byref(n), None))  # merged groups stay on the device
        assert n.value > 20 * 1000  # the trim engages
        assert _trimmed_values(qm, rm, multi) == _trimmed_values(qs, rs, single)
        _compare(E.decode_result(qm, rm, multi), E.decode_result(qs, rs, single), fns)
    finally:
        N.lib().pgx_result_release(rm)
        N.lib().pgx_result_release(rs)


def test_result_merge_groups_of_two_executions(ctxs, pair_segs):
    """The per-rank step of the cross-GPU sparse merge: the group records (key, count, sum, min, max) of two results
    side by side in one device buffer, merged (pgx_result_merge_groups) == one execution over all segments."""
    from pinot_amd import engine as E
    from pinot_amd import native as N
    L = N.lib()
    _, single = pair_segs
    ctx = ctxs[2]
    q = pql.compile(PAIRS_Q)
    fns = [a["fn"] for a in q["aggregations"]]
    qs = E._Query(ctx, q)
    halves = [single[:2], single[2:]]
    rs = [qs.execute(h) for h in halves]
    buf = C.c_void_p()
    try:
        ns = []
        for r in rs:
            n = C.c_int64()
            N.check(L.pgx_result_device_groups(r, C.byref(n), None))
            ns.append(n.value)
        total = sum(ns)
        N.check(L.pgx_device_alloc(ctx.handle, total * 40, C.byref(buf)))
        off = 0
        for r, n in zip(rs, ns):
            N.check(L.pgx_result_device_groups(r, C.byref(C.c_int64()), C.c_void_p(buf.value + off * 40)))
            off += n
        recs = np.zeros((total, 5), dtype=np.uint64)
        N.check(L.pgx_copy_to_host(ctx.handle, recs.ctypes.data, buf, total * 40))
        assert recs[:, 1].sum() == sum(r for r in [_count(L, x) for x in rs])  # doc counts travel in word 1
        st = (C.c_int64 * 4)()
        for r in rs:
            s4 = (C.c_int64 * 4)()
            N.check(L.pgx_result_stats(r, s4))
            for i in range(4):
                st[i] += s4[i]
        merged = C.c_void_p()
        N.check(L.pgx_result_merge_groups(ctx.handle, rs[0], buf, total, st, C.byref(merged)))
        whole = qs.execute(single)
        try:
            assert _trimmed_values(qs, merged, halves[0]) == _trimmed_values(qs, whole, single)
            _compare(E.decode_result(qs, merged, halves[0]), E.decode_result(qs, whole, single), fns)
        finally:
            L.pgx_result_release(merged)
            L.pgx_result_release(whole)
    finally:
        for r in rs:
            L.pgx_result_release(r)
        if buf.value:
            L.pgx_device_free(ctx.handle, buf)


def _count(L, r):
    st = (C.c_int64 * 4)()
    from pinot_amd import native as N
    N.check(L.pgx_result_stats(r, st))
    return st[0]


def test_execute_async_matches_sync(ctxs, diff_segs, pair_segs):
    from pinot_amd import engine as E
    from pinot_amd import native as N
    L = N.lib()
    _, single, _, fmt = diff_segs
    _, psingle = pair_segs
    ctx = ctxs[2]
    cases = [(pql.compile(t % fmt), single) for t in MULTI_QUERIES] + [(pql.compile(PAIRS_Q), psingle)]
    qs = [E._Query(ctx, q) for q, _ in cases]
    pending = [qq.execute_async(segs) for qq, (_, segs) in zip(qs, cases)]  # all in flight at once
    for qq, (q, segs), r in zip(qs, cases, pending):
        assert L.pgx_result_wait(r, -1) == 0
        got = _decode(ctx, qq, r, segs)
        ref = _decode(ctx, qq, qq.execute(segs), segs)
        _compare(got, ref, [a["fn"] for a in q["aggregations"]])


def test_execute_async_error_surfaces(ctxs):
    from pinot_amd import engine as E
    from pinot_amd import native as N
    L = N.lib()
    ctx = ctxs[2]
    s, _ = H.build_pair("str", {"x": np.array(["u", "v", "w"] * 100), "m": np.arange(300, dtype=np.int32)})
    seg = E.IndexSegment(ctx, s)
    qq = E._Query(ctx, pql.compile("SELECT SUM(x) FROM t"))  # numeric aggregation on a STRING column
    r = qq.execute_async([seg])
    try:
        assert L.pgx_result_wait(r, -1) == N.PGX_ERR_UNSUPPORTED
        assert b"STRING" in L.pgx_last_error()
        st = (C.c_int64 * 4)()
        assert L.pgx_result_stats(r, st) == N.PGX_ERR_UNSUPPORTED
    finally:
        L.pgx_result_release(r)
