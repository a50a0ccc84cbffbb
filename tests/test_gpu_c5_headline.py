"""Parity of the execution the headline (C5) bench number comes from (BASELINE configs[4]; SURVEY 8a rows a-7, a-9,
a-10, a-15..a-17, a-19, a-20).

bench.py runs C5 with three queries in flight (`pgx_execute_async` on three HIP streams), each carrying
PGX_X_THROUGHPUT (every segment planned into one launch per kernel: a different plan than the batched one once there
are >= 2 x 512 segments, pgx_host.cpp run_batched), with the packed count + sum dense update on (default).  These
tests run exactly that:

* `test_c5_throughput_inflight_vs_oracle`: 1,152 C5 segments (small rows, so the oracle stays quick; the plan change
  depends on the segment count, not on rows), three executions in flight on three streams with PGX_X_THROUGHPUT, and
  a batched execution; each result (every group's sum, plus all four ExecutionStatistics) equals the oracle's combine
  over all segments: the vectorised filter `(f1 IN ... OR f2 = 7) AND f3 <> 3` and per-gk sums over the
  regenerated (bit-identical) dictIds, MCombineGroupByOperator.java:139-233.
* `test_c5_full_size_shard_linearity`: the bench's own 4,096 x 2M-row result equals the merge of 8 disjoint shard
  results (combine linearity: every function is a sum or count here), and the first shard (512 segments) equals the
  oracle.
"""
import concurrent.futures as CF
import ctypes as C

import numpy as np
import pytest

from oracle import c_oracle
from pinot_amd import pql, synth
from tests import helpers as H

pytestmark = pytest.mark.gpu

WL = synth.WORKLOADS["c5"]
NPROJ = 2  # numEntriesScannedPostFilter = docs x projection columns (gk, m)


@pytest.fixture(scope="module")
def ctx():
    from pinot_amd import engine as E
    c = E.Context(0)
    yield c
    c.close()


def _oracle(seg_ids, rows, q):
    """Per-gk (sum, count) of the C5 query over the given segments: dictIds regenerated on the host by the C twin's
    generator (pgo_synth_ids: the ids pgx_synth_column packs on the device, tests/test_gpu_fullsize.py pins the two
    bit-identical), the predicate evaluated vectorised (IN as a dictId lookup table)."""
    f1 = np.zeros(1000, dtype=bool)
    f1[[int(v) for v in q["filter"]["children"][0]["children"][0]["values"]]] = True
    mvals = synth.make_dictionary("metric", 65536).astype(np.float64)

    def one(s):
        ids = {c.name: c_oracle.synth_ids(synth.column_seed(WL.seed, s, ci), rows, c.card)
               for ci, c in enumerate(WL.columns)}
        sel = (f1[ids["f1"]] | (ids["f2"] == 7)) & (ids["f3"] != 3)
        return (np.bincount(ids["gk"][sel], weights=mvals[ids["m"][sel]], minlength=1000),
                np.bincount(ids["gk"][sel], minlength=1000))

    sums = np.zeros(1000)
    counts = np.zeros(1000, dtype=np.int64)
    with CF.ThreadPoolExecutor(16) as ex:
        for sm, ct in ex.map(one, seg_ids):
            sums += sm
            counts += ct
    return sums, counts


def _check(got_map, st, sums, counts, nseg, rows):
    exp = {str(g): [float(sums[g])] for g in range(1000) if counts[g]}
    assert set(got_map) == set(exp)
    for k, v in exp.items():
        H.assert_values_equal(got_map[k], v, ["sum"])
    docs = int(counts.sum())
    assert list(st) == [docs, 0, docs * NPROJ, nseg * rows]


def _hip_streams(k):
    """k HIP streams of this process (the HIP runtime libpgx uses), as handles for pgx_exec_opts.stream."""
    hip = C.CDLL("libamdhip64.so")
    out = []
    for _ in range(k):
        s = C.c_void_p()
        assert hip.hipStreamCreate(C.byref(s)) == 0
        out.append(s)
    return hip, out


def test_c5_throughput_inflight_vs_oracle(ctx):
    from pinot_amd import engine as E
    from pinot_amd import native as N
    L = N.lib()
    nseg, rows = 1152, 65536 + 4321  # >= 2 x 512 segments; two roaring chunks per segment, the second partial
    seg_ids = list(range(nseg))
    data = synth.DeviceSegments(ctx, WL, seg_ids, rows=rows)
    try:
        req = pql.compile(WL.query)
        q = E._Query(ctx, req)
        segs = data.segments
        seg_arr = (C.c_void_p * nseg)(*[s.handle.value for s in segs])
        hip, streams = _hip_streams(3)
        pending = []
        for i in range(3):  # as bench.py submit(): bind, then execute asynchronously on stream i, three in flight
            binds, owner = q.bindings(segs, seg_arr)
            opts = N.ExecOpts(streams[i].value, None, 0, N.PGX_X_THROUGHPUT)
            r = C.c_void_p()
            N.check(L.pgx_execute_async(ctx.handle, q.handle, seg_arr, nseg, binds, C.byref(opts), C.byref(r)))
            pending.append((r, owner))
        r_batched = q.execute(segs)  # the batched (latency) plan of the same query, beside them
        sums, counts = _oracle(seg_ids, rows, req)
        for r, _owner in pending + [(r_batched, None)]:
            N.check(L.pgx_result_wait(r, -1))
            blk = E.decode_result(q, r, segs)
            _check(blk.get_aggregation_group_by_result().as_map(), blk.stats.as_list(), sums, counts, nseg, rows)
            L.pgx_result_release(r)
        q.close()
        for s in streams:
            hip.hipStreamDestroy(s)
    finally:
        data.free()


def test_c5_full_size_shard_linearity(ctx):
    from pinot_amd import engine as E
    from pinot_amd import multigpu
    from pinot_amd import native as N
    L = N.lib()
    rows = WL.rows
    data = synth.DeviceSegments(ctx, WL, list(range(WL.segments)), rows=rows)  # the bench's 4,096 x 2M rows
    try:
        req = pql.compile(WL.query)
        q = E._Query(ctx, req)
        segs = data.segments
        full = q.execute(segs, flags=N.PGX_X_THROUGHPUT)
        fmap = E.decode_result(q, full, segs).get_aggregation_group_by_result().as_map()
        fst = E.decode_result(q, full, segs).stats.as_list()
        L.pgx_result_release(full)
        acc = {}
        ast = np.zeros(4, dtype=np.int64)
        shard_maps = []
        for rank in range(8):  # bench.py's own 8-GPU shards (multigpu.shard, strong scaling)
            ids = multigpu.shard(WL.segments, 8, rank, "strong")
            sub = [segs[i] for i in ids]
            r = q.execute(sub, flags=N.PGX_X_THROUGHPUT)
            blk = E.decode_result(q, r, sub)
            m = blk.get_aggregation_group_by_result().as_map()
            shard_maps.append((ids, m, blk.stats.as_list()))
            for k, v in m.items():
                acc[k] = acc.get(k, 0.0) + v[0]
            ast += np.array(blk.stats.as_list(), dtype=np.int64)
            L.pgx_result_release(r)
        assert set(acc) == set(fmap)
        for k, v in fmap.items():
            assert v[0] == acc[k], k  # integer sums below 2^53: exact in any order
        assert list(ast) == fst
        for ids, m, st in shard_maps[:1]:  # one shard (512 segments) against the oracle; the rest by linearity
            sums, counts = _oracle(ids, rows, req)
            _check(m, st, sums, counts, len(ids), rows)
        q.close()
    finally:
        data.free()


def test_plan_cache_replays_vs_oracle(ctx, monkeypatch, capfd):
    """The plan cache (pgx_host.cpp run_query): a second execution of the same query over the same segments replays the
    first one's plan (the host-profile line carries the "cached" mark) with the same result, statistics included; the
    throughput flag does not change the key; a different segment list (a subset) plans afresh.  The replay without the
    throughput flag launches the bitmap programs and the query kernel in two halves (the second half's programs on the
    side stream beside the first half's query kernel).  Oracle as above."""
    from pinot_amd import engine as E
    from pinot_amd import native as N
    monkeypatch.setenv("PGX_DEBUG", "host_profile")
    nseg, rows = 96, 65536 + 999  # >= 64 segments: a replay without the throughput flag runs in two halves
    seg_ids = list(range(nseg))
    data = synth.DeviceSegments(ctx, WL, seg_ids, rows=rows)
    try:
        req = pql.compile(WL.query)
        q = E._Query(ctx, req)
        segs = data.segments
        sums, counts = _oracle(seg_ids, rows, req)
        for k, flags in enumerate([0, 0, N.PGX_X_THROUGHPUT]):
            r = q.execute(segs, flags=flags)
            blk = E.decode_result(q, r, segs)
            _check(blk.get_aggregation_group_by_result().as_map(), blk.stats.as_list(), sums, counts, nseg, rows)
            N.lib().pgx_result_release(r)
            lines = [x for x in capfd.readouterr().err.splitlines() if x.startswith("[pgx host us]")]
            assert lines and (" cached=" in lines[-1]) == (k > 0), lines
        sub = segs[:20]
        r = q.execute(sub)
        blk = E.decode_result(q, r, sub)
        s2, c2 = _oracle(seg_ids[:20], rows, req)
        _check(blk.get_aggregation_group_by_result().as_map(), blk.stats.as_list(), s2, c2, 20, rows)
        N.lib().pgx_result_release(r)
        lines = [x for x in capfd.readouterr().err.splitlines() if x.startswith("[pgx host us]")]
        assert lines and " cached=" not in lines[-1], lines
        q.close()
    finally:
        data.free()


def test_plan_cache_batched_list_promotes(ctx, monkeypatch, capfd):
    """A list long enough to be planned in batches (>= 2 x 512 segments, flags 0): the first execution runs batched,
    the second plans the whole list at once and keeps the plan, the third replays it (host-profile marks: "b.dicts"
    for batched, "cached" for a replay).  Every result equals the oracle's."""
    from pinot_amd import engine as E
    from pinot_amd import native as N
    monkeypatch.setenv("PGX_DEBUG", "host_profile")
    nseg, rows = 1100, 4096 + 17
    seg_ids = list(range(nseg))
    data = synth.DeviceSegments(ctx, WL, seg_ids, rows=rows)
    try:
        req = pql.compile(WL.query)
        q = E._Query(ctx, req)
        segs = data.segments
        sums, counts = _oracle(seg_ids, rows, req)
        marks = []
        for _ in range(3):
            r = q.execute(segs)
            blk = E.decode_result(q, r, segs)
            _check(blk.get_aggregation_group_by_result().as_map(), blk.stats.as_list(), sums, counts, nseg, rows)
            N.lib().pgx_result_release(r)
            lines = [x for x in capfd.readouterr().err.splitlines() if x.startswith("[pgx host us]")]
            assert lines, "no host profile line"
            marks.append((" b.dicts=" in lines[-1], " cached=" in lines[-1]))
        assert marks == [(True, False), (False, False), (False, True)], marks
        q.close()
    finally:
        data.free()
