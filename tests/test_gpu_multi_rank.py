"""The cross-process sparse merge of bench.py's N>1 path (multigpu.device_sparse_merge) end to end on the GPU box: two
ranks (processes sharing cuda:0 over gloo -- RCCL needs one device per rank) each execute the query over their own
segments, exchange their device-resident group records by key hash (all_to_all_single), merge them on the device
(pgx_result_merge_groups), trim on the device and send the kept groups to rank 0.  Rank 0's result must equal ONE
execution over all segments: the same global group count, the same ExecutionStatistics, and per function the same
multiset of kept values (trimToSize ties at the threshold are arbitrary in the reference too)."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

QUERY = "SELECT COUNT(*), SUM(m), MIN(m), MAX(m), AVG(m) FROM t WHERE m > -4000 GROUP BY ga, gb"
# VERDICT r5 missing #1: results the device record exchange refused before -- two value columns (c3m2's shape: the
# planes count + 3 per column) and a DOUBLE metric with its own dictionary per segment (c3f's shape: f64 sum planes)
SHAPES = {
    "one_int": (QUERY, None),
    "two_int_columns": ("SELECT SUM(m), SUM(m2), MAX(m), COUNT(*) FROM t WHERE m > -4000 GROUP BY ga, gb", None),
    "double_metric": ("SELECT SUM(d), MIN(d), MAX(d), AVG(d) FROM t WHERE m > -4000 GROUP BY ga, gb", {"d": "DOUBLE"}),
}


def _raw(i):
    rng = np.random.default_rng(300 + i)
    n, card = 120000 + 5000 * i, 3000
    raw = {"ga": rng.integers(0, card, size=n).astype(np.int32),
           "gb": rng.integers(0, card, size=n).astype(np.int32) * 3,
           "m": rng.integers(-5000, 5000, size=n).astype(np.int32),
           "m2": rng.integers(0, 4096, size=n).astype(np.int32),
           "d": rng.uniform(-1000.0, 1000.0, size=n)}  # non-dyadic: a dictionary of its own in every segment
    raw["ga"][:card] = np.arange(card)  # identical dictionaries on every rank: one key space
    raw["gb"][:card] = np.arange(card) * 3
    raw["m"][:10000] = np.arange(-5000, 5000)
    raw["m2"][:4096] = np.arange(4096)
    return raw


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, shape="one_int"):
    import ctypes as C
    from datetime import timedelta

    import torch.distributed as dist

    from pinot_amd import engine as E
    from pinot_amd import multigpu, pql
    from pinot_amd import native as N
    from tests import helpers as H
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=timedelta(seconds=60))
    try:
        text, types = SHAPES[shape]
        ctx = E.Context(0)
        segs = [E.IndexSegment(ctx, H.build_pair("r%d_%d" % (rank, i), _raw(2 * i + rank), types=types)[0])
                for i in range(2)]
        qq = E._Query(ctx, pql.compile(text))
        r = qq.execute(segs)
        n = C.c_int64()
        w = C.c_int32()
        assert N.lib().pgx_result_device_groups(r, C.byref(n), None) == 0  # the device record exchange is taken
        N.check(N.lib().pgx_result_record_words(r, C.byref(w)))
        maps, total, stats = multigpu.device_sparse_merge(ctx, qq, r, segs, "cuda:0")
        N.lib().pgx_result_release(r)
        q.put((rank, (maps, total, stats, w.value)))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def _values(maps):
    return [sorted(v[0] / v[1] if isinstance(v, tuple) else v for v in m.values()) for m in maps]


def _run_ranks(target, world, *args):
    """Spawn `world` rank processes; each puts (rank, answer) on the queue.  Bounded waits: a hang fails the test."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = dict(q.get(timeout=150) for _ in procs)
        for p in procs:
            p.join(timeout=30)
            assert p.exitcode == 0, res
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
                p.join(timeout=10)
    return res


@pytest.mark.parametrize("shape", list(SHAPES))
def test_two_rank_device_sparse_merge_equals_one_execution(shape):
    import ctypes as C

    from oracle import pinot_oracle as O  # noqa: F401  (H.oracle_answer)
    from pinot_amd import engine as E
    from pinot_amd import native as N
    from pinot_amd import pql
    from tests import helpers as H
    res = _run_ranks(_worker, 2, shape)
    maps, total, stats, words = res[0]
    assert res[1][0] is None and res[1][1] == total  # every rank learns the global group count
    text, types = SHAPES[shape]
    req = pql.compile(text)
    assert words == 1 + 1 + 3 * len({a["column"] for a in req["aggregations"] if a["column"] != "*"})
    # one execution over all four segments, and the oracle's combine + trimToSize over them
    c = E.Context(0)
    pairs = [H.build_pair("all%d" % k, _raw(k), types=types) for k in range(4)]
    segs = [E.IndexSegment(c, p[0]) for p in pairs]
    qq = E._Query(c, req)
    r = qq.execute(segs)
    try:
        ng = C.c_int64()
        N.check(N.lib().pgx_result_num_groups(r, C.byref(ng)))
        assert total == ng.value > 20000  # the trim engages
        st = (C.c_int64 * 4)()
        N.check(N.lib().pgx_result_stats(r, st))
        assert list(stats) == list(st)
        o = H.oracle_answer([p[1] for p in pairs], req, literal=True)
        assert total == len(o["map"]) and list(stats) == list(o["stats"])
        want = [sorted(v[0] / v[1] if isinstance(v, tuple) else v for v in m.values()) for m in o["trimmed"]]
        if shape == "double_metric":  # f64 sums merged in arbitrary order: north_star's 1e-9 relative
            for g, w in zip(_values(maps), want):
                np.testing.assert_allclose(g, w, rtol=1e-9)
        else:
            assert _values(maps) == _values(E.trimmed_maps(qq, r, segs)) == want
    finally:
        N.lib().pgx_result_release(r)
        c.close()


# ------------------------------------------------------------------------------------------------
# Ranks with DIFFERENT dictionaries (VERDICT r2 missing #4): multigpu.union_key_domains gives every rank the same key
# space (pgx_query_set_key_domain over the union of all ranks' dictionary values), so the dense tables all-reduce by
# slot and the sparse groups merge on the device by packed key -- no value-keyed host gather.
# ------------------------------------------------------------------------------------------------
DENSE_QUERY = "SELECT COUNT(*), SUM(m), MIN(m), MAX(m), AVG(m) FROM t WHERE m > -4500 GROUP BY ga"


def _raw_differ(rank, i):
    """Rank 0's ga values are 0..599, rank 1's 300..899 (each misses values the other holds); gb likewise shifted."""
    rng = np.random.default_rng(500 + 10 * rank + i)
    n = 90000 + 3000 * i
    ga = rng.integers(0, 600, size=n).astype(np.int32) + 300 * rank
    gb = (rng.integers(0, 20000, size=n).astype(np.int32) + 8000 * rank) * 7  # 900 x 28000 keys: sparse
    m = rng.integers(-5000, 5000, size=n).astype(np.int32)
    m[:10000] = np.arange(-5000, 5000)  # one value dictionary everywhere: the partitioned (device-resident) path
    return {"ga": ga, "gb": gb, "m": m}


def _differ_worker(rank, world, port, q):
    import ctypes as C
    from datetime import timedelta

    import torch
    import torch.distributed as dist

    from pinot_amd import engine as E
    from pinot_amd import multigpu, pql
    from pinot_amd import native as N
    from tests import helpers as H
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=timedelta(seconds=60))
    try:
        L = N.lib()
        ctx = E.Context(0)
        segs = [E.IndexSegment(ctx, H.build_pair("d%d_%d" % (rank, i), _raw_differ(rank, i))[0]) for i in range(2)]
        arr = (C.c_void_p * len(segs))(*[s.handle.value for s in segs])
        out = {}
        # dense: identical slot layout after the union, planes all-reduced, decoded from the merged table
        qd = E._Query(ctx, pql.compile(DENSE_QUERY))
        multigpu.union_key_domains(qd, segs)
        slots = C.c_int64()
        N.check(L.pgx_query_dense_slots(qd.handle, arr, len(segs), C.byref(slots)))
        ops = []
        for p in range(1 + len(qd.fns)):
            op = C.c_int32()
            N.check(L.pgx_query_dense_plane_op(qd.handle, arr, len(segs), p, C.byref(op)))
            ops.append(op.value)
        t = torch.zeros(len(ops) * slots.value, dtype=torch.int64, device="cuda:0")
        r = qd.execute(segs, flags=N.PGX_X_KEEP_DENSE_ON_DEVICE, dense_out=C.c_void_p(t.data_ptr()),
                       dense_out_bytes=t.numel() * 8)
        st = (C.c_int64 * 4)()
        N.check(L.pgx_result_stats(r, st))
        L.pgx_result_release(r)
        torch.cuda.synchronize()
        multigpu.merge_dense_planes(t, ops)
        stt = torch.tensor(list(st), dtype=torch.int64)
        dist.all_reduce(stt)
        s4 = (C.c_int64 * 4)(*stt.tolist())
        rd = C.c_void_p()
        N.check(L.pgx_result_from_dense(ctx.handle, qd.handle, arr, len(segs), C.c_void_p(t.data_ptr()), s4,
                                        C.byref(rd)))
        blk = E.decode_result(qd, rd, segs)
        L.pgx_result_release(rd)
        out["dense"] = (slots.value, blk.get_aggregation_group_by_result().as_map(), list(s4))
        # sparse: the device path must be taken (device-resident groups on every rank)
        qs = E._Query(ctx, pql.compile(QUERY))
        multigpu.union_key_domains(qs, segs)
        r = qs.execute(segs)
        n = C.c_int64()
        assert L.pgx_result_device_groups(r, C.byref(n), None) == 0
        maps, total, stats = multigpu.device_sparse_merge(ctx, qs, r, segs, "cuda:0")
        L.pgx_result_release(r)
        out["sparse"] = (maps, total, stats)
        q.put((rank, out))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def test_two_ranks_with_different_dictionaries_merge_on_device():
    import ctypes as C

    from pinot_amd import engine as E
    from pinot_amd import native as N
    from pinot_amd import pql
    from tests import helpers as H
    res = _run_ranks(_differ_worker, 2)
    c = E.Context(0)
    segs = [E.IndexSegment(c, H.build_pair("dall%d" % k, _raw_differ(k // 2, k % 2))[0]) for k in range(4)]
    try:
        # dense: the merged table decodes to exactly one execution's groups over all four segments
        slots, dmap, dstats = res[0]["dense"]
        assert slots == res[1]["dense"][0] == 900  # union of 0..599 and 300..899
        qd = E._Query(c, pql.compile(DENSE_QUERY))
        r = qd.execute(segs)
        blk = E.decode_result(qd, r, segs)
        N.lib().pgx_result_release(r)
        exp = blk.get_aggregation_group_by_result().as_map()
        assert set(dmap) == set(exp) and len(exp) == 900
        for k, v in exp.items():
            got = dmap[k]
            assert got[0] == v[0] and got[2] == v[2] and got[3] == v[3]  # COUNT, MIN, MAX exact
            assert got[1] == v[1] and got[4] == v[4]  # integer SUM below 2^53: exact in any order
        assert dstats == blk.stats.as_list()
        # sparse: global group count, statistics and the kept values of one execution
        maps, total, stats = res[0]["sparse"]
        assert res[1]["sparse"][0] is None and res[1]["sparse"][1] == total
        qs = E._Query(c, pql.compile(QUERY))
        r = qs.execute(segs)
        ng = C.c_int64()
        N.check(N.lib().pgx_result_num_groups(r, C.byref(ng)))
        assert total == ng.value > 20000
        st = (C.c_int64 * 4)()
        N.check(N.lib().pgx_result_stats(r, st))
        assert list(stats) == list(st)
        assert _values(maps) == _values(E.trimmed_maps(qs, r, segs))
        N.lib().pgx_result_release(r)
    finally:
        c.close()
