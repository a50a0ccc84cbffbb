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


def _raw(i):
    rng = np.random.default_rng(300 + i)
    n, card = 120000 + 5000 * i, 3000
    raw = {"ga": rng.integers(0, card, size=n).astype(np.int32),
           "gb": rng.integers(0, card, size=n).astype(np.int32) * 3,
           "m": rng.integers(-5000, 5000, size=n).astype(np.int32)}
    raw["ga"][:card] = np.arange(card)  # identical dictionaries on every rank: one key space
    raw["gb"][:card] = np.arange(card) * 3
    raw["m"][:10000] = np.arange(-5000, 5000)
    return raw


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist

    from pinot_amd import engine as E
    from pinot_amd import multigpu, pql
    from tests import helpers as H
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ctx = E.Context(0)
        segs = [E.IndexSegment(ctx, H.build_pair("r%d_%d" % (rank, i), _raw(2 * i + rank))[0]) for i in range(2)]
        qq = E._Query(ctx, pql.compile(QUERY))
        r = qq.execute(segs)
        maps, total, stats = multigpu.device_sparse_merge(ctx, qq, r, segs, "cuda:0")
        from pinot_amd import native as N
        N.lib().pgx_result_release(r)
        q.put((rank, (maps, total, stats)))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def _values(maps):
    return [sorted(v[0] / v[1] if isinstance(v, tuple) else v for v in m.values()) for m in maps]


def test_two_rank_device_sparse_merge_equals_one_execution():
    import torch.multiprocessing as mp

    from pinot_amd import engine as E
    from pinot_amd import native as N
    from pinot_amd import pql
    from tests import helpers as H
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0, res
    maps, total, stats = res[0]
    assert res[1][0] is None and res[1][1] == total  # every rank learns the global group count
    # one execution over all four segments
    c = E.Context(0)
    segs = [E.IndexSegment(c, H.build_pair("all%d" % k, _raw(k))[0]) for k in range(4)]
    qq = E._Query(c, pql.compile(QUERY))
    r = qq.execute(segs)
    try:
        import ctypes as C
        ng = C.c_int64()
        N.check(N.lib().pgx_result_num_groups(r, C.byref(ng)))
        assert total == ng.value > 20000  # the trim engages
        st = (C.c_int64 * 4)()
        N.check(N.lib().pgx_result_stats(r, st))
        assert list(stats) == list(st)
        assert _values(maps) == _values(E.trimmed_maps(qq, r, segs))
    finally:
        N.lib().pgx_result_release(r)
        c.close()
