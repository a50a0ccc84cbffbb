"""World-size-2 gloo tests (CPU) of the multi-GPU layer (pinot_amd/multigpu.py): segment sharding and the
cross-rank merge of partials, checked against a single-process merge of the same rows.

The per-rank partials are built here in the library's own plane encodings (pgx.h pgx_query_dense_plane_op) from raw
rows, exactly as the GPU would leave them in HBM; the GPU side of the same path runs in bench.py --gpus N."""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from pinot_amd import multigpu  # noqa: E402

SIGN = np.uint64(1 << 63)


def _ord_i64(x):
    return (x.astype(np.int64).view(np.uint64) ^ SIGN).view(np.int64)


def _rows(seed, n, card):
    rng = np.random.default_rng(seed)
    return rng.integers(0, card, n), rng.integers(-(1 << 20), 1 << 20, n), rng.random(n) * 1e6


def dense_table(keys, iv, fv, slots):
    """planes: 0 count (i64 add) | sum(iv) i64 add | min(iv) ord | max(iv) ord | sum(fv) f64 add"""
    t = np.zeros((5, slots), dtype=np.int64)
    t[2] = -1  # ~0: MIN identity
    np.add.at(t[0], keys, 1)
    np.add.at(t[1], keys, iv)
    mn = np.full(slots, np.iinfo(np.int64).max)
    np.minimum.at(mn, keys, iv)
    mx = np.full(slots, np.iinfo(np.int64).min)
    np.maximum.at(mx, keys, iv)
    has = t[0] > 0
    t[2][has] = _ord_i64(mn[has])
    t[3][has] = _ord_i64(mx[has])
    f = np.zeros(slots)
    np.add.at(f, keys, fv)
    t[4] = f.view(np.int64)
    return t


OPS = [multigpu.PLANE_ADD_I64, multigpu.PLANE_ADD_I64, multigpu.PLANE_MIN_ORD, multigpu.PLANE_MAX_ORD,
       multigpu.PLANE_ADD_F64]
NSEG, ROWS, SLOTS = 6, 5000, 97


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = multigpu.shard(NSEG, world, rank, "strong")
        parts = [_rows(s, ROWS, SLOTS) for s in mine]
        k = np.concatenate([p[0] for p in parts])
        iv = np.concatenate([p[1] for p in parts])
        fv = np.concatenate([p[2] for p in parts])
        t = torch.from_numpy(dense_table(k, iv, fv, SLOTS).reshape(-1).copy())
        multigpu.merge_dense_planes(t, OPS)
        fns = ["count", "sum", "min", "max", "avg"]
        vals = [(float(len(iv)), len(iv)), (float(iv.sum()), len(iv)), (float(iv.min()), len(iv)),
                (float(iv.max()), len(iv)), (float(iv.sum()), len(iv))]
        agg = multigpu.merge_aggregation(fns, vals)
        q.put((rank, mine, t.numpy().copy(), agg))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_covers_every_segment_once():
    for world in (1, 2, 3, 8):
        got = sorted(s for r in range(world) for s in multigpu.shard(4096, world, r, "strong"))
        assert got == list(range(4096))
        weak = [multigpu.shard(8, world, r, "weak") for r in range(world)]
        assert all(len(w) == 8 for w in weak) and len({s for w in weak for s in w}) == 8 * world


def test_two_rank_merge_matches_single_process():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    assert sorted(res[0][1] + res[1][1]) == list(range(NSEG))
    allp = [_rows(s, ROWS, SLOTS) for s in range(NSEG)]
    k = np.concatenate([p[0] for p in allp])
    iv = np.concatenate([p[1] for p in allp])
    fv = np.concatenate([p[2] for p in allp])
    exp = dense_table(k, iv, fv, SLOTS).reshape(-1)
    for rank, _, t, agg in res:
        t2 = t.reshape(5, SLOTS)
        e2 = exp.reshape(5, SLOTS)
        assert np.array_equal(t2[:4], e2[:4]), "integer / ordered planes must merge bit-exactly"
        np.testing.assert_allclose(t2[4].view(np.float64), e2[4].view(np.float64), rtol=1e-9)
        assert agg[0] == (float(len(iv)), len(iv))
        assert agg[1][0] == float(iv.sum()) and agg[2][0] == float(iv.min()) and agg[3][0] == float(iv.max())
        assert agg[4] == (float(iv.sum()), len(iv))


# ------------------------------------------------------------------------------------------------
# Sparse group-by across ranks (multigpu.gather_group_partials / merge_group_partials / trim_to_size): every rank
# combines its segments with the oracle, hands its groups over as value-keyed arrays, rank 0 merges and trims; the
# result must equal the oracle's combine (MCombineGroupByOperator + trimToSize) over ALL segments.
# ------------------------------------------------------------------------------------------------
SP_NSEG, SP_ROWS = 4, 12000
SP_QUERY = "SELECT SUM(m), MIN(m), MAX(m), COUNT(*), AVG(m) FROM t GROUP BY g1, g2 TOP 10"


def _sparse_segments():
    from oracle import pinot_oracle as O
    segs = []
    for s in range(SP_NSEG):
        rng = np.random.default_rng(100 + s)
        # per-segment value domains differ (different dictionaries on different ranks); ~40k distinct keys overall
        raw = {"g1": rng.integers(0, 200, SP_ROWS).astype(np.int32) * 7 + s,
               "g2": rng.integers(-100, 100, SP_ROWS).astype(np.int32),
               "m": rng.integers(0, 1 << 20, SP_ROWS).astype(np.int32)}
        segs.append(O.OSegment.from_raw(raw))
    return segs


def _partial_arrays(merged, fns):
    keys = list(merged)
    ncols = len(keys[0].split("\t")) if keys else 2
    cols = [np.array([int(k.split("\t")[c]) for k in keys], dtype=np.int64) for c in range(ncols)]
    vals = np.zeros((len(fns), len(keys)))
    cnts = np.zeros((len(fns), len(keys)), dtype=np.int64)
    for j, k in enumerate(keys):
        for i, f in enumerate(fns):
            v = merged[k][i]
            if f == "count":
                cnts[i, j] = v
            elif f in ("avg", "avgmv"):
                vals[i, j], cnts[i, j] = v[0], v[1]
            else:
                vals[i, j] = v
    return cols, vals, cnts


def _sparse_worker(rank, world, port, q):
    import torch.distributed as dist
    from oracle import pinot_oracle as O
    from pinot_amd import pql
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        req = pql.compile(SP_QUERY)
        fns = [a["fn"] for a in req["aggregations"]]
        segs = _sparse_segments()
        mine = multigpu.shard(SP_NSEG, world, rank, "strong")
        local = O.combine_group_by([O.run_group_by(segs[s], req) for s in mine], req)["merged"]
        parts = multigpu.gather_group_partials(*_partial_arrays(local, fns))
        out = None
        if rank == 0:
            cols, vals, cnts = multigpu.merge_group_partials(fns, parts)
            kept = multigpu.trim_to_size(fns, vals, cnts, req["group_by"].get("top_n", 10))
            out = (cols, vals, cnts, kept)
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_two_rank_sparse_group_merge_and_trim_match_oracle_combine():
    import torch.multiprocessing as mp
    from oracle import pinot_oracle as O
    from pinot_amd import pql
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sparse_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    cols, vals, cnts, kept = res[0]
    req = pql.compile(SP_QUERY)
    fns = [a["fn"] for a in req["aggregations"]]
    exp = O.combine_group_by([O.run_group_by(s, req) for s in _sparse_segments()], req)
    keys = ["%d\t%d" % (a, b) for a, b in zip(cols[0], cols[1])]
    assert len(keys) == len(exp["merged"]) > 20000  # the trim engages
    assert set(keys) == set(exp["merged"])
    for j, k in enumerate(keys):
        e = exp["merged"][k]
        for i, f in enumerate(fns):
            if f == "count":
                assert cnts[i, j] == e[i]
            elif f == "avg":
                assert cnts[i, j] == e[i][1] and abs(vals[i, j] - e[i][0]) <= 1e-9 * abs(e[i][0])
            elif f == "sum":
                assert abs(vals[i, j] - e[i]) <= 1e-9 * abs(e[i])
            else:
                assert vals[i, j] == e[i]  # MIN / MAX bit-exact
    for i, f in enumerate(fns):  # trimmed: same size and the same multiset of kept values (ties are arbitrary)
        got = sorted(float(cnts[i, j]) if f == "count" else
                     (vals[i, j] / cnts[i, j] if f == "avg" else vals[i, j]) for j in kept[i])
        want = sorted(float(v) if f == "count" else (v[0] / v[1] if f == "avg" else v)
                      for v in exp["trimmed"][i].values())
        assert len(got) == len(want) == exp["trim_size"]
        np.testing.assert_allclose(got, want, rtol=1e-9)


# ------------------------------------------------------------------------------------------------
# Dense key identity across ranks: slot i of a dense table means the same group on every GPU only
# when every rank built the same global dictionaries; otherwise the merge goes by key value.
# ------------------------------------------------------------------------------------------------
def _dict_segments(rank):
    """Rank-specific value sets: rank 1's group column holds values rank 0 never sees (and misses some of rank 0's)."""
    from oracle import pinot_oracle as O
    rng = np.random.default_rng(40 + rank)
    segs = []
    for s in range(2):
        n = 3000
        g = rng.choice(np.arange(rank * 7, rank * 7 + 40), n)  # rank 0: 0..39, rank 1: 7..46
        segs.append(O.OSegment.from_raw({"g": g.astype(np.int32), "m": rng.integers(0, 1000, n).astype(np.int32)}))
    return segs


def _dict_worker(rank, world, port, q):
    import torch.distributed as dist
    from oracle import pinot_oracle as O
    from pinot_amd import pql
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        segs = _dict_segments(rank)
        # key spaces: identical dictionaries on both ranks need no exchange (fingerprints agree), differing ones gather
        # their values; a second call with the same segment set is served from the cache (no collective at all)
        calls = []
        real = multigpu._gather_bytes
        multigpu._gather_bytes = lambda payload, device: calls.append(1) or real(payload, device)
        same_q, differ_q = _FakeQuery(["g"]), _FakeQuery(["g"])
        same_segs = [_FakeSeg({"g": _FakeCol(np.arange(40, dtype=np.int64), "INT")})]
        multigpu.union_key_domains(same_q, same_segs)
        n_same = len(calls)
        differ_segs = [_FakeSeg({"g": _FakeCol(np.unique(s.columns["g"].dictionary), "INT")}) for s in segs]
        multigpu.union_key_domains(differ_q, differ_segs)
        n_differ = len(calls) - n_same
        again = _FakeQuery(["g"])
        multigpu.union_key_domains(again, differ_segs)
        multigpu._gather_bytes = real
        checks = (n_same, n_differ, len(calls) - n_same - n_differ, same_q.set[0][1] == list(range(40)),
                  differ_q.set[0][1] == list(range(47)), again.set == differ_q.set)
        req = pql.compile("SELECT COUNT(*), SUM(m), MIN(m), MAX(m) FROM t GROUP BY g")
        fns = [a["fn"] for a in req["aggregations"]]
        local = O.combine_group_by([O.run_group_by(s, req) for s in segs], req)["merged"]
        parts = multigpu.gather_group_partials(*_partial_arrays(local, fns))
        out = multigpu.merge_group_partials(fns, parts) if rank == 0 else None
        q.put((rank, (checks, out)))
    finally:
        dist.destroy_process_group()


def test_two_rank_dense_layout_agreement_and_value_keyed_merge():
    import torch.multiprocessing as mp
    from oracle import pinot_oracle as O
    from pinot_amd import pql
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dict_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in (0, 1):
        assert res[r][0] == (0, 1, 0, True, True, True)  # same decision and the same union (0..46) on every rank
    cols, vals, cnts = res[0][1]
    req = pql.compile("SELECT COUNT(*), SUM(m), MIN(m), MAX(m) FROM t GROUP BY g")
    exp = O.combine_group_by([O.run_group_by(s, req) for r in (0, 1) for s in _dict_segments(r)], req)["merged"]
    got = {str(int(k)): [int(cnts[0, j]), vals[1, j], vals[2, j], vals[3, j]] for j, k in enumerate(cols[0])}
    assert set(got) == set(exp) and len(got) == 47
    for k, e in exp.items():
        assert got[k] == [e[0], e[1], e[2], e[3]]


# ------------------------------------------------------------------------------------------------
# Device-side sparse merge plumbing (multigpu.exchange_group_records): group records routed by key hash with one
# all_to_all_single; every key lands on exactly one rank, every record arrives once.
# ------------------------------------------------------------------------------------------------
def _a2a_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(rank)
        n = 5000 + 777 * rank
        keys = torch.randint(0, 1 << 40, (n,), generator=g, dtype=torch.int64)
        keys[:100] = torch.arange(100)  # keys present on every rank
        recs = torch.stack([keys, torch.ones(n, dtype=torch.int64), keys % 97, keys % 13, keys % 7], dim=1)
        out = multigpu.exchange_group_records(recs, world)
        q.put((rank, (recs.numpy(), out.numpy())))
    finally:
        dist.destroy_process_group()


def test_three_rank_group_record_exchange():
    import torch
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_a2a_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sent = np.concatenate([res[r][0] for r in range(3)])
    got = np.concatenate([res[r][1] for r in range(3)])
    assert sorted(map(tuple, sent.tolist())) == sorted(map(tuple, got.tolist()))
    for r in range(3):
        out = res[r][1]
        dest = multigpu.group_destination(torch.from_numpy(out[:, 0]), 3).numpy()
        assert np.all(dest == r)
    # the shared keys 0..99 are each on exactly one rank, all three copies together
    for k in range(100):
        holders = [r for r in range(3) if np.any(res[r][1][:, 0] == k)]
        assert len(holders) == 1 and np.sum(res[holders[0]][1][:, 0] == k) == 3


def test_trim_to_size_with_global_total():
    """Candidates = per-partition top-K of disjoint partitions: the threshold applies to the global group count."""
    rng = np.random.default_rng(0)
    vals = rng.permutation(12000).astype(np.float64)[None, :]
    cnts = np.ones((1, 12000), dtype=np.int64)
    kept = multigpu.trim_to_size(["sum"], vals, cnts, 10, total=50000)[0]  # 50000 > 20000: keep the best 5000
    assert len(kept) == 5000 and set(vals[0, kept]) == set(range(7000, 12000))
    assert len(multigpu.trim_to_size(["sum"], vals, cnts, 10, total=15000)[0]) == 12000  # below the threshold: all


# ------------------------------------------------------------------------------------------------
# Cross-process key identity (multigpu.union_key_domains): every rank contributes its group columns' dictionary values,
# every rank sets the SAME sorted union as the query's key domain (pgx_query_set_key_domain), whatever it holds itself.
# ------------------------------------------------------------------------------------------------
class _FakeCol:
    def __init__(self, values, dt):
        self.values = values
        self.meta = type("M", (), {"data_type": dt})()


class _FakeSeg:
    def __init__(self, cols):
        self.cols = cols

    def column(self, name):
        return self.cols[name]


class _FakeQuery:
    """Records the domains union_key_domains sets (the library call is the GPU tests' part)."""
    def __init__(self, group_cols):
        self.group_cols = group_cols
        self.set = {}

    def set_key_domain(self, g, values, dt):
        if dt == "STRING":
            vals = sorted(set(values), key=lambda v: v.encode("utf-8"))
        else:
            vals = np.unique(np.asarray(values, dtype=np.float64 if dt in ("FLOAT", "DOUBLE") else np.int64)).tolist()
        self.set[g] = (dt, vals)


def _cache_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        calls = []
        real = multigpu._gather_bytes
        multigpu._gather_bytes = lambda payload, device: calls.append(1) or real(payload, device)
        a = _FakeSeg({"g": _FakeCol(np.arange(rank * 5, rank * 5 + 20, dtype=np.int64), "INT")})
        a.uid = 1000 + rank
        seen = []
        for step in range(4):
            segs = [a]
            if rank == 1 and step >= 2:  # only rank 1's segment set changes (a new segment, e.g. a realtime snapshot)
                b = _FakeSeg({"g": _FakeCol(np.arange(100, 103, dtype=np.int64), "INT")})
                b.uid = 2000 + step  # a fresh uid per step: never a cache hit on rank 1's side
                segs = [a, b]
            fq = _FakeQuery(["g"])
            before = len(calls)
            multigpu.union_key_domains(fq, segs)
            seen.append((len(calls) - before, fq.set[0][1]))
        multigpu._gather_bytes = real
        q.put((rank, seen))
    finally:
        dist.destroy_process_group()


def test_union_domain_cache_decides_collectively():
    """one rank's segment set changes while the other's does not.  Every rank must miss together
    (the same collectives run on both: no hang, no pairing with the next collective) and see the new union."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_cache_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0] == res[1]
    base = list(range(0, 25))
    grown = base + [100, 101, 102]
    # step 0: miss (differing dictionaries gather), 1: hit, 2 and 3: rank 1 changed -> both ranks gather again
    assert [c for c, _ in res[0]] == [1, 0, 1, 1]
    assert [v for _, v in res[0]] == [base, base, grown, grown]


def _domain_segments(rank):
    segs = []
    for s in range(2):
        ints = np.arange(rank * 50 + s * 10, rank * 50 + s * 10 + 60, dtype=np.int64)  # overlapping ranges
        strs = ["k%d" % (rank * 3 + s + i) for i in range(4)] + ["été", "a\tb"]
        dbl = np.array([0.5 * rank, 1.25, -3.0 + s])
        segs.append(_FakeSeg({"i": _FakeCol(ints, "INT"), "s": _FakeCol(strs, "STRING"), "d": _FakeCol(dbl, "DOUBLE")}))
    return segs


def _domain_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fq = _FakeQuery(["i", "s", "d"])
        multigpu.union_key_domains(fq, _domain_segments(rank) if rank < 2 else [])  # rank 2 holds no segment
        q.put((rank, fq.set))
    finally:
        dist.destroy_process_group()


def test_union_key_domains_identical_on_every_rank():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_domain_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0] == res[1] == res[2]
    every = _domain_segments(0) + _domain_segments(1)
    exp_i = sorted({int(v) for s in every for v in s.column("i").values})
    exp_s = sorted({v for s in every for v in s.column("s").values}, key=lambda v: v.encode("utf-8"))
    exp_d = sorted({float(v) for s in every for v in s.column("d").values})
    assert res[0][0] == ("INT", exp_i) and res[0][1] == ("STRING", exp_s) and res[0][2] == ("DOUBLE", exp_d)
    assert len(exp_i) == 120  # rank 0: 0..69, rank 1: 50..119


# ------------------------------------------------------------------------------------------------
# Multi-value GROUP BY across ranks (VERDICT r3 missing #1): each rank's partial is its segments' combined group map
# (keys expanded per value, MINMV / MAXMV folded per doc, MinMVAggregationFunction.java:103-119); the value-keyed
# merge (multigpu.merge_group_partials: sum / count / AVGMV pairs add, MINMV / MAXMV take Math.min / Math.max like
# combineTwoValues) must equal the oracle's combine over every rank's segments.
# ------------------------------------------------------------------------------------------------
MV_QUERY = "SELECT COUNT(*), SUMMV(vals), MINMV(vals), MAXMV(vals), AVGMV(vals), COUNTMV(vals) FROM t GROUP BY tags, d"


def _mv_segments(rank):
    from oracle import pinot_oracle as O
    rng = np.random.default_rng(70 + rank)
    segs = []
    for s in range(2):
        n = 1500
        tags = [rng.integers(0, 12, rng.integers(1, 4)).tolist() for _ in range(n)]
        vals = [rng.integers(-500, 500, rng.integers(1, 4)).tolist() for _ in range(n)]
        segs.append(O.OSegment.from_raw({"tags": tags, "vals": vals,
                                         "d": rng.integers(rank, 5 + rank, n).astype(np.int32)}))
    return segs


def _mv_worker(rank, world, port, q):
    import torch.distributed as dist
    from oracle import pinot_oracle as O
    from pinot_amd import pql
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        req = pql.compile(MV_QUERY)
        fns = [a["fn"] for a in req["aggregations"]]
        local = O.combine_group_by([O.run_group_by(s, req) for s in _mv_segments(rank)], req)["merged"]
        parts = multigpu.gather_group_partials(*_partial_arrays(local, fns))
        q.put((rank, multigpu.merge_group_partials(fns, parts) if rank == 0 else None))
    finally:
        dist.destroy_process_group()


def test_two_rank_mv_group_by_merge_matches_oracle():
    import torch.multiprocessing as mp
    from oracle import pinot_oracle as O
    from pinot_amd import pql
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_mv_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    cols, vals, cnts = res[0]
    req = pql.compile(MV_QUERY)
    exp = O.combine_group_by([O.run_group_by(s, req) for r in (0, 1) for s in _mv_segments(r)], req)["merged"]
    got = {}
    for j in range(len(cols[0])):
        key = "%d\t%d" % (cols[0][j], cols[1][j])
        got[key] = [int(cnts[0, j]), vals[1, j], vals[2, j], vals[3, j], (vals[4, j], int(cnts[4, j])), vals[5, j]]
    assert set(got) == set(exp)
    for k, e in exp.items():
        g = got[k]
        assert g[0] == e[0] and g[1] == e[1] and g[2] == e[2] and g[3] == e[3]
        assert g[4][0] == e[4][0] and g[4][1] == e[4][1] and g[5] == e[5]
