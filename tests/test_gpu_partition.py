"""GPU parity of the partitioned sparse group-by (pgx_part.cpp run_partitioned: record-emitting query kernel, two
radix passes, per-partition LDS aggregation) for LONG_MAP-sized key spaces: against the oracle, against the global
hash-table path (PGX_X_NO_PARTITION), across segments with different group dictionaries, and through its resize /
re-split / fallback branches (PGX_DEBUG=part_small starts from undersized buckets and a single pass)."""
import numpy as np
import pytest

from pinot_amd import pql
from tests import helpers as H
from tests.test_gpu_parity import FILTERS, _rand_segment, _run_inner

pytestmark = pytest.mark.gpu

AGGS = "SELECT COUNT(*), SUM(m), MIN(m), MAX(m), AVG(m) FROM t"


@pytest.fixture(scope="module")
def ctx():
    from pinot_amd import engine as E
    c = E.Context(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def seg(ctx):
    from pinot_amd import engine as E
    rng = np.random.default_rng(21)
    n = 8192 * 5 + 333
    raw = _rand_segment(rng, n, {"a": 3000, "b": 40, "c": 700, "s": 6, "g1": 13, "g2": 900, "m": 5000}, "p",
                        sorted_col="s")
    seg, oseg = H.build_pair("p", raw, inverted=("b", "c"))
    fmt = {"b0": int(np.unique(raw["b"])[0]), "b1": int(np.unique(raw["b"])[5]), "b2": int(np.unique(raw["b"])[9]),
           "s0": int(np.unique(raw["s"])[1]), "s1": int(np.unique(raw["s"])[4])}
    return E.IndexSegment(ctx, seg), oseg, fmt


def _map(blk):
    g = blk.get_aggregation_group_by_result()
    return g.as_map() if g is not None else {}


def _execute(ctx, segs, q, flags):
    from pinot_amd import engine as E
    from pinot_amd import native as N
    qq = E._Query(ctx, q)
    r = qq.execute(segs, flags=flags)
    try:
        return E.decode_result(qq, r, segs)
    finally:
        N.lib().pgx_result_release(r)


@pytest.mark.parametrize("mode", ["narrow", "direct", "gather", "radix"])
@pytest.mark.parametrize("flt", FILTERS)
@pytest.mark.parametrize("group", [" GROUP BY g2, a, c", " GROUP BY a, c, g1", " GROUP BY c, g2, s, g1"])
def test_partitioned_matches_oracle(ctx, seg, flt, group, mode, monkeypatch):
    """Both sparse paths: narrow records (default: the scan's 256-way split, pgx_narrow_split, wavefront tables; the
    first two key shapes need records wider than 32 bits out of the scan, the u16 array; "direct": the records carry
    value offsets instead of dictIds, PGX_PART_NARROW=direct; "gather": the records carry the dictId's index in a
    global table of value offsets, gathered by the aggregation, PGX_PART_NARROW=gather) and the 8-byte radix path
    (PGX_PART_NARROW=0)."""
    monkeypatch.setenv("PGX_PART_NARROW", {"narrow": "1", "direct": "direct", "gather": "gather", "radix": "0"}[mode])
    gseg, oseg, fmt = seg
    q = pql.compile(AGGS + (flt % fmt) + group)
    blk, st = _run_inner(ctx, gseg, q)
    o = H.oracle_answer([oseg], q, literal=True)
    s = st.as_list()
    assert s == list(o["stats"])  # incl. numEntriesScannedInFilter (literal iterator algebra)
    gr = blk.get_aggregation_group_by_result()
    m = gr.as_map() if gr is not None else {}
    assert set(m) == set(o["map"])
    fns = [a["fn"] for a in q["aggregations"]]
    for k, v in o["map"].items():
        H.assert_values_equal(m[k], v, fns)
    if gr is not None:
        assert gr.storage_mode == o["mode"]


@pytest.mark.parametrize("text", [
    AGGS + " GROUP BY g2, a, c",
    "SELECT COUNT(*) FROM t WHERE a > 0 GROUP BY a, c",
    "SELECT MAX(m), COUNT(*) FROM t WHERE b IN (%(b0)s, %(b2)s) GROUP BY g1, s",
])
@pytest.mark.parametrize("force_hash", [False, True])
def test_partitioned_equals_hash_table(ctx, seg, text, force_hash):
    from pinot_amd import native as N
    gseg, _, fmt = seg
    q = pql.compile(text % fmt)
    base = N.PGX_X_FORCE_HASH if force_hash else 0
    part = _execute(ctx, [gseg], q, base)
    table = _execute(ctx, [gseg], q, base | N.PGX_X_NO_PARTITION)
    assert _map(part) == _map(table)
    assert part.stats.as_list() == table.stats.as_list()


def test_partitioned_multi_segment_remap(ctx):
    """Group columns with a different dictionary per segment (keys merged by value through the remap tables), one
    shared dictionary for the aggregated column (one value base: the partitioned path's precondition)."""
    from pinot_amd import engine as E
    rng = np.random.default_rng(5)
    mdom = np.sort(rng.choice(np.arange(-10 ** 6, 10 ** 6), size=300, replace=False)).astype(np.int32)
    gsegs, osegs = [], []
    for i in range(3):
        n = 20000 + 7001 * i
        mid = rng.integers(0, len(mdom), size=n)
        mid[:len(mdom)] = np.arange(len(mdom))
        raw = {"k": (rng.integers(0, 3000 + 500 * i, size=n) * 7).astype(np.int32),
               "x": np.array(["v%d" % v for v in rng.integers(0, 2000 + 100 * i, size=n)]),
               "m": mdom[rng.permutation(mid)]}
        s, o = H.build_pair("ps%d" % i, raw)
        gsegs.append(E.IndexSegment(ctx, s))
        osegs.append(o)
    q = pql.compile(AGGS + " WHERE m > -500000 GROUP BY x, k")
    blk = E.InstancePlanMakerImplV2(ctx).make_inter_segment_plan(gsegs, q).execute()
    o = H.oracle_answer(osegs, q, literal=False)
    m = blk.get_aggregation_group_by_result().as_map()
    assert set(m) == set(o["map"])
    fns = [a["fn"] for a in q["aggregations"]]
    for k, v in o["map"].items():
        H.assert_values_equal(m[k], v, fns)


def _pairs_segment(ctx, n, card, seed):
    from pinot_amd import engine as E
    rng = np.random.default_rng(seed)
    raw = {"ga": rng.integers(0, card, size=n).astype(np.int32),
           "gb": rng.integers(0, card, size=n).astype(np.int32) * 3,
           "m": rng.integers(-5000, 5000, size=n).astype(np.int32),
           "m2": (rng.integers(0, 3000, size=n) * 7 - 9000).astype(np.int32)}
    raw["md"] = raw["m2"] / 4.0 + 0.25  # DOUBLE, exact in binary
    raw["ga"][:card] = np.arange(card)
    raw["gb"][:card] = np.arange(card) * 3
    raw["m"][:2] = [-5000, 4999]
    s, _ = H.build_pair("pp%d" % seed, raw, types={"md": "DOUBLE"})
    return E.IndexSegment(ctx, s), raw


def _expected(raw):
    key = raw["ga"].astype(np.int64) * (1 << 32) + raw["gb"].astype(np.int64)
    u, inv = np.unique(key, return_inverse=True)
    m = raw["m"].astype(np.int64)
    cnt = np.bincount(inv)
    sm = np.bincount(inv, weights=m)
    mn = np.full(len(u), np.iinfo(np.int64).max)
    mx = np.full(len(u), np.iinfo(np.int64).min)
    np.minimum.at(mn, inv, m)
    np.maximum.at(mx, inv, m)
    out = {}
    for i, k in enumerate(u.tolist()):
        out["%d\t%d" % (k >> 32, k & 0xFFFFFFFF)] = (int(cnt[i]), float(sm[i]), float(mn[i]), float(mx[i]))
    return out


@pytest.mark.parametrize("n,card", [(400000, 1000), (1200000, 2000)])
def test_partitioned_debug_resize_and_fallback(ctx, monkeypatch, n, card):
    """PGX_DEBUG=part_small: pass-1 buckets start undersized (resize from the measured counts), one pass of 128
    partitions (~n distinct groups overflow the LDS tables: re-split), and at most one re-split: the 1.2M-row case
    still overflows and falls back to the global hash table.  Both must be exact."""
    monkeypatch.setenv("PGX_DEBUG", "part_small")
    monkeypatch.setenv("PGX_PART_NARROW", "0")  # the radix path's own resize / re-split branches
    gseg, raw = _pairs_segment(ctx, n, card, seed=card)
    q = pql.compile("SELECT COUNT(*), SUM(m), MIN(m), MAX(m) FROM t GROUP BY ga, gb")
    got = _map(_execute(ctx, [gseg], q, 0))
    exp = _expected(raw)
    assert len(got) == len(exp)
    for k, (c, s, lo, hi) in exp.items():
        g = got[k]
        assert (int(g[0]), float(g[1]), float(g[2]), float(g[3])) == (c, s, lo, hi)


def _trim_expect(exp, fn, size=5000):
    rows = list(exp.values())
    if fn == "count":
        vals = sorted((r[0] for r in rows), reverse=True)
    elif fn == "sum":
        vals = sorted((r[1] for r in rows), reverse=True)
    elif fn == "min":
        vals = sorted(r[2] for r in rows)
    elif fn == "max":
        vals = sorted((r[3] for r in rows), reverse=True)
    else:
        vals = sorted((r[1] / r[0] for r in rows), reverse=True)
    return vals[:size]


@pytest.mark.parametrize("flags", [0, "table"])
def test_combine_trim_on_device(ctx, flags):
    """Combine trim (a-19) over more than 20,000 groups: the 5,000 best groups per function (MIN ascending, AVG by
    sum/count).  Sparse results trim on the device (radix select) and read back only the kept groups; the hash-table
    path trims on the host.  Kept values must equal the expected top values (ties at the threshold are unpinned, so
    values are compared as sorted lists) and every kept group must carry its own untrimmed value."""
    from pinot_amd import engine as E
    from pinot_amd import native as N
    gseg, raw = _pairs_segment(ctx, 300000, 700, seed=77)
    exp = _expected(raw)
    assert len(exp) > 20000
    q = pql.compile("SELECT COUNT(*), SUM(m), MIN(m), MAX(m), AVG(m) FROM t GROUP BY ga, gb")
    qq = E._Query(ctx, q)
    r = qq.execute([gseg], flags=N.PGX_X_NO_PARTITION if flags == "table" else 0)
    try:
        maps = E.trimmed_maps(qq, r, [gseg])
    finally:
        N.lib().pgx_result_release(r)
    for i, fn in enumerate(qq.fns):
        m = maps[i]
        assert len(m) == 5000
        if fn == "avg":
            got = sorted((s / c for s, c in m.values()), reverse=True)
        else:
            got = sorted(m.values(), reverse=(fn != "min"))
        assert got == _trim_expect(exp, fn), fn
        col = {"count": 0, "sum": 1, "min": 2, "max": 3}.get(fn)
        for k, v in m.items():
            e = exp[k]
            assert (v == (float(e[1]), e[0])) if fn == "avg" else (v == e[col]), (fn, k, v, e)


def test_group_partials_split_then_merged_equal_one_launch(ctx):
    """The cross-GPU sparse merge (multigpu.merge_group_partials over engine.group_partials): segments split over two
    'ranks' with different dictionaries, each rank's groups read back by VALUE, merged on the host, equal the groups
    of one launch over all segments."""
    from pinot_amd import engine as E
    from pinot_amd import multigpu as MG
    from pinot_amd import native as N
    rng = np.random.default_rng(8)
    mdom = np.sort(rng.choice(np.arange(-10 ** 6, 10 ** 6), size=300, replace=False)).astype(np.int32)
    gsegs = []
    for i in range(3):
        n = 30000 + 5003 * i
        raw = {"k": (rng.integers(0, 2500 + 400 * i, size=n) * 3).astype(np.int32),
               "x": np.array(["w%d" % v for v in rng.integers(0, 1500 + 90 * i, size=n)]),
               "m": mdom[rng.integers(0, len(mdom), size=n)]}
        s, _ = H.build_pair("gp%d" % i, raw)
        gsegs.append(E.IndexSegment(ctx, s))
    q = pql.compile(AGGS + " GROUP BY x, k")
    fns = [a["fn"] for a in q["aggregations"]]
    whole = _map(_execute(ctx, gsegs, q, 0))
    parts = []
    for part in (gsegs[:2], gsegs[2:]):
        qq = E._Query(ctx, q)
        r = qq.execute(part)
        try:
            parts.append(E.group_partials(qq, r, part))
        finally:
            N.lib().pgx_result_release(r)
    cols, vals, cnts = MG.merge_group_partials(fns, parts)
    everything = [np.arange(vals.shape[1])] * len(fns)
    maps = E.render_group_maps(E._Query(ctx, q), gsegs, cols, vals, cnts, everything)
    merged = {k: [maps[i][k] for i in range(len(fns))] for k in maps[0]}
    assert set(merged) == set(whole) and len(whole) > 20000
    for k, v in whole.items():
        H.assert_values_equal(merged[k], v, fns)


@pytest.mark.parametrize("text", [AGGS + " GROUP BY g2, a, c", "SELECT COUNT(*) FROM t WHERE a > 0 GROUP BY a, c",
                                  "SELECT MIN(m), MAX(m) FROM t WHERE b <> %(b1)s GROUP BY c, g2, s, g1"])
def test_radix_row_records_equal_oracle(ctx, seg, text, monkeypatch):
    """The 8-byte radix path (PGX_PART_NARROW=0): row-order value records, two radix passes, LDS aggregation; COUNT-only
    keys and MIN / MAX-only functions included.  Against the oracle."""
    monkeypatch.setenv("PGX_PART_NARROW", "0")
    gseg, oseg, fmt = seg
    q = pql.compile(text % fmt)
    blk, st = _run_inner(ctx, gseg, q)
    o = H.oracle_answer([oseg], q, literal=True)
    assert st.as_list() == list(o["stats"])
    m = _map(blk)
    assert set(m) == set(o["map"])
    fns = [a["fn"] for a in q["aggregations"]]
    for k, v in o["map"].items():
        H.assert_values_equal(m[k], v, fns)


@pytest.mark.parametrize("case", ["uniform", "coarse", "skew", "count_only", "min_only"])
def test_narrow_paths_and_fallback(ctx, monkeypatch, capfd, case):
    """Narrow records end to end against numpy (every group's count / sum / min / max, exact), including the cases that
    must change course: "coarse" (PGX_DEBUG=narrow_k2=0: 256 partitions of ~1,500 groups overflow the 192-slot wavefront
    tables: the 8-byte radix path takes over) and "skew" (half the rows on one key: its slab and partition outgrow the
    capacities sized for a uniform mix, which are resized from the measured fills and the affected passes rerun).  COUNT-only records carry no value (26-bit records, one u32 array)."""
    from pinot_amd import engine as E
    rng = np.random.default_rng(99)
    n, card = 400000, 3000  # 3000 x 3000 keys > 2^22: a sparse (LONG_MAP) plan
    dom = np.sort(rng.choice(np.arange(-70000, 70000), size=20000, replace=False)).astype(np.int32)
    raw = {"ga": rng.integers(0, card, size=n).astype(np.int32),
           "gb": rng.integers(0, card, size=n).astype(np.int32) * 3,
           "m": dom[rng.integers(0, len(dom), size=n)]}  # 20,000 values: a value image the aggregation holds in LDS
    raw["ga"][:card] = np.arange(card)
    raw["gb"][:card] = np.arange(card) * 3
    if case == "skew":
        raw["ga"][card:n // 2 + card] = 7
        raw["gb"][card:n // 2 + card] = 21
    # narrow_log: one "[pgx narrow] ... ovf=a/b/c" line per narrow attempt
    monkeypatch.setenv("PGX_DEBUG", "narrow_log,narrow_k2=0" if case == "coarse" else "narrow_log")
    s, _ = H.build_pair("nw_" + case, raw)
    gseg = E.IndexSegment(ctx, s)
    try:
        text = {"count_only": "SELECT COUNT(*) FROM t GROUP BY ga, gb",
                "min_only": "SELECT MIN(m) FROM t GROUP BY ga, gb"}.get(case, "SELECT COUNT(*), SUM(m), MIN(m), MAX(m) "
                                                                           "FROM t GROUP BY ga, gb")
        q = pql.compile(text)
        got = _map(_execute(ctx, [gseg], q, 0))
        exp = _expected(raw)
        assert len(got) == len(exp)
        for k, (c, sm, lo, hi) in exp.items():
            g = got[k]
            if case == "count_only":
                assert int(g[0]) == c
            elif case == "min_only":
                assert float(g[0]) == lo
            else:
                assert (int(g[0]), float(g[1]), float(g[2]), float(g[3])) == (c, sm, lo, hi)
        lines = [x for x in capfd.readouterr().err.splitlines() if x.startswith("[pgx narrow]")]
        assert len(lines) == 1, lines  # the narrow path was attempted ...
        kept = lines[0].endswith("ok=1")
        assert kept == (case != "coarse"), lines  # ... and kept unless a wavefront table overflowed
        if case == "skew":  # the hot key's partition outgrew the first capacities: resized from the fills, rerun
            assert "attempts=1 " not in lines[0], lines
    finally:
        gseg.destroy()


@pytest.mark.parametrize("metric", ["int_own_dict", "int_gather", "long_own_dict", "double", "double_uniform",
                                    "double_radix"])
def test_partitioned_per_segment_metric_dictionaries(ctx, metric, monkeypatch):
    """VERDICT r4 missing #1: every segment builds its own metric dictionary (SegmentDictionaryCreator builds one per
    segment), so no two segments share a value image.  Integer metrics take a partitioned path with value offsets
    rebased per segment (JSeg.emit_rebase: one query-wide value base), not the global hash table -- the narrow records
    (64-bit second-stage records when the offsets are too wide for 32); a DOUBLE metric's records carry its index in the
    concatenation of the segments' dictionaries, aggregated in f64.  Groups (LONG_MAP key space > 2^22) and every function == the oracle's combine.
    "double_uniform" (ADVICE r5): non-dyadic doubles, whose f64 sums depend on the addition order -- the device adds
    with LDS atomics in arbitrary order, the reference in doc order -- so SUM / AVG are asserted to north_star's 1e-9
    relative (COUNT / MIN / MAX stay exact).  "int_gather": the integer records carry the dictId's index in a global
    table of every segment's value offsets (IMG 5, PGX_PART_NARROW=gather); DOUBLE metrics run the narrow records with
    the doubles gathered from the concatenated dictionaries (IMG 6), "double_radix" the 8-byte radix records."""
    if metric == "int_gather":
        monkeypatch.setenv("PGX_PART_NARROW", "gather")
    elif metric == "double_radix":
        monkeypatch.setenv("PGX_PART_NARROW", "0")
    import ctypes as C
    import json

    from pinot_amd import engine as E
    from pinot_amd import native as N
    L = N.lib()
    rng = np.random.default_rng(77)
    gsegs, osegs = [], []
    for i in range(3):
        n = 5000 + 800 * i
        if metric == "double":
            m = rng.integers(-40000, 40000, size=n) / 8.0 + 0.125 * i
            types = {"m": "DOUBLE"}
        elif metric in ("double_uniform", "double_radix"):
            m = rng.uniform(-5000.0, 5000.0, size=n)
            types = {"m": "DOUBLE"}
        elif metric == "long_own_dict":
            m = (rng.integers(0, 3_000_000_000, size=n) + (1 << 33) + 977 * i).astype(np.int64)
            types = {"m": "LONG"}
        else:
            m = (rng.integers(-2 ** 20, 2 ** 20, size=n) * (3 + i)).astype(np.int32)  # disjoint-ish value sets
            types = None
        raw = {"k": (rng.integers(0, 3000, size=n) * 7).astype(np.int32),
               "x": np.array(["v%d" % v for v in rng.integers(0, 2000, size=n)]), "m": m}
        s, o = H.build_pair("pd%s%d" % (metric, i), raw, types=types)
        gsegs.append(E.IndexSegment(ctx, s))
        osegs.append(o)
    q = pql.compile(AGGS + " WHERE k > 70 GROUP BY x, k")
    N.check(L.pgx_timing_start(ctx.handle))
    blk = E.InstancePlanMakerImplV2(ctx).make_inter_segment_plan(gsegs, q).execute()
    out = (C.c_double * 3)()
    js = C.create_string_buffer(8192)
    N.check(L.pgx_timing_stop(ctx.handle, out, js, len(js)))
    kernels = json.loads(js.value.decode())["kernels"]
    if metric == "double_radix":  # the concatenated dictionaries, f64 aggregation on the radix path
        assert "pgx_part_aggregate_f64" in kernels, kernels
    elif metric.startswith("double"):  # narrow records, the doubles gathered by the aggregation (IMG 6)
        assert "pgx_narrow_aggregate" in kernels and "pgx_part_aggregate_f64" not in kernels, kernels
    else:  # value offsets on the narrow records (no shared image: IMG 3, direct values) -- 32-bit offsets of LONG
        # values ride 64-bit second-stage records (narrow_wide) instead of the 8-byte radix path
        assert "pgx_narrow_aggregate" in kernels and "pgx_part_aggregate" not in kernels, kernels
    o = H.oracle_answer(osegs, q, literal=True)
    m = blk.get_aggregation_group_by_result().as_map()
    assert 10000 < len(o["map"]) < 20000  # sparse, below the combine trim
    assert set(m) == set(o["map"])
    fns = [a["fn"] for a in q["aggregations"]]
    for k, v in o["map"].items():
        H.assert_values_equal(m[k], v, fns, rel=1e-9 if metric.startswith("double") else 0.0)
    assert blk.stats.as_list() == list(o["stats"])


@pytest.mark.parametrize("mode", ["narrow", "radix"])
def test_partitioned_plan_cache_replays(ctx, seg, mode, monkeypatch, capfd):
    """A partitioned plan is kept with its slabs / buckets and partitions (pgx_plan_cache.cpp plan_cacheable, pgx_part.cpp replay_narrow,
    replay_part): the second and third executions of the same query over the same segment replay it (the host-profile
    line's "cached" mark; no second narrow sizing run), and every result -- decoded only after all three ran, so each
    result's group outputs are its own and the shared key tables outlive the replays -- equals the oracle's."""
    from pinot_amd import engine as E
    from pinot_amd import native as N
    monkeypatch.setenv("PGX_DEBUG", "host_profile,narrow_log")
    monkeypatch.setenv("PGX_PART_NARROW", "1" if mode == "narrow" else "0")
    gseg, oseg, fmt = seg
    q = pql.compile(AGGS + " WHERE a > 100 GROUP BY g2, a, c")
    o = H.oracle_answer([oseg], q, literal=True)
    qq = E._Query(ctx, q)
    results, marks, narrow_runs = [], [], 0
    for _ in range(3):
        results.append(qq.execute([gseg]))
        err = capfd.readouterr().err.splitlines()
        lines = [x for x in err if x.startswith("[pgx host us]")]
        narrow_runs += sum(x.startswith("[pgx narrow]") for x in err)
        assert lines, err
        marks.append(" cached=" in lines[-1])
    assert marks == [False, True, True]
    assert narrow_runs == (1 if mode == "narrow" else 0)
    fns = [a["fn"] for a in q["aggregations"]]
    for r in results:
        blk = E.decode_result(qq, r, [gseg])
        m = _map(blk)
        assert set(m) == set(o["map"])
        for k, v in o["map"].items():
            H.assert_values_equal(m[k], v, fns)
        assert blk.stats.as_list() == list(o["stats"])
        N.lib().pgx_result_release(r)
    qq.close()


MULTI_AGGS = "SELECT COUNT(*), SUM(m), MIN(m), MAX(b), SUM(c), AVG(b), MIN(s) FROM t"


def _kernels_of(ctx, fn):
    """Run fn() inside a kernel-timing window; returns (fn's value, kernel names that ran)."""
    import ctypes as C
    import json

    from pinot_amd import native as N
    L = N.lib()
    N.check(L.pgx_timing_start(ctx.handle))
    v = fn()
    out = (C.c_double * 3)()
    js = C.create_string_buffer(16384)
    N.check(L.pgx_timing_stop(ctx.handle, out, js, len(js)))
    return v, set(json.loads(js.value.decode())["kernels"])


@pytest.mark.parametrize("mode", ["narrow", "radix"])
@pytest.mark.parametrize("group", [" GROUP BY g2, a, c", " GROUP BY a, c, g1"])
def test_partitioned_several_value_columns(ctx, seg, group, mode, monkeypatch):
    """Functions over four value columns (m, b, c, s) with sparse keys: one partitioned pipeline run per column, the
    later passes' planes joined into the first pass's groups by key on the device (pgx_part.cpp run_value_columns,
    pgx_merge.hip pgx_join_*), not the global hash table.  Every group and function == the oracle's; statistics too."""
    monkeypatch.setenv("PGX_PART_NARROW", "1" if mode == "narrow" else "0")
    gseg, oseg, fmt = seg
    q = pql.compile(MULTI_AGGS + " WHERE a > 40" + group)
    (blk, st), kernels = _kernels_of(ctx, lambda: _run_inner(ctx, gseg, q))
    assert "pgx_join" in kernels, kernels
    assert ("pgx_narrow_aggregate" if mode == "narrow" else "pgx_part_aggregate") in kernels, kernels
    o = H.oracle_answer([oseg], q, literal=True)
    assert st.as_list() == list(o["stats"])
    m = _map(blk)
    assert set(m) == set(o["map"])
    fns = [a["fn"] for a in q["aggregations"]]
    for k, v in o["map"].items():
        H.assert_values_equal(m[k], v, fns)


def test_several_value_columns_trim_on_device(ctx):
    """Combine trim over > 20,000 groups of a two-column result (planes: count, then sum / min / max per column): the
    5,000 best groups of every function, each carrying its own untrimmed value (the trim's key reads the function's
    own plane)."""
    from pinot_amd import engine as E
    from pinot_amd import native as N
    gseg, raw = _pairs_segment(ctx, 300000, 3000, seed=78)  # 9M-slot key space: sparse (partitioned) keys
    raw2 = dict(raw)
    exp_m = _expected(raw)
    raw2["m"] = raw["m2"]
    exp_m2 = _expected(raw2)
    assert len(exp_m) > 20000
    q = pql.compile("SELECT SUM(m), MAX(m2), MIN(m2), MIN(m), COUNT(*) FROM t GROUP BY ga, gb")
    qq = E._Query(ctx, q)
    r, kernels = _kernels_of(ctx, lambda: qq.execute([gseg]))
    assert "pgx_join" in kernels, kernels
    try:
        maps = E.trimmed_maps(qq, r, [gseg])
    finally:
        N.lib().pgx_result_release(r)
    for i, (fn, exp, col) in enumerate([("sum", exp_m, 1), ("max", exp_m2, 3), ("min", exp_m2, 2), ("min", exp_m, 2),
                                        ("count", exp_m, 0)]):
        m = maps[i]
        assert len(m) == 5000
        got = sorted(m.values(), reverse=(fn != "min"))
        assert got == _trim_expect(exp, fn), (i, fn)
        for k, v in m.items():
            assert v == exp[k][col], (i, fn, k, v, exp[k])


@pytest.mark.parametrize("mode", ["narrow", "radix"])
def test_partitioned_double_and_int_value_columns(ctx, mode, monkeypatch):
    """A DOUBLE metric with its own dictionary in every segment beside an INT metric: the DOUBLE column's records
    carry its index in the concatenated dictionaries (JSeg.emit_rebase = the segment's place), aggregated in f64
    (pgx_part_aggregate_f64); the INT column runs its own pass and the two join by key.  Every group == the oracle's
    (f64 sums to 1e-12 relative: the device adds in another order), statistics too.  Narrow records (the doubles
    gathered by the aggregation) or the 8-byte radix records (PGX_PART_NARROW=0)."""
    from pinot_amd import engine as E
    if mode == "radix":
        monkeypatch.setenv("PGX_PART_NARROW", "0")
    rng = np.random.default_rng(91)
    gsegs, osegs = [], []
    for i in range(3):
        n = 6000 + 700 * i
        raw = {"k": (rng.integers(0, 2500, size=n) * 5).astype(np.int32),
               "x": np.array(["w%d" % v for v in rng.integers(0, 1800, size=n)]),
               "d": rng.integers(-30000, 30000, size=n) / 16.0 + 0.5 * i,
               "m": rng.integers(-7000, 7000, size=n).astype(np.int32)}
        sg, og = H.build_pair("pdm%d" % i, raw, types={"d": "DOUBLE"})
        gsegs.append(E.IndexSegment(ctx, sg))
        osegs.append(og)
    q = pql.compile("SELECT SUM(d), MIN(d), MAX(d), AVG(d), SUM(m), COUNT(*) FROM t WHERE k > 90 GROUP BY x, k")
    blk, kernels = _kernels_of(ctx, lambda: E.InstancePlanMakerImplV2(ctx).make_inter_segment_plan(gsegs, q).execute())
    agg = "pgx_narrow_aggregate" if mode == "narrow" else "pgx_part_aggregate_f64"
    assert agg in kernels and "pgx_join" in kernels, kernels
    o = H.oracle_answer(osegs, q, literal=True)
    m = blk.get_aggregation_group_by_result().as_map()
    assert 10000 < len(o["map"]) < 20000
    assert set(m) == set(o["map"])
    fns = [a["fn"] for a in q["aggregations"]]
    for k, v in o["map"].items():
        H.assert_values_equal(m[k], v, fns, rel=1e-12)
    assert blk.stats.as_list() == list(o["stats"])


@pytest.mark.parametrize("mode", ["narrow", "radix"])
def test_double_value_column_trim_on_device(ctx, mode, monkeypatch):
    """Combine trim over > 20,000 groups of a DOUBLE metric on the partitioned path: SUM / AVG keys read the f64 sum
    plane (TK_SUMF / TK_AVGF), MIN / MAX the ordered-f64 planes; the 5,000 best of each, every kept group with its own
    value.  Narrow records with gathered doubles (no key ranges from the aggregation: the trim finds them) or the radix
    path."""
    from pinot_amd import engine as E
    from pinot_amd import native as N
    if mode == "radix":
        monkeypatch.setenv("PGX_PART_NARROW", "0")
    gseg, raw = _pairs_segment(ctx, 300000, 3000, seed=79)
    raw2 = dict(raw)
    raw2["m"] = raw["md"]
    key = raw["ga"].astype(np.int64) * (1 << 32) + raw["gb"].astype(np.int64)
    u, inv = np.unique(key, return_inverse=True)
    cnt = np.bincount(inv)
    sm = np.bincount(inv, weights=raw["md"])
    mx = np.full(len(u), -np.inf)
    np.maximum.at(mx, inv, raw["md"])
    exp = {"%d\t%d" % (k >> 32, k & 0xFFFFFFFF): (int(cnt[i]), float(sm[i]), 0.0, float(mx[i]))
           for i, k in enumerate(u.tolist())}
    assert len(exp) > 20000
    q = pql.compile("SELECT SUM(md), MAX(md), AVG(md) FROM t GROUP BY ga, gb")
    qq = E._Query(ctx, q)
    r, kernels = _kernels_of(ctx, lambda: qq.execute([gseg]))
    assert ("pgx_narrow_aggregate" if mode == "narrow" else "pgx_part_aggregate_f64") in kernels, kernels
    try:
        maps = E.trimmed_maps(qq, r, [gseg])
    finally:
        N.lib().pgx_result_release(r)
    for i, fn in enumerate(["sum", "max", "avg"]):
        m = maps[i]
        assert len(m) == 5000
        if fn == "avg":
            got = sorted((s_ / c for s_, c in m.values()), reverse=True)
        else:
            got = sorted(m.values(), reverse=True)
        want = _trim_expect(exp, fn)
        assert np.allclose(got, want, rtol=1e-12, atol=0), fn
        for k, v in m.items():
            e = exp[k]
            if fn == "sum":
                assert abs(v - e[1]) <= 1e-9 * max(1.0, abs(e[1])), (k, v, e)
            elif fn == "max":
                assert v == e[3], (k, v, e)
