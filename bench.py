"""Benchmark of the MI355X segment query hot path (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c5|c2|c3|c1|c4|c6|c7]
  (N>1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...)

The default workload is c5, BASELINE configs[4] -- the metric's own shape: bitmap inverted-index AND/OR filter +
group-by SUM over 4096 x 2M-row segments, sharded over the GPUs.  A "step" is one execution of the query over all of
this rank's segments resident in HBM: predicate values resolved to dictId space for every segment (a-4, in the
library), bitmap sub-tree expansion, filter + decode + aggregate in the fused HIP kernel, the on-device combine, the
result back to the host, and for N>1 the cross-GPU merge.  Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (/opt/skills/guides/MI355X_MICROARCH.md, chip-level parameters)
METRIC = "rows/sec for filter+group-by SUM at 1/2/4/8 GPUs; % of HBM roofline"
# bounded CPU-baseline samples (segments, rows per segment): ~10-30 s of single-core work over 8 threads in total
CPU_SAMPLE = {"c2": (8, 32_000_000), "c5": (64, 2_000_000), "c3": (8, 16_000_000), "c3d": (8, 16_000_000),
              "c3f": (8, 16_000_000),
              "c6": (8, 8_000_000)}


def source_hash():
    """Hash of the library and kernel sources: stamps PMC traffic files (tools/pmc_traffic.py) so a measurement is only
    reported for the code it was taken on."""
    import hashlib
    h = hashlib.sha1()
    d = os.path.join(ROOT, "pinot_amd", "csrc")
    for f in sorted(os.listdir(d)):
        if f.endswith((".cpp", ".hip", ".h")):
            h.update(f.encode())
            h.update(open(os.path.join(d, f), "rb").read())
    return h.hexdigest()[:16]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default=os.environ.get("PGX_WORKLOAD", "c5"))
    ap.add_argument("--rows", type=int, default=0, help="override rows per segment (smoke/debug only)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--profile-iters", type=int, default=0, help="only run K steps (for rocprofv3 PMC passes)")
    ap.add_argument("--no-partition", action="store_true",
                    help="sparse group-by through the global hash table (PGX_X_NO_PARTITION), not the partitioned path")
    return ap.parse_args()


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch
        import torch.distributed as dist
        backend = os.environ.get("PGX_DIST_BACKEND", "nccl")  # "gloo": rehearse N ranks on fewer GPUs (box has 1)
        if backend != "nccl":
            local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return world, rank, local


def barrier_sync(world):
    import torch
    torch.cuda.synchronize()
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        torch.cuda.synchronize()


def cpu_baseline(wl, query, seg_rows, nseg, threads):
    """The oracle's C twin (oracle/pinot_oracle_c.c: one thread per segment, per-row readInt, 10000 / 5000-doc blocks,
    double SUM, hash-map group keys) on a bounded sample of the same workload, generated bit-identically on the host and
    timed on this host's cores: best of 5 after 2 warm-ups.  C5's leaves read the segments' roaring
    inverted indexes as the reference's BitmapBasedFilterOperator does (OR of the IN list's bitmaps, the NEQ leaf's
    flipped bitmap, AND block leapfrogging the OR block's iterator; tests/test_c_oracle_bitmap.py pins it)."""
    import numpy as np
    from oracle import c_oracle
    from pinot_amd import synth
    dicts = {c.name: synth.make_dictionary(c.dict_kind, c.card).astype(np.float64) for c in wl.columns}
    segs = [None] * nseg
    invs = [{} for _ in range(nseg)]

    def gen(s):
        cols = {}
        for ci, c in enumerate(wl.columns):
            if c.paired:
                fwd = c_oracle.synth_fwd(synth.column_seed(wl.seed, 0, ci), seg_rows, c.bits, c.card,
                                         pair_seed=synth.column_seed(wl.seed, s, 99), npairs=wl.npairs)
            else:
                fwd = c_oracle.synth_fwd(synth.column_seed(wl.seed, s, ci), seg_rows, c.bits, c.card)
            dv = (synth.make_dictionary(c.dict_kind, c.card, s).astype(np.float64)
                  if c.dict_kind in ("metric_seg", "metric_f64_seg") else dicts[c.name])
            cols[c.name] = (fwd, c.bits, dv, c.card)
            if c.inverted:  # the .bitmap.inv the GPU segments carry (synth.DeviceSegments._inverted_indexes)
                invs[s][c.name] = c_oracle.inverted_build(
                    c_oracle.synth_ids(synth.column_seed(wl.seed, s, ci), seg_rows, c.card), c.card)
        segs[s] = c_oracle.Segment(seg_rows, cols)

    ths = [threading.Thread(target=gen, args=(s,)) for s in range(nseg)]
    [t.start() for t in ths]
    [t.join() for t in ths]
    kw = {"threads": threads, "metric": "m"}
    if wl.name == "c2":
        kw.update(filter_col="dA", lo=64, hi=191)
    elif wl.name in ("c3", "c3d", "c3f"):
        kw.update(group_cols=("g1", "g2"))
    elif wl.name == "c5":  # (f1 IN (...) OR f2 = 7) AND f3 <> 3 GROUP BY gk: leaves as dictId bitsets
        f1 = [int(v) for v in query["filter"]["children"][0]["children"][0]["values"]]

        def bits(card, ids):
            w = np.zeros((card + 31) // 32, dtype=np.uint32)
            for i in ids:
                w[i >> 5] |= np.uint32(1 << (i & 31))
            return w
        kw.update(group_cols=("gk",), leaves=[("f1", bits(1000, f1)), ("f2", bits(100, [7])),
                                              ("f3", bits(10, [i for i in range(10) if i != 3]))],
                  prog=[0, 1, -2, 2, -1], inverted=invs, excl=[0, 0, 1])
    elif wl.name == "c6":  # ten range leaves ORed, as dictId bitsets: w_i < C6_CUT
        leaves = []
        for k, c in enumerate(wl.columns[:10]):
            w = np.zeros((c.card + 31) // 32, dtype=np.uint32)
            for i in range(synth.C6_CUT[k % 3]):
                w[i >> 5] |= np.uint32(1 << (i & 31))
            leaves.append((c.name, w))
        kw.update(group_cols=("gk",), leaves=leaves, prog=[0] + [x for i in range(1, 10) for x in (i, -2)])
    else:
        return None
    times = []
    out = None
    for it in range(7):
        t0 = time.perf_counter()
        out = c_oracle.run(segs, **kw)
        dt = time.perf_counter() - t0
        if it >= 2:
            times.append(dt)
    best = min(times)
    return {"value": nseg * seg_rows / best, "unit": "rows/s", "cores": threads, "kind": "port",
            "sample": "%d segments x %d rows of the same synthetic %s data (host-generated bit-identically), "
                      "oracle/pinot_oracle_c.c one thread per segment on %d threads, best of 5 after 2 warm-ups; "
                      "%.3f s per query" % (nseg, seg_rows, wl.name, threads, best),
            "result_count": int(sum(r["count"] for r in out))}


def cpu_baseline_c1(data):
    """C1 on the C twin (oracle/pinot_oracle_c.c): the whole baseball segment (100k rows), per-row readInt of yearID,
    the dictId interval of yearID >= 2000 (RangeOfflineDictionaryPredicateEvaluator), LONG_MAP group keys over
    playerName's dictIds, double SUM(runs); one thread (one segment); best of 20 after 3 warm-ups."""
    import numpy as np
    from oracle import c_oracle
    sd = data.seg_data
    cols = {}
    for name in ("yearID", "playerName", "runs"):
        c = sd.columns[name]
        fwd = np.frombuffer(bytes(c.fwd_bytes) + b"\0" * 8, dtype=np.uint8)
        dv = None if c.data_type == "STRING" else np.asarray(c.dictionary_values(), dtype=np.float64)
        cols[name] = (fwd, c.bits, dv, c.cardinality)
    years = np.asarray(sd.columns["yearID"].dictionary_values())
    lo = int(np.searchsorted(years, 2000, side="left"))
    seg = c_oracle.Segment(sd.total_docs, cols)
    kw = dict(filter_col="yearID", lo=lo, hi=len(years) - 1, metric="runs", group_cols=("playerName",), threads=1)
    times, out = [], None
    for it in range(23):
        t0 = time.perf_counter()
        out = c_oracle.run([seg], **kw)
        if it >= 3:
            times.append(time.perf_counter() - t0)
    best = min(times)
    return {"value": sd.total_docs / best, "unit": "rows/s", "cores": 1, "kind": "port",
            "sample": "the whole C1 segment (%d rows, the same bytes the GPU scans), oracle/pinot_oracle_c.c on one "
                      "thread, best of 20 after 3 warm-ups; %.3f ms per query" % (sd.total_docs, best * 1e3),
            "result_count": int(out[0]["count"]), "groups": int(out[0]["num_groups"])}


def cpu_baseline_c4(data, req):
    """C4 on the oracle's star-tree restatement (oracle/pinot_oracle.py star_tree_docs: StarTreeIndexOperator's BFS over
    the OFF_HEAP nodes, then the SUM scan of the selected docs, sum_by_group): the whole C4 segment, one thread, best of
    3 after 1 warm-up.  Pure Python: a port, not the reference's JIT-compiled Java."""
    import numpy as np
    from oracle import pinot_oracle as O
    sd = data.seg_data
    cols = {}
    for name, c in sd.columns.items():
        d = np.asarray(c.dictionary_values()).astype(np.int64)
        cols[name] = O.OColumn(name, c.data_type, d, c.dict_ids().astype(np.int64), c.is_sorted, c.has_inverted,
                               c.bits)
    os_ = O.OSegment(cols, sd.total_docs, sd.total_raw_docs)
    metrics = [a["column"] for a in req["aggregations"]]
    gcols = req["group_by"]["columns"]
    times, docs = [], None
    for it in range(4):
        t0 = time.perf_counter()
        docs = O.star_tree_docs(os_, sd.star_tree, req, sd.total_raw_docs)
        O.sum_by_group(os_, docs, metrics, gcols)
        if it >= 1:
            times.append(time.perf_counter() - t0)
    best = min(times)
    return {"value": sd.total_raw_docs / best, "unit": "raw rows represented/s", "cores": 1, "kind": "port",
            "sample": "the whole C4 segment (%d raw rows, %d docs incl. star-tree aggregates), star-tree traversal + "
                      "%d selected docs summed by oracle/pinot_oracle.py on one thread, best of 3 after 1 warm-up; "
                      "%.3f ms per query" % (sd.total_raw_docs, sd.total_docs, len(docs), best * 1e3),
            "docs_scanned": int(len(docs))}


def main():
    args = parse()
    world, rank, local = dist_setup(args)
    import ctypes as C

    import numpy as np
    import torch

    from pinot_amd import engine as E
    from pinot_amd import native as N
    from pinot_amd import pql, synth

    ctx = E.Context(local)
    from pinot_amd import multigpu
    t_gen = time.perf_counter()
    if args.workload == "c1":  # baseball quick-start shape, one 100k-row segment (latency-bound)
        data = synth.BaseballSegments(ctx, rows=args.rows or None)
        wl = synth.Workload("c1", "BASELINE configs[0]: baseballStats quick-start shape (100k rows, synthetic), "
                            "sum(runs) where yearID>=2000 group by playerName", 1, data.rows, [], synth.C1_QUERY, 1,
                            "weak")
        rows = data.rows
    elif args.workload == "c4":  # star-tree segment (weak scaling: one segment per GPU)
        data = synth.StarTreeSegments(ctx, rows=args.rows or None)
        wl = synth.Workload("c4", "BASELINE configs[3]: star-tree over 6 dims (cards %s) + 3 metrics, %d raw rows "
                            "per segment, maxLeafRecords 100000, filtered group-by served from pre-aggregated docs"
                            % (synth.C4_CARDS, data.rows), 1, data.rows, [], synth.C4_QUERY, 4, "weak")
        rows = data.rows
    else:
        wl = synth.WORKLOADS[args.workload]
        rows = args.rows or wl.rows
        seg_ids = multigpu.shard(wl.segments, world, rank, wl.scaling)
        data = synth.DeviceSegments(ctx, wl, seg_ids, rows=rows)
    t_gen = time.perf_counter() - t_gen
    req = pql.compile(wl.query)
    q = E._Query(ctx, req)
    segs = data.segments
    seg_arr = (C.c_void_p * len(segs))(*[s.handle.value for s in segs])
    L = N.lib()

    dense = False
    dense_t = None
    plane_ops = []
    if req.get("group_by") and world > 1:
        # one key space on every rank: the union of all ranks' group-column dictionaries, set once per query
        # shape (segment metadata, like staging); dense tables then all-reduce by slot over RCCL, sparse groups merge
        # on the device by packed key
        nccl = os.environ.get("PGX_DIST_BACKEND", "nccl") == "nccl"
        multigpu.union_key_domains(q, segs, device="cuda:%d" % local if nccl else None)
        slots = C.c_int64()
        N.check(L.pgx_query_dense_slots(q.handle, seg_arr, len(segs), C.byref(slots)))
        dense = 0 <= slots.value <= (1 << 22)  # -1: multi-value group-by, merged by key
    # Queries in flight (PGX_INFLIGHT, default 3): steps i + 1 and i + 2 are submitted (pgx_execute_async: predicate binding and
    # host planning on the library's threads, kernels on its own HIP stream) before step i is completed (wait, trim +
    # read-back, cross-GPU merge), as a server overlaps consecutive queries.  Every step still runs its whole query;
    # the line also reports the one-query-at-a-time latency (PGX_INFLIGHT=1 gives that timing for every step).
    inflight = max(1, int(os.environ.get("PGX_INFLIGHT", "3")))
    if world > 1 and req.get("group_by") and not dense:
        inflight = 1  # sparse cross-GPU merges (all-to-all + device merge) run one query at a time
    streams = [torch.cuda.Stream(device="cuda:%d" % local) for _ in range(inflight)]
    if dense:
        nplanes = 1 + len(req["aggregations"])
        for p in range(nplanes):
            op = C.c_int32()
            N.check(L.pgx_query_dense_plane_op(q.handle, seg_arr, len(segs), p, C.byref(op)))
            plane_ops.append(op.value)
        dense_t = [torch.zeros(nplanes * slots.value, dtype=torch.int64, device="cuda:%d" % local)
                   for _ in range(inflight)]

    merged = [None]

    def submit(i):
        """Start step i: a-4 per segment (pgx_bind_predicates), then the asynchronous execution on stream i."""
        binds, _owner = q.bindings(segs, seg_arr)  # the library copies the bindings before pgx_execute_async returns
        r = C.c_void_p()
        hs = streams[i % inflight].cuda_stream
        flags = N.PGX_X_THROUGHPUT if inflight > 1 else 0  # queries overlap: one launch per kernel, not batches
        if args.no_partition:
            flags |= N.PGX_X_NO_PARTITION
        if dense:
            d = dense_t[i % inflight]
            opts = N.ExecOpts(hs, C.c_void_p(d.data_ptr()), d.numel() * 8, N.PGX_X_KEEP_DENSE_ON_DEVICE | flags)
        else:
            opts = N.ExecOpts(hs, None, 0, flags)
        N.check(L.pgx_execute_async(ctx.handle, q.handle, seg_arr, len(segs), binds, C.byref(opts), C.byref(r)))
        return r

    def complete(i, r):
        """Finish step i: wait, then the combine output (trimToSize, kept groups read back) or the cross-GPU merge."""
        N.check(L.pgx_result_wait(r, -1))
        if dense:
            d = dense_t[i % inflight]
            st = (C.c_int64 * 4)()
            N.check(L.pgx_result_stats(r, st))
            L.pgx_result_release(r)
            multigpu.merge_dense_planes(d, plane_ops)
            stats_t = torch.tensor(list(st), dtype=torch.int64, device=d.device)
            torch.distributed.all_reduce(stats_t)
            out = C.c_void_p()
            s4 = (C.c_int64 * 4)(*stats_t.tolist())
            N.check(L.pgx_result_from_dense(ctx.handle, q.handle, seg_arr, len(segs), C.c_void_p(d.data_ptr()), s4,
                                            C.byref(out)))
            E.trim_and_gather(q, out)
            return out
        if req.get("group_by") and world > 1:  # sparse keys
            dev = "cuda:%d" % local
            n = C.c_int64()
            resident = L.pgx_result_device_groups(r, C.byref(n), None) == 0
            flag = torch.tensor([int(resident)], dtype=torch.int64, device=dev)
            torch.distributed.all_reduce(flag, op=torch.distributed.ReduceOp.MIN)
            if flag.item():  # one key space, groups in HBM: all-to-all by key hash + device merge + device trim
                maps, _total, _st = multigpu.device_sparse_merge(ctx, q, r, segs, dev)
                if rank == 0:
                    merged[0] = maps
            else:  # groups not device-resident (global hash table): host merge of every rank's groups by VALUE
                fns = [a["fn"] for a in req["aggregations"]]
                parts = multigpu.gather_group_partials(*E.group_partials(q, r, segs))
                if rank == 0:
                    cols, vals, cnts = multigpu.merge_group_partials(fns, parts)
                    kept = multigpu.trim_to_size(fns, vals, cnts, req["group_by"].get("top_n", 10))
                    merged[0] = E.render_group_maps(q, segs, cols, vals, cnts, kept)
        elif req.get("group_by"):  # the server's combine output: trimToSize, kept groups read back (a-19)
            E.trim_and_gather(q, r)
        if world > 1 and not req.get("group_by"):  # aggregation-only: combine the scalar partials across GPUs
            vals = []
            for k in range(len(req["aggregations"])):
                v, c = C.c_double(), C.c_int64()
                N.check(L.pgx_result_agg(r, k, C.byref(v), C.byref(c)))
                vals.append((v.value, c.value))
            merged[0] = multigpu.merge_aggregation([a["fn"] for a in req["aggregations"]], vals,
                                                   device="cuda:%d" % local)
        return r

    def run_steps(k, keep_last=False):
        """k steps with up to `inflight` queries in flight; returns the last step's result when keep_last."""
        pending = [submit(i) for i in range(min(inflight, k))]
        last = None
        for i in range(k):
            r = complete(i, pending.pop(0))
            if i + inflight < k:
                pending.append(submit(i + inflight))
            if keep_last and i == k - 1:
                last = r
            else:
                L.pgx_result_release(r)
        return last

    def step():  # one query, nothing in flight beside it (latency; tools): the batched plan
        nonlocal inflight
        saved, inflight = inflight, 1
        try:
            return complete(0, submit(0))
        finally:
            inflight = saved

    if args.profile_iters:  # exactly K steps and nothing else (PMC passes divide the step kernels' counters by K)
        run_steps(args.profile_iters)
        barrier_sync(world)
        if rank == 0:
            print(json.dumps({"profile_steps": args.profile_iters}))
        return

    run_steps(args.warmup)
    barrier_sync(world)
    # one-query-at-a-time latency, untimed for the line's value: single steps after two lone warm-ups (a lone query
    # plans afresh, then keeps its plan: the plan cache's replay is what a server repeating a query shape sees); the
    # latency-bound workloads (C1, C4) take more samples
    t_lat = []
    n_lat = 15 if args.workload in ("c1", "c4") else 3
    for k in range(2 + n_lat):
        t1 = time.perf_counter()
        L.pgx_result_release(step())
        if k >= 2:
            t_lat.append(time.perf_counter() - t1)
    barrier_sync(world)
    prof = None
    if os.environ.get("PGX_BENCH_CPROFILE"):  # host-overhead hunting: Python profile of the timed steps (not for lines)
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    t0 = time.perf_counter()
    last = run_steps(args.steps, keep_last=True)
    barrier_sync(world)
    elapsed = time.perf_counter() - t0
    if prof is not None:
        prof.disable()
        prof.dump_stats(os.environ["PGX_BENCH_CPROFILE"])
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda:%d" % local)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()

    # result summary (for the log) and kernel roofline on rank 0
    st = (C.c_int64 * 4)()
    N.check(L.pgx_result_stats(last, st))
    summary = None
    ngroups = 0
    if rank == 0:
        if req.get("group_by"):  # do not read a sparse result back whole: group count + the top of the trim
            ng = C.c_int64()
            N.check(L.pgx_result_num_groups(last, C.byref(ng)))
            ngroups = ng.value
            top = E.trimmed_maps(q, last, segs)[0]
            best = sorted(top.items(), key=lambda kv: kv[1], reverse=q.fns[0] != "min")[:3]
            summary = {"groups": ngroups, "top3_" + q.fns[0]: best}
        else:
            summary = E.decode_result(q, last, segs).get_aggregation_result()
    L.pgx_result_release(last)
    total_rows = rows * (wl.segments * world if wl.scaling == "weak" else wl.segments)
    value = total_rows / (elapsed / args.steps)

    # Kernel time of the SAME step (same plans, batches and streams): every library launch of a few more steps is
    # bracketed by HIP events on its own stream; the union of the busy intervals is the GPU time a step costs
    # (pgx_timing_start / pgx_timing_stop).  Run after the timed loop so the events do not perturb it.
    timing_steps = 5
    tout = (C.c_double * 3)()
    tjson = C.create_string_buffer(8192)
    N.check(L.pgx_timing_start(ctx.handle))
    run_steps(timing_steps)
    N.check(L.pgx_timing_stop(ctx.handle, tout, tjson, len(tjson)))
    step_kernels = json.loads(tjson.value.decode())
    kernel_ms = tout[0] / timing_steps
    if rank != 0:
        return
    # forward-index bytes of every column the kernel decodes, serialized roaring bytes of every bitmap a
    # bitmap-index leaf ORs (inverted columns, non-RANGE predicates: FilterPlanNode.java:118-132), dictionaries.
    bitmap_leaves = [(lf, np.nonzero(E.leaf_matching_ids(segs[0].column(lf["column"]), lf))[0])
                     for lf in q.leaves if wl.name != "c4" and data.is_inverted(lf["column"]) and lf["op"] != "RANGE"]
    scan_cols = {lf["column"] for lf in q.leaves} - {lf["column"] for lf, _ in bitmap_leaves}
    used = sorted(scan_cols | {a["column"] for a in req["aggregations"] if a["column"] != "*"}
                  | set((req.get("group_by") or {}).get("columns", [])))
    dict_cols = sorted({a["column"] for a in req["aggregations"] if a["column"] != "*"})
    if wl.name == "c4":
        from pinot_amd import startree as ST
        algo_bytes = data.algorithmic_bytes(used, dict_cols, int(st[0]), len(ST.parse(data.seg_data.star_tree)[1]))
    else:
        algo_bytes = data.algorithmic_bytes(used, dict_cols, bitmap_leaves)
    # + output_bytes of the final partial table: key + one 8-byte value per function per group
    algo_bytes += ngroups * 8 * (1 + len(req["aggregations"]))
    # every kernel of the step: the query-specialised kernels (hiprtc, pgx_jit.cpp; PGX_JIT=0 selects the generic
    # interpreter kernel), bitmap programs, partition / aggregation / trim kernels -- busy union per step
    kernel_name = "all kernels of the step (busy union): " + ", ".join(
        "%s x%d" % (k, v[0] // timing_steps) for k, v in sorted(step_kernels["kernels"].items()))
    ms_step = 1e3 * elapsed / args.steps
    achieved = algo_bytes / (kernel_ms * 1e-3) / 1e9
    traffic = None
    tf = os.path.join(ROOT, "profiles", "traffic_%s.json" % wl.name)
    if os.path.exists(tf) and not args.no_partition:  # (the traffic files are the default execution's)
        tj = json.load(open(tf))
        # PMC FETCH/WRITE of the same command (tools/profile_wl.sh), valid only for the kernel sources it was measured
        # on: a stale file (sources changed since) reports null instead of an old number
        if tj.get("rows") == rows and tj.get("source_hash") == source_hash():
            traffic = tj.get("hbm_bytes_per_launch")
    cpu = None
    if world == 1 and not args.no_cpu_baseline and wl.name in CPU_SAMPLE:
        nseg, seg_rows = CPU_SAMPLE[wl.name]
        cpu = cpu_baseline(wl, req, min(rows, seg_rows), nseg, 8)
    elif world == 1 and not args.no_cpu_baseline and wl.name == "c1":
        cpu = cpu_baseline_c1(data)
    elif world == 1 and not args.no_cpu_baseline and wl.name == "c4":
        cpu = cpu_baseline_c4(data, req)
    if merged[0] is not None and req.get("group_by"):
        top = merged[0][0]
        best = sorted(top.items(), key=lambda kv: kv[1], reverse=q.fns[0] != "min")[:3]
        summary = {"local": summary, "merged_over_gpus": {"top3_" + q.fns[0]: best}}
    elif merged[0] is not None:
        summary = {"local": summary, "merged_over_gpus": merged[0]}
    line = {
        "metric": METRIC, "value": value, "unit": "rows/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": ms_step, "higher_is_better": True,
        "queries_in_flight": inflight, "single_query_ms": 1e3 * min(t_lat),
        "single_query_ms_median": 1e3 * sorted(t_lat)[len(t_lat) // 2],
        "scaling": wl.scaling, "vs_baseline": None, "dtype": "int64",
        "data": "synthetic: device-generated v1 fixed-bit segments (seed %d), dictionaries per SURVEY 8d" % wl.seed,
        "config": {"workload": wl.name + ": " + wl.description, "query": wl.query,
                   "rows_per_segment": rows, "segments": len(segs) * (world if wl.scaling == "weak" else 1),
                   "rows_total": total_rows, "parallelism": "dp%d (segment sharding)" % world,
                   **({"exec": "PGX_X_NO_PARTITION (global hash table)"} if args.no_partition else {})},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": kernel_name, "kernel_ms": kernel_ms, "algorithmic_bytes": algo_bytes,
                     # the same bytes over the whole step (host planning, copies and launch gaps included)
                     "achieved_per_step": algo_bytes / (ms_step * 1e-3) / 1e9,
                     "frac_per_step": algo_bytes / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS,
                     "kernel_sum_ms": tout[1] / timing_steps, "kernel_span_ms": tout[2] / timing_steps,
                     "gpu_idle_ms_per_step": ms_step - kernel_ms,
                     "kernels_per_step": {k: [v[0] / timing_steps, v[1] / timing_steps]
                                          for k, v in step_kernels["kernels"].items()}},
        "cpu_baseline": cpu,
        "result": summary, "stats": list(st), "gen_s": t_gen,
    }
    print(json.dumps(line))
    data.free()


if __name__ == "__main__":
    main()
