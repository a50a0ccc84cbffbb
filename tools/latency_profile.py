"""Where a lone query's time goes on the host (C1 / C4 single_query_ms): cProfile of N one-at-a-time steps of
bench.py's own submit / complete path, plus the library's host-phase marks (PGX_DEBUG=host_profile).
    python tools/latency_profile.py --workload c1 [--n 200]"""
import argparse
import cProfile
import ctypes as C
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c1")
    ap.add_argument("--n", type=int, default=200)
    args = ap.parse_args()
    from pinot_amd import engine as E
    from pinot_amd import native as N
    from pinot_amd import pql, synth
    ctx = E.Context(0)
    data = synth.BaseballSegments(ctx) if args.workload == "c1" else synth.StarTreeSegments(ctx)
    req = pql.compile(synth.C1_QUERY if args.workload == "c1" else synth.C4_QUERY)
    q = E._Query(ctx, req)
    segs = data.segments
    seg_arr = (C.c_void_p * len(segs))(*[s.handle.value for s in segs])
    L = N.lib()

    def one():
        binds, _owner = q.bindings(segs, seg_arr)
        r = C.c_void_p()
        opts = N.ExecOpts(0, None, 0, 0)
        N.check(L.pgx_execute_async(ctx.handle, q.handle, seg_arr, len(segs), binds, C.byref(opts), C.byref(r)))
        N.check(L.pgx_result_wait(r, -1))
        E.trim_and_gather(q, r)
        L.pgx_result_release(r)

    for _ in range(20):
        one()
    ts = []
    for _ in range(args.n):
        t = time.perf_counter()
        one()
        ts.append(time.perf_counter() - t)
    ts.sort()
    print("lone query ms: min %.4f median %.4f" % (1e3 * ts[0], 1e3 * ts[len(ts) // 2]))
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(args.n):
        one()
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(18)


if __name__ == "__main__":
    main()
