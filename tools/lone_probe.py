"""Lone-query timeline of a bench workload: N one-at-a-time queries (the plan cache's replay after two warm-ups,
as bench.py's single_query_ms), wall time per call; run under `rocprofv3 --kernel-trace` for the kernels' timeline
and with PGX_DEBUG=host_profile for the library's host marks.
    python tools/lone_probe.py --workload c5 [--n 8] [--flags 0]"""
import argparse
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c5")
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--flags", type=int, default=0)
    args = ap.parse_args()
    import torch
    from pinot_amd import engine as E
    from pinot_amd import multigpu, pql, synth
    from pinot_amd import native as N
    ctx = E.Context(0)
    wl = synth.WORKLOADS[args.workload]
    data = synth.DeviceSegments(ctx, wl, multigpu.shard(wl.segments, 1, 0, wl.scaling), rows=wl.rows)
    req = pql.compile(wl.query)
    q = E._Query(ctx, req)
    segs = data.segments
    seg_arr = (C.c_void_p * len(segs))(*[s.handle.value for s in segs])
    L = N.lib()
    stream = torch.cuda.Stream(device="cuda:0")

    def one():
        binds, _owner = q.bindings(segs, seg_arr)
        r = C.c_void_p()
        opts = N.ExecOpts(stream.cuda_stream, None, 0, args.flags)
        N.check(L.pgx_execute_async(ctx.handle, q.handle, seg_arr, len(segs), binds, C.byref(opts), C.byref(r)))
        N.check(L.pgx_result_wait(r, -1))
        if req.get("group_by"):
            E.trim_and_gather(q, r)
        L.pgx_result_release(r)

    for k in range(2 + args.n):
        t = time.perf_counter()
        one()
        print("call %d: %.3f ms" % (k, 1e3 * (time.perf_counter() - t)), flush=True)


if __name__ == "__main__":
    main()
