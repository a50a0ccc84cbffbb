"""GPU experiment harness (not a test): where one C5 bench step's wall time goes.  Times the step's parts separately
(pgx_bind_predicates, pgx_execute, trim + gather) and pgx_execute_timed's wall vs summed kernel time.
usage: python tools/c5_breakdown.py [segments] [steps]"""
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from pinot_amd import engine as E  # noqa: E402
from pinot_amd import native as N  # noqa: E402
from pinot_amd import pql, synth  # noqa: E402


def main():
    nseg = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    ctx = E.Context(0)
    wl = synth.WORKLOADS["c5"]
    data = synth.DeviceSegments(ctx, wl, list(range(nseg)))
    segs = data.segments
    arr = (C.c_void_p * len(segs))(*[s.handle.value for s in segs])
    L = N.lib()
    q = E._Query(ctx, pql.compile(wl.query))
    for bs in os.environ.get("BREAKDOWN_BATCH", "512").split(","):
        os.environ["PGX_BATCH_SEGS"] = bs
        run(ctx, q, segs, arr, L, nseg, steps, bs)
    data.free()
    ctx.close()


def run(ctx, q, segs, arr, L, nseg, steps, bs):
    parts = {"bind": 0.0, "execute": 0.0, "trim": 0.0, "release": 0.0}
    for i in range(steps + 3):
        t0 = time.perf_counter()
        binds, _own = q.bindings(segs, arr)
        t1 = time.perf_counter()
        r = C.c_void_p()
        opts = N.ExecOpts(0, None, 0, 0)
        N.check(L.pgx_execute(ctx.handle, q.handle, arr, len(segs), binds, C.byref(opts), C.byref(r)))
        t2 = time.perf_counter()
        E.trim_and_gather(q, r)
        t3 = time.perf_counter()
        L.pgx_result_release(r)
        del _own
        t4 = time.perf_counter()
        if i >= 3:
            for k, d in zip(parts, (t1 - t0, t2 - t1, t3 - t2, t4 - t3)):
                parts[k] += d * 1e3 / steps
    binds, keep = q.bindings(segs)
    tot, kern = C.c_double(), C.c_double()
    N.check(L.pgx_execute_timed(ctx.handle, q.handle, arr, len(segs), binds, 10, C.byref(tot), C.byref(kern), None))
    print(json.dumps({"segments": nseg, "batch_segs": bs, "step_parts_ms": {k: round(v, 3) for k, v in parts.items()},
                      "step_ms": round(sum(parts.values()), 3), "timed_total_ms": round(tot.value, 3),
                      "timed_kernel_ms": round(kern.value, 3)}), flush=True)


if __name__ == "__main__":
    main()
