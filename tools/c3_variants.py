"""GPU experiment harness (not a test): C3-shaped group-by queries over the C3 segments (8 x 125M rows) via
pgx_execute_timed, one query per process (run under rocprofv3 for per-kernel times).
usage: VARIANT_QUERY=<name> python tools/c3_variants.py [segments]"""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from pinot_amd import engine as E  # noqa: E402
from pinot_amd import native as N  # noqa: E402
from pinot_amd import pql, synth  # noqa: E402

QUERIES = {"full": "SELECT SUM(m), MIN(m), MAX(m) FROM T GROUP BY g1, g2 TOP 10",
           "sum": "SELECT SUM(m) FROM T GROUP BY g1, g2 TOP 10",
           "count": "SELECT COUNT(*) FROM T GROUP BY g1, g2 TOP 10",
           "minmax": "SELECT MIN(m), MAX(m) FROM T GROUP BY g1, g2 TOP 10"}


def main():
    nseg = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    ctx = E.Context(0)
    wl = synth.WORKLOADS["c3"]
    data = synth.DeviceSegments(ctx, wl, list(range(nseg)))
    segs = data.segments
    arr = (C.c_void_p * len(segs))(*[s.handle.value for s in segs])
    L = N.lib()
    name = os.environ.get("VARIANT_QUERY", "full")
    q = E._Query(ctx, pql.compile(QUERIES[name]))
    binds, keep = q.bindings(segs)
    tot, kern = C.c_double(), C.c_double()
    N.check(L.pgx_execute_timed(ctx.handle, q.handle, arr, len(segs), binds, 3, C.byref(tot), C.byref(kern), None))
    print(json.dumps({"query": name, "segments": nseg, "kernel_ms": round(kern.value, 4), "total_ms": round(tot.value, 4)}),
          flush=True)
    data.free()
    ctx.close()


if __name__ == "__main__":
    main()
