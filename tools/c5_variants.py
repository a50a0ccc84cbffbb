"""GPU experiment harness (not a test): kernel time of C5-shaped queries over a subset of the C5 segments under planner
variants (PGX_RCHUNK, PGX_BATCH_SEGS, ...), via pgx_execute_timed.  usage: python tools/c5_variants.py [segments]"""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from pinot_amd import engine as E  # noqa: E402
from pinot_amd import native as N  # noqa: E402
from pinot_amd import pql, synth  # noqa: E402


def main():
    nseg = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    ctx = E.Context(0)
    wl = synth.WORKLOADS["c5"]
    data = synth.DeviceSegments(ctx, wl, list(range(nseg)))
    segs = data.segments
    arr = (C.c_void_p * len(segs))(*[s.handle.value for s in segs])
    L = N.lib()
    f1 = wl.query[wl.query.index("f1 IN"):wl.query.index(") OR") + 1]
    queries = {"c5": wl.query,
               "c5_count": "SELECT COUNT(*) FROM T WHERE (%s OR f2 = 7) AND f3 <> 3 GROUP BY gk TOP 10" % f1,
               "c5_nogroup": "SELECT SUM(m) FROM T WHERE (%s OR f2 = 7) AND f3 <> 3" % f1,
               "scan_only": "SELECT SUM(m) FROM T GROUP BY gk TOP 10",
               "c2like": "SELECT COUNT(*), SUM(m) FROM T WHERE gk BETWEEN 0 AND 499",
               "c2like_f1": "SELECT COUNT(*), SUM(m) FROM T WHERE f1 BETWEEN 0 AND 499"}
    only = os.environ.get("VARIANT_QUERIES")
    if only:
        queries = {k: v for k, v in queries.items() if k in only.split(",")}
    variants = [("sep", {"PGX_RCHUNK": "0", "PGX_COMPACT": "0"}), ("sep+compact", {"PGX_RCHUNK": "0", "PGX_COMPACT": "1"}),
                ("rchunk", {"PGX_RCHUNK": "1", "PGX_COMPACT": "0"}),
                ("rchunk+compact", {"PGX_RCHUNK": "1", "PGX_COMPACT": "1"})]
    if os.environ.get("VARIANTS_JSON"):  # [[name, {env}], ...]
        variants = [tuple(v) for v in json.loads(os.environ["VARIANTS_JSON"])]
    for qn, text in queries.items():
        q = E._Query(ctx, pql.compile(text))
        binds, keep = q.bindings(segs)
        for vn, env in variants:
            os.environ.update(env)
            tot, kern = C.c_double(), C.c_double()
            N.check(L.pgx_execute_timed(ctx.handle, q.handle, arr, len(segs), binds, 5, C.byref(tot), C.byref(kern),
                                        None))
            print(json.dumps({"query": qn, "variant": vn, "segments": nseg, "kernel_ms": round(kern.value, 4)}),
                  flush=True)
    data.free()
    ctx.close()


if __name__ == "__main__":
    main()
