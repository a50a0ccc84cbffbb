"""Turn a rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE counter CSV into profiles/traffic_<workload>.json.

gfx950 corrections (/opt/skills/guides/MI355X_MICROARCH.md, HBM section): FETCH_SIZE is in KiB and reports exactly half
of the bytes of a wide coalesced streaming read, so read bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE is exact.
usage: python tools/pmc_traffic.py <fetch.csv>[,<write.csv>] <kernel-substring> <workload> <rows> [out.json] [steps]

With `steps` (the counter passes ran `bench.py --profile-iters <steps>`: exactly that many bench steps), every dispatch
of the named kernels is summed and divided by the step count: the HBM bytes one STEP moves, whatever its batching.
The file is stamped with bench.source_hash(): bench.py reports it only while the kernel sources are unchanged.
"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import source_hash  # noqa: E402


def main():
    path, kname, workload, rows = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
    out = sys.argv[5] if len(sys.argv) > 5 and sys.argv[5] else "profiles/traffic_%s.json" % workload
    steps = int(sys.argv[6]) if len(sys.argv) > 6 else 0
    knames = kname.split("+")  # several kernels per query (e.g. pgx_roaring_program+pgxq): bytes summed per query
    rows_all = []
    for p in path.split(","):
        rows_all += list(csv.DictReader(open(p)))
    per = {k: ({}, {}) for k in knames}
    for r in rows_all:
        name_k = r.get("Kernel_Name", "")
        ks = [k for k in knames if k in name_k]
        if not ks:
            continue
        fetch, write = per[ks[0]]
        d = r.get("Dispatch_Id") or r.get("Correlation_Id")
        name = r.get("Counter_Name")
        v = float(r.get("Counter_Value", 0))
        if name == "FETCH_SIZE":
            fetch[d] = fetch.get(d, 0.0) + v
        elif name == "WRITE_SIZE":
            write[d] = write.get(d, 0.0) + v
    if not any(f or w for f, w in per.values()):
        sys.exit("no %s dispatches in %s" % (kname, path))
    med = lambda xs: sorted(xs)[len(xs) // 2] if xs else 0.0
    f0, w0 = per[knames[0]]
    nq = max(len(f0), len(w0), 1)
    breakdown = {}
    total = 0.0
    for k in knames:
        f, w = per[k]
        # launches of this kernel per query (C3's pgx_partition runs twice), relative to the first kernel's count
        per_q = max(1, round(max(len(f), len(w)) / nq))
        b = (2 * med(list(f.values())) * 1024 + med(list(w.values())) * 1024) * per_q
        breakdown[k] = {"dispatches": max(len(f), len(w)), "launches_per_query": per_q, "hbm_bytes_per_query": b}
        total += b
    if steps:  # per step: every dispatch summed (batched steps launch each kernel several times)
        breakdown, total = {}, 0.0
        for k in knames:
            f, w = per[k]
            b = (2 * sum(f.values()) * 1024 + sum(w.values()) * 1024) / steps
            breakdown[k] = {"dispatches": max(len(f), len(w)), "launches_per_step": max(len(f), len(w)) / steps,
                            "hbm_bytes_per_step": b}
            total += b
    res = {"workload": workload, "rows": rows, "kernel": kname, "dispatches": nq, "steps": steps or None,
           "source_hash": source_hash(),
           "fetch_size_kib_median": med(list(f0.values())), "write_size_kib_median": med(list(w0.values())),
           "hbm_bytes_per_launch": total, "per_kernel": breakdown,
           "correction": "read bytes = 2 x FETCH_SIZE x 1024 (gfx950 half-count), write bytes = WRITE_SIZE x 1024"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
