"""Turn a rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE counter CSV into profiles/traffic_<workload>.json.

gfx950 corrections (/opt/skills/guides/MI355X_MICROARCH.md, HBM section): FETCH_SIZE is in KiB and reports exactly half
of the bytes of a wide coalesced streaming read, so read bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE is exact.
usage: python tools/pmc_traffic.py <fetch.csv>[,<write.csv>] <kernel-substring> <workload> <rows> [out.json]
"""
import csv
import json
import sys


def main():
    path, kname, workload, rows = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
    out = sys.argv[5] if len(sys.argv) > 5 else "profiles/traffic_%s.json" % workload
    fetch, write = {}, {}
    rows_all = []
    for p in path.split(","):
        rows_all += list(csv.DictReader(open(p)))
    for r in rows_all:
        if kname not in r.get("Kernel_Name", ""):
            continue
        d = r.get("Dispatch_Id") or r.get("Correlation_Id")
        name = r.get("Counter_Name")
        v = float(r.get("Counter_Value", 0))
        if name == "FETCH_SIZE":
            fetch[d] = fetch.get(d, 0.0) + v
        elif name == "WRITE_SIZE":
            write[d] = write.get(d, 0.0) + v
    if not fetch and not write:
        sys.exit("no %s dispatches in %s" % (kname, path))
    f = sorted(fetch.values())
    w = sorted(write.values())
    med = lambda xs: xs[len(xs) // 2] if xs else 0.0
    res = {"workload": workload, "rows": rows, "kernel": kname, "dispatches": max(len(f), len(w)),
           "fetch_size_kib_median": med(f), "write_size_kib_median": med(w),
           "hbm_bytes_per_launch": 2 * med(f) * 1024 + med(w) * 1024,
           "correction": "read bytes = 2 x FETCH_SIZE x 1024 (gfx950 half-count), write bytes = WRITE_SIZE x 1024"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
