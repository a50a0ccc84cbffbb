"""Per-step GPU timeline from a rocprofv3 kernel trace (not a test).

usage: python tools/timeline.py <kernel_trace.csv> [gap_ms] [regex]

Kernels matching `regex` (default: the query path's pgxq / bitmap programs / partition kernels) are split into steps at
host gaps longer than `gap_ms`; per step it prints the span (first start -> last end), the union of busy intervals,
the summed kernel time, and per kernel name the launch count and summed duration.  The union is the GPU time a step
really costs; span - union is time the GPU idled inside the step (host planning, copies, launch latency)."""
import csv
import json
import re
import sys


def load(path, rx):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name") or r.get("KernelName") or ""
            if not re.search(rx, name):
                continue
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name.split("(")[0]))
    rows.sort()
    return rows


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    path = sys.argv[1]
    gap = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    rx = sys.argv[3] if len(sys.argv) > 3 else r"pgxq|pgx_roaring|pgx_part|pgx_partition|pgx_init|pgx_compact"
    rows = load(path, rx)
    steps, cur = [], []
    for r in rows:
        if cur and r[0] - max(e for _, e, _ in cur) > gap * 1e6:
            steps.append(cur)
            cur = []
        cur.append(r)
    if cur:
        steps.append(cur)
    for i, st in enumerate(steps):
        span = max(e for _, e, _ in st) - min(s for s, _, _ in st)
        per = {}
        for s, e, n in st:
            c, d = per.get(n, (0, 0))
            per[n] = (c + 1, d + e - s)
        print(json.dumps({"step": i, "span_ms": round(span / 1e6, 3), "busy_ms": round(union([(s, e) for s, e, _ in st]) / 1e6, 3),
                          "sum_ms": round(sum(e - s for s, e, _ in st) / 1e6, 3),
                          "kernels": {n: [c, round(d / 1e6, 3)] for n, (c, d) in per.items()}}))


if __name__ == "__main__":
    main()
