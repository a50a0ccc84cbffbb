"""Reconcile the bench line's HIP-event kernel timing with rocprofv3's kernel trace of the same run (not a test).

usage: python tools/reconcile.py <kernel_trace.csv> <bench.json> [out.json]

bench.py's line times its last `timing_steps` (5) steps with HIP events on each launch's own stream
(pgx_timing_start / stop, kernels_per_step: launches and summed ms per step).  Those launches are the LAST ones of the
run, so the trace's last 5 x launches_per_step launches of each kernel are the same launches: their mean rocprof
duration is compared with the line's per-launch mean."""
import csv
import json
import sys


def main():
    trace, bench = sys.argv[1], sys.argv[2]
    line = json.loads(open(bench).read().strip().splitlines()[-1])
    kps = line["roofline"]["kernels_per_step"]
    steps = 5
    rows = {}
    with open(trace) as f:
        for r in csv.DictReader(f):
            name = (r.get("Kernel_Name") or "").replace("(anonymous namespace)::", "")
            name = name.split("(")[0].split("<")[0].replace("void ", "").strip()
            name = name.split("::")[-1]
            rows.setdefault(name, []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    out = {"kernel_ms_busy_union_per_step": line["roofline"]["kernel_ms"], "kernels": {}}
    for k, (launches, ms) in kps.items():
        n = int(round(launches * steps))
        tr = sorted(rows.get(k, []))[-n:] if n else []
        if not tr:
            continue
        rocprof_ms = sum(e - s for s, e in tr) / len(tr) / 1e6
        event_ms = ms / launches
        out["kernels"][k] = {"launches_compared": len(tr), "hip_event_ms_per_launch": round(event_ms, 4),
                             "rocprof_ms_per_launch": round(rocprof_ms, 4),
                             "ratio": round(rocprof_ms / event_ms, 4) if event_ms else None}
    js = json.dumps(out, indent=1)
    print(js)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(js)


if __name__ == "__main__":
    main()
