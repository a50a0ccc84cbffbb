"""Summarise a rocprofv3 counter_collection.csv: per kernel (name prefix), the mean of every counter per dispatch.
usage: python tools/pmc_summary.py <counter_collection.csv> [kernel-substring ...]"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    want = sys.argv[2:]
    acc = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(path)):
        name = r.get("Kernel_Name") or r.get("Kernel-Name") or ""
        if want and not any(w in name for w in want):
            continue
        key = (name[:60], r.get("Dispatch_Id") or r.get("Dispatch-Id"))
        acc[name[:60]][(key[1], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for k, d in acc.items():
        per = defaultdict(list)
        for (disp, cn), vals in d.items():
            per[cn].append(sum(vals))
        print(k)
        for cn in sorted(per):
            v = per[cn]
            print("  %-24s %16.4g  (n=%d)" % (cn, sum(v) / len(v), len(v)))


if __name__ == "__main__":
    main()
