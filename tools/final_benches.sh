#!/bin/bash
# Round-end bench lines (N=1) for every BASELINE config and the extra shapes, with their CPU baselines:
# gpurun_out/final/<wl>_bench.json (+ .err)
set -euo pipefail
OUT=gpurun_out/final
mkdir -p $OUT
for wl in c5 c1 c2 c3 c4 c6 c7 c3d c3m2 c3f; do
  timeout -k 10 300 python bench.py --workload $wl > $OUT/${wl}_bench.json 2> $OUT/${wl}_bench.err
  echo "$wl done: $(python tools/bench_summary.py $OUT/${wl}_bench.json)"
done
