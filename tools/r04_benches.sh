#!/bin/bash
# Round 4 end: one bench line per workload (N = 1, CPU baselines included) on the final sources.
set -o pipefail
O=gpurun_out/r04/benches
mkdir -p $O
for w in c5 c1 c2 c3 c4 c6 c7; do
  timeout -k 10 400 python -u bench.py --workload $w > $O/$w.err 2>&1
  rc=$?; echo "[$w rc=$rc]"; python tools/bench_summary.py $O/$w.err
  grep '^{' $O/$w.err | tail -1 > $O/${w}_bench.json
  [ $rc -ne 0 ] && exit $rc
done
