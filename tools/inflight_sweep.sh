#!/bin/bash
# Queries-in-flight sweep of bench.py (run via gpurun from the repo root): one summary line per (workload, depth).
#   usage: tools/inflight_sweep.sh <out> "<workloads>" "<depths>" [bench args...]
set -o pipefail
O=gpurun_out/$1; WLS=$2; DEPTHS=$3; shift 3
mkdir -p $O
for w in $WLS; do
  for d in $DEPTHS; do
    PGX_INFLIGHT=$d timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline "$@" > $O/${w}_if$d.err 2>&1
    rc=$?; echo "[$w inflight=$d rc=$rc] $(python tools/bench_summary.py $O/${w}_if$d.err | tr "\n" " " | cut -c1-120)"
    [ $rc -ne 0 ] && { tail -5 $O/${w}_if$d.err; exit $rc; }
  done
done
exit 0
