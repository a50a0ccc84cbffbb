#!/bin/bash
# Round 4 experiment (temporary knob PGX_NA_DBG, results void): narrow aggregation time with parts knocked out
# (1: no table atomics, 2: misses dropped, 4: no group output), C3 one query at a time under rocprofv3.
set -o pipefail
O=gpurun_out/r04/agg_ko
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for d in 0 1 2 4 7; do
  PGX_NA_DBG=$d PGX_INFLIGHT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/d$d -o c3 -- \
    python3 bench.py --workload c3 --profile-iters 2 --no-cpu-baseline > $O/d$d.log 2>&1
  echo "[dbg $d rc=$?] $(awk -F'",' 'NR>1 && /narrow_aggregate/ {split($2,b,","); printf "agg_us=%.1f calls=%s", b[3]/1000, b[1]}' $O/d$d/c3_kernel_stats.csv)"
done
