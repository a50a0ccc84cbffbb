#!/bin/bash
# Round 4 final profiles on the frozen kernel sources: for C5, C3 and C2 a kernel trace of the bench (three queries in
# flight) with its per-step busy union, and per-step PMC FETCH / WRITE traffic (tools/profile_wl.sh).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for w in "c5 10" "c3 5" "c2 10"; do
  set -- $w
  timeout -k 10 420 bash tools/profile_wl.sh $1 $2 > gpurun_out/final_$1.log 2>&1
  rc=$?; echo "[profile $1 rc=$rc]"; tail -2 gpurun_out/final_$1.log | cut -c1-300
  [ $rc -ne 0 ] && exit $rc
  python3 tools/bench_summary.py gpurun_out/prof_$1/bench.json
done
