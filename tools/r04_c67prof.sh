#!/bin/bash
# Round 4 end: kernel trace + PMC traffic for C6 and C7 on the final sources, then their bench lines with traffic.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for w in "c6 10" "c7 10"; do
  set -- $w
  timeout -k 10 420 bash tools/profile_wl.sh $1 $2 --no-cpu-baseline > gpurun_out/final_$1.log 2>&1
  rc=$?; echo "[profile $1 rc=$rc]"; tail -2 gpurun_out/final_$1.log | cut -c1-300
  [ $rc -ne 0 ] && exit $rc
  cp gpurun_out/prof_$1/traffic_$1.json profiles/traffic_$1.json
done
O=gpurun_out/r04/benches
mkdir -p $O
for w in c6 c7; do
  timeout -k 10 400 python -u bench.py --workload $w > $O/$w.err 2>&1
  rc=$?; echo "[$w rc=$rc]"; python tools/bench_summary.py $O/$w.err
  grep '^{' $O/$w.err | tail -1 > $O/${w}_bench.json
  [ $rc -ne 0 ] && exit $rc
done
exit 0
