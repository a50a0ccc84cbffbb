#!/bin/bash
# Round 4: narrow scan-kernel shape A/B (threads, rows per lane, rows per lane per tile) on C3, one query at a time
# under rocprofv3 (kernel stats per variant), after a parity pass of the narrow tests with the first variant.
set -o pipefail
O=gpurun_out/r04/c3d
mkdir -p $O
T="timeout -k 10"
step() {  # step <log> <seconds> <cmd...>
  local log=$1 secs=$2; shift 2
  $T $secs "$@" > $log 2>&1
  local rc=$?
  echo "[step rc=$rc] $*" | cut -c1-160
  tail -2 $log | cut -c1-300
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
PT="python -u -m pytest -v --timeout 300 --timeout-method thread"
PGX_NARROW_T=1024 PGX_NARROW_R=8 PGX_NARROW_TL=16 step $O/partition.log 600 $PT tests/test_gpu_partition.py -k "narrow"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
prof() {  # prof <name> <env...>
  local name=$1; shift
  env "$@" PGX_INFLIGHT=1 $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$name -o c3 -- \
    python3 bench.py --workload c3 --profile-iters 2 > $O/$name.log 2>&1
  local rc=$?
  echo "[prof $name rc=$rc]"
  if [ $rc -ne 0 ]; then tail -3 $O/$name.log; exit $rc; fi
  find $O/$name -name "*kernel_stats.csv" -exec awk -F'","' 'NR>1 && NR<10 {printf "  %-40.40s %s\n", $1, $4}' {} \;
}
prof v0 PGX_NARROW_T=512
prof v1 PGX_NARROW_T=1024 PGX_NARROW_R=8 PGX_NARROW_TL=16
prof v1b PGX_NARROW_T=1024 PGX_NARROW_R=8
prof v3 PGX_NARROW_R=8 PGX_NARROW_TL=16
