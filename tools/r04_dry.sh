#!/bin/bash
# Round 4 experiment (temporary knobs): narrow C3 kernel times with the scan's / split's record stores skipped.
set -o pipefail
O=gpurun_out/r04/dry
mkdir -p $O
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
prof() {  # prof <name> <env...>
  local name=$1; shift
  env "$@" PGX_INFLIGHT=1 $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$name -o c3 -- \
    python3 bench.py --workload c3 --profile-iters 2 > $O/$name.log 2>&1
  local rc=$?
  echo "[prof $name rc=$rc]"
  if [ $rc -ne 0 ]; then tail -3 $O/$name.log; exit $rc; fi
  awk -F'",' 'NR>1 {split($1,a,"("); n=a[1]; gsub(/"/,"",n); split($2,b,","); printf "  %-50.50s calls=%s avg_us=%.1f\n", n, b[1], b[3]/1000}' $O/$name/c3_kernel_stats.csv | head -8
}
prof base PGX_NARROW_DRY=0
prof dry1 PGX_NARROW_DRY=1
prof dry2 PGX_NARROW_DRY=2
