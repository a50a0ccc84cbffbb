#!/bin/bash
# Round 4: narrow aggregation misses claim the empty way they saw (one LDS round trip): parity, C3 kernel stats.
set -o pipefail
O=gpurun_out/r04/c3m
mkdir -p $O
T="timeout -k 10"
PT="python -u -m pytest -v --timeout 300 --timeout-method thread"
$T 900 $PT tests/test_gpu_partition.py tests/test_gpu_configs.py -k "narrow or matches_oracle or c3" > $O/tests.log 2>&1
rc=$?; echo "[tests rc=$rc]"; tail -1 $O/tests.log; grep -E "FAILED|ERROR" $O/tests.log | head -5; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
PGX_INFLIGHT=1 $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof1 -o c3 -- \
  python3 bench.py --workload c3 --profile-iters 2 > $O/prof1.log 2>&1
rc=$?; echo "[prof1 rc=$rc]"; [ $rc -ne 0 ] && { tail -3 $O/prof1.log; exit $rc; }
awk -F'",' 'NR>1 {split($1,a,"("); n=a[1]; gsub(/"/,"",n); split($2,b,","); printf "  %-50.50s calls=%s avg_us=%.1f\n", n, b[1], b[3]/1000}' $O/prof1/c3_kernel_stats.csv | grep -v synth | head -5
