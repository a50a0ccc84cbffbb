#!/bin/bash
# Round 4: narrow C3 path, one query at a time (clean kernel times) and three in flight; plus the fixed parity tests.
set -o pipefail
mkdir -p gpurun_out/r04/c3b
T="timeout -k 10"
step() {  # step <log> <seconds> <cmd...>
  local log=$1 secs=$2; shift 2
  $T $secs "$@" > $log 2>&1
  local rc=$?
  echo "[step rc=$rc] $*" | cut -c1-160
  tail -2 $log | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
PT="python -u -m pytest -v --timeout 300 --timeout-method thread"
step gpurun_out/r04/c3b/partition.log 600 $PT tests/test_gpu_partition.py -k "narrow"
export PGX_NARROW_DEBUG=1
PGX_INFLIGHT=1 step gpurun_out/r04/c3b/bench1.err 300 python -u bench.py --workload c3 --steps 5 --warmup 2 --no-cpu-baseline
grep "pgx narrow" gpurun_out/r04/c3b/bench1.err | tail -2
python tools/bench_summary.py gpurun_out/r04/c3b/bench1.err
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
PGX_INFLIGHT=1 step gpurun_out/r04/c3b/prof1.log 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d gpurun_out/r04/c3b/prof1 -o c3 -- python3 bench.py --workload c3 --profile-iters 2
find gpurun_out/r04/c3b/prof1 -name "*kernel_stats.csv" -exec head -12 {} \;
unset PGX_NARROW_DEBUG
step gpurun_out/r04/c3b/bench3.err 300 python -u bench.py --workload c3 --steps 10 --warmup 3 --no-cpu-baseline
python tools/bench_summary.py gpurun_out/r04/c3b/bench3.err
step gpurun_out/r04/c3b/tests.log 900 $PT tests/test_gpu_mv.py tests/test_gpu_dense_pack.py tests/test_gpu_c5_headline.py
grep -E "FAILED|passed|failed" gpurun_out/r04/c3b/tests.log | tail -8
