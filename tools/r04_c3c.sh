#!/bin/bash
# Round 4: narrow C3 path after the kernel rework: parity, one query at a time, three in flight.
set -o pipefail
mkdir -p gpurun_out/r04/c3c
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
step gpurun_out/r04/c3c/partition.log 600 $PT tests/test_gpu_partition.py -k "narrow or matches_oracle"
step gpurun_out/r04/c3c/configs.log 600 $PT tests/test_gpu_configs.py -k c3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
PGX_INFLIGHT=1 step gpurun_out/r04/c3c/prof1.log 300 rocprofv3 --kernel-trace --stats --output-format csv \
  -d gpurun_out/r04/c3c/prof1 -o c3 -- python3 bench.py --workload c3 --profile-iters 2
find gpurun_out/r04/c3c/prof1 -name "*kernel_stats.csv" -exec head -6 {} \; | cut -c1-160
step gpurun_out/r04/c3c/bench3.err 300 python -u bench.py --workload c3 --steps 10 --warmup 3 --no-cpu-baseline
python tools/bench_summary.py gpurun_out/r04/c3c/bench3.err
# host overhead of the latency-bound configs: library phases (PGX_HOST_PROFILE) and the Python profile of the steps
PGX_HOST_PROFILE=1 PGX_BENCH_CPROFILE=gpurun_out/r04/c3c/c1.prof step gpurun_out/r04/c3c/c1.err 300 python -u bench.py \
  --workload c1 --steps 200 --warmup 20 --no-cpu-baseline
python tools/bench_summary.py gpurun_out/r04/c3c/c1.err
grep "pgx host us" gpurun_out/r04/c3c/c1.err | tail -3 | cut -c1-300
python -c "
import pstats; pstats.Stats('gpurun_out/r04/c3c/c1.prof').sort_stats('tottime').print_stats(12)" | tail -20 | cut -c1-150
