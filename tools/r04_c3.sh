#!/bin/bash
# Round 4: narrow partitioned group-by on the GPU box: parity first (partition + C3 configs), then the C3 bench and a
# kernel-trace profile of it, then the other new parity tests.  A test FAILURE (rc 1) does not stop the script; a crash,
# abort or time limit does.
set -o pipefail
mkdir -p gpurun_out/r04/c3
T="timeout -k 10"
step() {  # step <log> <seconds> <cmd...>
  local log=$1 secs=$2; shift 2
  $T $secs "$@" > $log 2>&1
  local rc=$?
  echo "[step rc=$rc] $*" | cut -c1-200
  tail -3 $log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
PT="python -u -m pytest -v --timeout 300 --timeout-method thread"
step gpurun_out/r04/c3/partition.log 600 $PT tests/test_gpu_partition.py -k "narrow or matches_oracle"
step gpurun_out/r04/c3/configs.log 600 $PT tests/test_gpu_configs.py -k c3
step gpurun_out/r04/c3/bench.err 300 python -u bench.py --workload c3 --steps 10 --warmup 3 --no-cpu-baseline
grep '^{' gpurun_out/r04/c3/bench.err > gpurun_out/r04/c3/bench.json
python -c "
import json;d=json.loads(open('gpurun_out/r04/c3/bench.json').read().strip().splitlines()[-1])
print('ms_per_step', d['ms_per_step'], 'single', d['single_query_ms'], 'kernel_ms', d['roofline']['kernel_ms'])
print(json.dumps(d['roofline']['kernels_per_step']))"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step gpurun_out/r04/c3/prof.log 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04/c3/prof -o c3 -- python3 bench.py \
  --workload c3 --profile-iters 3
step gpurun_out/r04/new_tests.log 900 $PT tests/test_gpu_realtime.py tests/test_gpu_mv.py tests/test_gpu_bitmap.py \
  tests/test_gpu_dense_pack.py tests/test_gpu_c5_headline.py
grep -E "FAILED|passed|failed" gpurun_out/r04/new_tests.log | tail -15
