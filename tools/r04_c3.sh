#!/bin/bash
# Round 4: narrow partitioned group-by on the GPU box: parity first (partition + C3 configs), then the C3 bench and a
# kernel-trace profile of it, then the other new parity tests.
set -o pipefail
mkdir -p gpurun_out/r04/c3
T="timeout -k 10"
$T 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_partition.py \
  > gpurun_out/r04/c3/partition.log 2>&1 || { tail -40 gpurun_out/r04/c3/partition.log; exit 1; }
tail -3 gpurun_out/r04/c3/partition.log
$T 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_configs.py -k c3 \
  > gpurun_out/r04/c3/configs.log 2>&1 || { tail -40 gpurun_out/r04/c3/configs.log; exit 1; }
tail -3 gpurun_out/r04/c3/configs.log
$T 300 python -u bench.py --workload c3 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r04/c3/bench.json \
  2> gpurun_out/r04/c3/bench.err || { tail -20 gpurun_out/r04/c3/bench.err; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/r04/c3/bench.json').read().strip().splitlines()[-1])
print('ms_per_step', d['ms_per_step'], 'single', d['single_query_ms'], 'kernel_ms', d['roofline']['kernel_ms'])
print(json.dumps(d['roofline']['kernels_per_step']))"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04/c3/prof -o c3 -- python3 bench.py --workload c3 \
  --profile-iters 3 > gpurun_out/r04/c3/prof.log 2>&1 || { tail -20 gpurun_out/r04/c3/prof.log; exit 1; }
find gpurun_out/r04/c3/prof -name "*kernel_stats.csv" | head -3
$T 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_realtime.py tests/test_gpu_mv.py tests/test_gpu_bitmap.py tests/test_gpu_dense_pack.py \
  tests/test_gpu_c5_headline.py \
  > gpurun_out/r04/new_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r04/new_tests.log
exit $rc
