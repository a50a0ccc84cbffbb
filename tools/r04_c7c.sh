#!/bin/bash
# Round 4: batched hash lookups in the generated kernels: parity (configs, parity, partition fallbacks, MV), C7 A/B.
set -o pipefail
O=gpurun_out/r04/c7c
mkdir -p $O
T="timeout -k 10"
PT="python -u -m pytest -v --timeout 300 --timeout-method thread"
$T 900 $PT tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_partition.py tests/test_gpu_mv.py > $O/tests.log 2>&1
rc=$?; echo "[tests rc=$rc]"; tail -1 $O/tests.log; grep -E "FAILED|Error" $O/tests.log | head -8; [ $rc -ne 0 ] && exit $rc
for v in "PGX_HASH_BATCH=1" "PGX_HASH_BATCH=0"; do
  env $v $T 300 python -u bench.py --workload c7 --steps 10 --warmup 2 --no-cpu-baseline > $O/c7.err 2>&1
  echo "[c7 $v rc=$?] $(python tools/bench_summary.py $O/c7.err | head -1)"
done
