#!/bin/bash
# Round 4: hash group-by in the generated kernels: C7 (ARRAY_MAP keys) parity + bench, hash-path parity suites
# (forced hash, partition fallbacks, MV), interpreter A/B (PGX_JIT_HASH=0).
set -o pipefail
O=gpurun_out/r04/c7
mkdir -p $O
T="timeout -k 10"
PT="python -u -m pytest -v --timeout 300 --timeout-method thread"
$T 900 $PT tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_partition.py tests/test_gpu_mv.py tests/test_gpu_multi.py > $O/tests.log 2>&1
rc=$?; echo "[tests rc=$rc]"; tail -1 $O/tests.log; grep -E "FAILED|Error" $O/tests.log | head -8; [ $rc -ne 0 ] && exit $rc
$T 300 python -u bench.py --workload c7 --steps 10 --warmup 2 --no-cpu-baseline > $O/c7.err 2>&1
echo "[c7 rc=$?] $(python tools/bench_summary.py $O/c7.err)"
PGX_JIT_HASH=0 $T 300 python -u bench.py --workload c7 --steps 5 --warmup 1 --no-cpu-baseline > $O/c7i.err 2>&1
echo "[c7 interpreter rc=$?] $(python tools/bench_summary.py $O/c7i.err | head -1)"
