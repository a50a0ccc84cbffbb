#!/bin/bash
# Round 4: JIT hash group-by with plain-read fast paths: C7 parity + bench, forced-hash parity.
set -o pipefail
O=gpurun_out/r04/c7b
mkdir -p $O/dump
T="timeout -k 10"
PT="python -u -m pytest -v --timeout 300 --timeout-method thread"
$T 900 $PT tests/test_gpu_configs.py tests/test_gpu_parity.py > $O/tests.log 2>&1
rc=$?; echo "[tests rc=$rc]"; tail -1 $O/tests.log; grep -E "FAILED|Error" $O/tests.log | head -8; [ $rc -ne 0 ] && exit $rc
PGX_JIT_DUMP=$O/dump $T 300 python -u bench.py --workload c7 --steps 10 --warmup 2 --no-cpu-baseline > $O/c7.err 2>&1
echo "[c7 rc=$?] $(python tools/bench_summary.py $O/c7.err)"
