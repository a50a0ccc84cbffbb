#!/bin/bash
# Round 4: uniform segment pointers + carried tile base in the generated kernels: parity, then C7/C5/C6/C3/C2/C1 lines.
set -o pipefail
O=gpurun_out/r04/sg
mkdir -p $O/dump
T="timeout -k 10"
PT="python -u -m pytest -v --timeout 300 --timeout-method thread"
$T 900 $PT tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_c5_headline.py > $O/tests.log 2>&1
rc=$?; echo "[tests rc=$rc]"; tail -1 $O/tests.log; grep -E "FAILED|Error" $O/tests.log | head -8; [ $rc -ne 0 ] && exit $rc
PGX_JIT_DUMP=$O/dump $T 300 python -u bench.py --workload c7 --steps 10 --warmup 2 --no-cpu-baseline > $O/c7.err 2>&1
rc=$?; echo "[c7 rc=$rc] $(python tools/bench_summary.py $O/c7.err)"; [ $rc -ne 0 ] && exit $rc
for w in c5 c6 c3 c2 c1; do
  $T 300 python -u bench.py --workload $w --no-cpu-baseline > $O/$w.err 2>&1
  rc=$?; echo "[$w rc=$rc] $(python tools/bench_summary.py $O/$w.err)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
