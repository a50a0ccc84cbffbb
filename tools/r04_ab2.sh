#!/bin/bash
# Round 4: LDS hash probing with plain reads (P) against compare-and-swap probing (B): hash parity, then C7 lines.
set -o pipefail
O=gpurun_out/r04/ab2
mkdir -p $O
T="timeout -k 10"
PT="python -u -m pytest -v --timeout 300 --timeout-method thread"
$T 600 $PT tests/test_gpu_configs.py tests/test_gpu_parity.py -k "hash or c7 or fallback or c6" > $O/tests.log 2>&1
rc=$?; echo "[tests rc=$rc]"; tail -1 $O/tests.log; grep -E "FAILED|Error" $O/tests.log | head -8; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for v in B P; do
    PGX_LIB=pinot_amd/ab/lib$v.so $T 300 python -u bench.py --workload c7 --steps 20 --warmup 3 --no-cpu-baseline > $O/c7_${v}_$rep.err 2>&1
    rc=$?; echo "[c7 $v $rep rc=$rc] $(python tools/bench_summary.py $O/c7_${v}_$rep.err | head -1)"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
