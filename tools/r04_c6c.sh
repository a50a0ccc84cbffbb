#!/bin/bash
# Round 4: C6 with the register-budgeted tile shape (image on / off), C6 parity, and C2 / C5 lines unchanged.
set -o pipefail
O=gpurun_out/r04/c6c
mkdir -p $O/dump
T="timeout -k 10"
$T 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_configs.py -k c6 > $O/tests.log 2>&1
rc=$?; echo "[tests rc=$rc]"; tail -1 $O/tests.log; [ $rc -ne 0 ] && exit $rc
PGX_JIT_DUMP=$O/dump $T 300 python -u bench.py --workload c6 --steps 10 --warmup 2 --no-cpu-baseline > $O/c6.err 2>&1
echo "[c6 rc=$?] $(python tools/bench_summary.py $O/c6.err | head -1)"
PGX_NO_IMG=1 $T 300 python -u bench.py --workload c6 --steps 10 --warmup 2 --no-cpu-baseline > $O/v.err 2>&1
echo "[c6 noimg rc=$?] $(python tools/bench_summary.py $O/v.err | head -1)"
for w in c2 c5; do
  $T 300 python -u bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline > $O/$w.err 2>&1
  echo "[$w rc=$?] $(python tools/bench_summary.py $O/$w.err | head -1)"
done
