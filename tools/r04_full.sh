#!/bin/bash
# Round 4: the whole GPU test suite, then the C5 and C1 bench lines.
set -o pipefail
O=gpurun_out/r04/full
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "[tests rc=$rc]"; tail -3 $O/gpu_tests.log
grep -E "FAILED|ERROR" $O/gpu_tests.log | head -5
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline > $O/c5.err 2>&1
echo "[c5 rc=$?]"; python tools/bench_summary.py $O/c5.err
timeout -k 10 300 python -u bench.py --workload c1 --steps 200 --warmup 20 --no-cpu-baseline > $O/c1.err 2>&1
echo "[c1 rc=$?]"; python tools/bench_summary.py $O/c1.err
