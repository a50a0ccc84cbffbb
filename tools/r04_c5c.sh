#!/bin/bash
# Round 4: plan-cache tests, C5 bench (3 in flight) and one query at a time (PGX_INFLIGHT=1) with host phases.
set -o pipefail
O=gpurun_out/r04/c5c
mkdir -p $O
T="timeout -k 10"
$T 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_c5_headline.py > $O/tests.log 2>&1
rc=$?; echo "[tests rc=$rc]"; tail -1 $O/tests.log; grep -E "FAILED|Error" $O/tests.log | head -5; [ $rc -ne 0 ] && exit $rc
$T 300 python -u bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline > $O/c5.err 2>&1
echo "[c5 rc=$?]"; python tools/bench_summary.py $O/c5.err
PGX_INFLIGHT=1 PGX_HOST_PROFILE=1 $T 300 python -u bench.py --workload c5 --steps 6 --warmup 3 --no-cpu-baseline > $O/c5single.err 2>&1
echo "[c5single rc=$?]"; python tools/bench_summary.py $O/c5single.err
grep "pgx host us" $O/c5single.err | tail -2 | cut -c1-300
