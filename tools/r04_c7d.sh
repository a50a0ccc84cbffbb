#!/bin/bash
# Round 4: star-tree tile capacity fix + packed LDS hash planes: star / configs / parity / partition / MV GPU tests,
# smoke, C7 bench with and without the pack.
set -o pipefail
O=gpurun_out/r04/c7d
mkdir -p $O
T="timeout -k 10"
PT="python -u -m pytest -v --timeout 300 --timeout-method thread"
$T 1000 $PT tests/test_gpu_startree.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_partition.py tests/test_gpu_mv.py > $O/tests.log 2>&1
rc=$?; echo "[tests rc=$rc]"; tail -1 $O/tests.log; grep -E "FAILED|ERROR" $O/tests.log | head -5; [ $rc -ne 0 ] && exit $rc
$T 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo "[smoke rc=$?]"; tail -1 $O/smoke.log
for v in "PGX_DENSE_PACK=1" "PGX_DENSE_PACK=0"; do
  env $v $T 300 python -u bench.py --workload c7 --steps 10 --warmup 2 --no-cpu-baseline > $O/c7.err 2>&1
  echo "[c7 $v rc=$?] $(python tools/bench_summary.py $O/c7.err | head -1)"
done
