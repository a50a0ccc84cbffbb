#!/bin/bash
# Round 4: twelve-column queries in the generated kernel (C6): parity + JIT parity suite, C6 bench line.
set -o pipefail
O=gpurun_out/r04/c6
mkdir -p $O
T="timeout -k 10"
PT="python -u -m pytest -v --timeout 300 --timeout-method thread"
$T 600 $PT tests/test_gpu_configs.py -k c6 > $O/tests.log 2>&1
rc=$?; echo "[tests rc=$rc]"; tail -1 $O/tests.log; grep -E "FAILED|Error" $O/tests.log | head -5; [ $rc -ne 0 ] && exit $rc
$T 300 python -u bench.py --workload c6 --steps 20 --warmup 3 > $O/c6.err 2>&1
echo "[c6 rc=$?]"; python tools/bench_summary.py $O/c6.err; grep '^{' $O/c6.err | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['cpu_baseline'])"
