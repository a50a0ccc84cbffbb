#!/bin/bash
# Round 4 end, after the last library change: plan-cache / headline / multi-device / realtime GPU tests, the 2-rank
# rehearsal, the final profiles (C5, C3, C2) and one bench line per workload.
set -o pipefail
O=gpurun_out/r04/final2
mkdir -p $O
T="timeout -k 10"
PT="python -u -m pytest -v --timeout 300 --timeout-method thread"
$T 600 $PT tests/test_gpu_c5_headline.py tests/test_gpu_multi.py tests/test_gpu_realtime.py tests/test_gpu_batched.py > $O/tests.log 2>&1
rc=$?; echo "[tests rc=$rc]"; tail -1 $O/tests.log; grep -E "FAILED|ERROR" $O/tests.log | head -5; [ $rc -ne 0 ] && exit $rc
$T 800 bash tools/rehearse_multi.sh > $O/rehearse.log 2>&1
rc=$?; echo "[rehearse rc=$rc]"; for f in gpurun_out/multi/*.log; do echo "$f: $(grep '^{' $f | tail -1 | cut -c1-160)"; done
[ $rc -ne 0 ] && exit $rc
bash tools/r04_final.sh
rc=$?; [ $rc -ne 0 ] && exit $rc
for w in c5 c3 c2; do cp gpurun_out/prof_$w/traffic_$w.json profiles/traffic_$w.json; done
bash tools/r04_benches.sh
