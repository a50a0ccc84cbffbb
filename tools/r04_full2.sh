#!/bin/bash
# Round 4: the whole GPU test suite and smoke on the current sources.
set -o pipefail
O=gpurun_out/r04/full2
mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "[tests rc=$rc]"; tail -3 $O/gpu_tests.log; grep -E "FAILED|ERROR" $O/gpu_tests.log | head -5
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo "[smoke rc=$?]"; tail -2 $O/smoke.log
