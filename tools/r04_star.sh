#!/bin/bash
# Round 4: star-tree GPU tests after the tile-capacity fix, and smoke.
set -o pipefail
O=gpurun_out/r04/star
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_startree.py tests/test_gpu_configs.py -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "[tests rc=$rc]"; tail -1 $O/tests.log; grep -E "FAILED|ERROR" $O/tests.log | head -5
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo "[smoke rc=$?]"; tail -1 $O/smoke.log
