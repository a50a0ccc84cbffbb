#!/bin/bash
# Round 4: C5 host phases of the throughput (one launch per kernel) plan, three queries in flight.
set -o pipefail
O=gpurun_out/r04/c5b
mkdir -p $O
PGX_HOST_PROFILE=1 timeout -k 10 300 python -u bench.py --workload c5 --steps 6 --warmup 2 --no-cpu-baseline > $O/host3.err 2>&1
rc=$?; echo "[host3 rc=$rc]"
python tools/bench_summary.py $O/host3.err
grep "pgx host us" $O/host3.err | tail -3 | cut -c1-900
