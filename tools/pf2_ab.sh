#!/bin/bash
# A/B of the narrow scan's two-tile-ahead prefetch (PGX_DEBUG=pf2) against one tile ahead: parity subset under pf2,
# C3 bench lines interleaved twice, and one lone-query kernel trace each (run via gpurun from the repo root)
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p $OUT
PGX_DEBUG=pf2 timeout -k 10 400 python -u -m pytest tests/test_gpu_partition.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > $OUT/parity_pf2.log 2>&1
for rep in 1 2; do
  timeout -k 10 300 python bench.py --workload c3 --no-cpu-baseline > $OUT/c3_pf1_$rep.json 2> $OUT/c3_pf1_$rep.err
  PGX_DEBUG=pf2 timeout -k 10 300 python bench.py --workload c3 --no-cpu-baseline > $OUT/c3_pf2_$rep.json \
    2> $OUT/c3_pf2_$rep.err
done
PGX_DEBUG=pf2 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr -o c3pf2 -- \
  python3 tools/lone_probe.py --workload c3 --n 3 > $OUT/lone_pf2.log 2>&1
