#!/bin/bash
# A/B of the narrow scan's unit size (PGX_DEBUG=nunit=16: 16-record units, 32-record rings, 256-thread workgroups,
# two per CU) against the default (32-record units, 64-record rings, 512 threads): parity subset under nunit=16, then
# C3 bench lines interleaved twice (run via gpurun from the repo root)
set -euo pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
PGX_DEBUG=nunit=16 timeout -k 10 400 python -u -m pytest tests/test_gpu_partition.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > $OUT/parity_nunit16.log 2>&1
for rep in 1 2; do
  timeout -k 10 300 python bench.py --workload c3 --no-cpu-baseline > $OUT/c3_u32_$rep.json 2> $OUT/c3_u32_$rep.err
  PGX_DEBUG=nunit=16 timeout -k 10 300 python bench.py --workload c3 --no-cpu-baseline > $OUT/c3_u16_$rep.json \
    2> $OUT/c3_u16_$rep.err
done
