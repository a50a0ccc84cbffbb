#!/bin/bash
# A/B of LDS value images against dictionary gathers in the query kernels (PGX_DEBUG=noimg) at C5 (3.8% of rows
# selected): parity subset under noimg, C5 bench lines interleaved twice (run via gpurun from the repo root)
set -euo pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
PGX_DEBUG=noimg timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c5_headline.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > $OUT/parity_noimg.log 2>&1
for rep in 1 2; do
  timeout -k 10 300 python bench.py --workload c5 --no-cpu-baseline > $OUT/c5_img_$rep.json 2> $OUT/c5_img_$rep.err
  PGX_DEBUG=noimg timeout -k 10 300 python bench.py --workload c5 --no-cpu-baseline > $OUT/c5_noimg_$rep.json \
    2> $OUT/c5_noimg_$rep.err
done
