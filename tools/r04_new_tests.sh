#!/bin/bash
# Round 4: the new parity tests on the GPU box (bitmap memo order, packed dense updates, C5 headline execution).
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_bitmap.py tests/test_gpu_dense_pack.py tests/test_gpu_c5_headline.py \
  > gpurun_out/r04/new_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r04/new_tests.log
exit $rc
