#!/bin/bash
# round-3 first GPU call: default bench line, C5 profile (trace + per-step timeline + PMC traffic per step), GPU suite
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/r03_bench_c5.json 2> gpurun_out/r03_bench_c5.err || exit 1
PGX_HOST_PROFILE=1 timeout -k 10 200 python tools/c5_breakdown.py 4096 5 > gpurun_out/r03_c5_breakdown.log 2>&1 || exit 1
timeout -k 10 900 bash tools/profile_wl.sh c5 10 --no-cpu-baseline > gpurun_out/r03_prof_c5.log 2>&1 || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03_gputests.log 2>&1
