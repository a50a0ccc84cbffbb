#!/bin/bash
# GPU-box profiling recipe (run via gpurun from the repo root):
#   1. kernel trace + stats of the bench command        -> gpurun_out/prof/<wl>_kernel_stats.csv
#   2. PMC FETCH_SIZE pass, 3. PMC WRITE_SIZE pass      -> gpurun_out/pmc_{fetch,write}/
#   4. traffic per launch (gfx950 corrections)           -> profiles/traffic_<wl>.json (copied back under gpurun_out/)
# usage: tools/gpu_profile.sh <workload> [bench args...]
set -euo pipefail
export TMPDIR=/tmp
WL=${1:-c2}; shift || true
OUT=gpurun_out/prof_$WL
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o $WL --output-format csv -- \
  python3 bench.py --workload $WL --steps 20 --warmup 3 --no-cpu-baseline "$@" > $OUT/bench_under_rocprof.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o $WL --output-format csv -- \
  python3 bench.py --workload $WL --profile-iters 5 "$@" > $OUT/pmc_fetch.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o $WL --output-format csv -- \
  python3 bench.py --workload $WL --profile-iters 5 "$@" > $OUT/pmc_write.log 2>&1
find $OUT -name "*.csv" | sort > $OUT/files.txt
cat $OUT/files.txt
