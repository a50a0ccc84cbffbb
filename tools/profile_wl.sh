#!/bin/bash
# GPU-box profile of one workload (run via gpurun from the repo root):
#   kernel trace + stats of a bench run -> gpurun_out/prof_<wl>/trace/<wl>_kernel_stats.csv (+ bench JSON line)
#   FETCH_SIZE and WRITE_SIZE passes    -> gpurun_out/prof_<wl>/pmc_{fetch,write}/  and traffic_<wl>.json
# usage: tools/profile_wl.sh <workload> <steps> [bench args...]
set -euo pipefail
export TMPDIR=/tmp
WL=$1; STEPS=$2; shift 2
OUT=gpurun_out/prof_$WL
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o $WL --output-format csv -- \
  python3 bench.py --workload $WL --steps $STEPS --warmup 2 "$@" > $OUT/bench.log 2>&1
grep '^{' $OUT/bench.log > $OUT/bench.json
# the launches bench.py's roofline times (pgx_execute_timed: every segment in one launch per kernel), alone
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_timed -o $WL --output-format csv -- \
  python3 bench.py --workload $WL --profile-iters 10 "$@" > $OUT/bench_timed.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "${PGX_PMC_REGEX:-pgxq|pgx_roaring|pgx_part}" -d $OUT/pmc_fetch -o $WL --output-format csv -- \
  python3 bench.py --workload $WL --profile-iters 5 "$@" > $OUT/pmc_fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "${PGX_PMC_REGEX:-pgxq|pgx_roaring|pgx_part}" -d $OUT/pmc_write -o $WL --output-format csv -- \
  python3 bench.py --workload $WL --profile-iters 5 "$@" > $OUT/pmc_write.log 2>&1
ROWS=$(python3 -c "import json; print(json.load(open('$OUT/bench.json'))['config']['rows_per_segment'])")
python3 tools/pmc_traffic.py $OUT/pmc_fetch/${WL}_counter_collection.csv,$OUT/pmc_write/${WL}_counter_collection.csv \
  ${PGX_PMC_KERNELS:-pgxq} $WL $ROWS $OUT/traffic_$WL.json
rm -f $OUT/pmc_fetch/*_counter_collection.csv $OUT/pmc_write/*_counter_collection.csv $OUT/trace/*_kernel_trace.csv $OUT/trace_timed/*_kernel_trace.csv
