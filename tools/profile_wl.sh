#!/bin/bash
# GPU-box profile of one workload (run via gpurun from the repo root):
#   kernel trace + stats of a bench run        -> gpurun_out/prof_<wl>/trace/<wl>_kernel_stats.csv (+ bench JSON line)
#   per-step busy union of that trace           -> gpurun_out/prof_<wl>/timeline.jsonl (tools/timeline.py)
#   FETCH_SIZE and WRITE_SIZE passes over exactly PSTEPS bench steps (bench.py --profile-iters)
#                                               -> gpurun_out/prof_<wl>/traffic_<wl>.json: HBM bytes per STEP
# usage: tools/profile_wl.sh <workload> <steps> [bench args...]
set -euo pipefail
export TMPDIR=/tmp
WL=$1; STEPS=$2; shift 2
PSTEPS=${PGX_PMC_STEPS:-4}
KRX=${PGX_PMC_REGEX:-pgxq|pgx_roaring|pgx_part|pgx_narrow|pgx_trim|pgx_init|pgx_compact|pgx_group|pgx_fsm|pgx_mv|pgx_join|pgx_gather}
KLIST=${PGX_PMC_KERNELS:-pgxq+pgx_roaring+pgx_partition+pgx_part_aggregate+pgx_narrow_split+pgx_narrow_aggregate+pgx_narrow_compact+pgx_trim+pgx_init+pgx_compact+pgx_group+pgx_join+pgx_gather}
OUT=gpurun_out/prof_$WL
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o $WL --output-format csv -- \
  python3 bench.py --workload $WL --steps $STEPS --warmup 2 "$@" > $OUT/bench.log 2>&1
grep '^{' $OUT/bench.log > $OUT/bench.json
python3 tools/timeline.py $OUT/trace/${WL}_kernel_trace.csv 1.0 "$KRX" > $OUT/timeline.jsonl
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRX" -d $OUT/pmc_fetch -o $WL --output-format csv -- \
  python3 bench.py --workload $WL --profile-iters $PSTEPS "$@" > $OUT/pmc_fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRX" -d $OUT/pmc_write -o $WL --output-format csv -- \
  python3 bench.py --workload $WL --profile-iters $PSTEPS "$@" > $OUT/pmc_write.log 2>&1
ROWS=$(python3 -c "import json; print(json.load(open('$OUT/bench.json'))['config']['rows_per_segment'])")
python3 tools/pmc_traffic.py $OUT/pmc_fetch/${WL}_counter_collection.csv,$OUT/pmc_write/${WL}_counter_collection.csv \
  "$KLIST" $WL $ROWS $OUT/traffic_$WL.json $PSTEPS
python3 tools/reconcile.py $OUT/trace/${WL}_kernel_trace.csv $OUT/bench.json $OUT/reconcile_$WL.json > /dev/null || true
rm -f $OUT/pmc_fetch/*_counter_collection.csv $OUT/pmc_write/*_counter_collection.csv $OUT/trace/*_kernel_trace.csv
