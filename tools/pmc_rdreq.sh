#!/bin/bash
# Read-request widths per kernel (gfx950): TCC_EA0_RDREQ (all), _32B and TCC_BUBBLE (128-B) over a bench workload's
# --profile-iters steps, so the FETCH_SIZE x 2 streaming correction can be checked per kernel (mixed-width readers).
# usage (via gpurun, repo root): tools/pmc_rdreq.sh <workload> <out> [bench args...]
set -euo pipefail
export TMPDIR=/tmp
WL=$1; OUT=gpurun_out/$2; shift 2
mkdir -p $OUT
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum \
  --kernel-include-regex "${PGX_PMC_REGEX:-pgxq|pgx_roaring|pgx_narrow|pgx_part}" \
  -d $OUT/rq -o $WL --output-format csv -- python3 bench.py --workload $WL --profile-iters 3 "$@" > $OUT/rq_$WL.log 2>&1
python3 tools/pmc_summary.py $OUT/rq/${WL}_counter_collection.csv > $OUT/rq_${WL}_summary.txt
rm -f $OUT/rq/*_counter_collection.csv
