#!/bin/bash
# One PMC pass of SQ issue/wait counters (+ GRBM) over a bench workload's timed launches (run via gpurun from the repo
# root): gpurun_out/<out>/sq/<wl>_counter_collection.csv.   usage: tools/pmc_sq.sh <workload> <out> [bench args...]
set -euo pipefail
export TMPDIR=/tmp
WL=$1; OUT=gpurun_out/$2; shift 2
mkdir -p $OUT
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU \
  SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --kernel-include-regex "${PGX_PMC_REGEX:-pgxq|pgx_roaring|pgx_part}" \
  -d $OUT/sq -o $WL --output-format csv -- \
  python3 bench.py --workload $WL --profile-iters 3 "$@" > $OUT/sq_$WL.log 2>&1
python3 tools/pmc_summary.py $OUT/sq/${WL}_counter_collection.csv > $OUT/sq_${WL}_summary.txt
rm -f $OUT/sq/*_counter_collection.csv
