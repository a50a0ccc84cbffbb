#!/bin/bash
# Memory-level parallelism of a workload's kernels (run via gpurun from the repo root): in-flight L2->EA read requests
# (TCC_EA0_RDREQ_LEVEL: average latency = LEVEL / RDREQ, average in flight = LEVEL / active cycles), DRAM credit stalls
# (the memory side refusing requests: bandwidth-saturated) over bench --profile-iters steps.
#   usage: tools/pmc_mlp.sh <workload> <out> [bench args...]
set -euo pipefail
export TMPDIR=/tmp
WL=$1; OUT=gpurun_out/$2; shift 2
mkdir -p $OUT
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum \
  GRBM_GUI_ACTIVE --kernel-include-regex "${PGX_PMC_REGEX:-pgxq|pgx_roaring|pgx_narrow|pgx_part}" \
  -d $OUT/mlp -o $WL --output-format csv -- python3 bench.py --workload $WL --profile-iters 3 "$@" > $OUT/mlp_$WL.log 2>&1
python3 tools/pmc_summary.py $OUT/mlp/${WL}_counter_collection.csv > $OUT/mlp_${WL}_summary.txt
rm -f $OUT/mlp/*_counter_collection.csv
