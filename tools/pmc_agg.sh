#!/bin/bash
# SQ counters of the narrow aggregation alone (tools/narrow_agg_bench.py), one PMC pass per counter set (run via gpurun
# from the repo root): gpurun_out/<out>/<tag>_{a,b}.txt.   usage: tools/pmc_agg.sh <out> <tag> [harness args...]
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/$1; TAG=$2; shift 2
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU \
  SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-include-regex pgx_narrow_aggregate \
  -d $OUT/pa -o $TAG --output-format csv -- python3 tools/narrow_agg_bench.py --reps 2 "$@" > $OUT/${TAG}_run_a.log 2>&1
python3 tools/pmc_summary.py $OUT/pa/${TAG}_counter_collection.csv > $OUT/${TAG}_a.txt
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES \
  --kernel-include-regex pgx_narrow_aggregate \
  -d $OUT/pb -o $TAG --output-format csv -- python3 tools/narrow_agg_bench.py --reps 2 "$@" > $OUT/${TAG}_run_b.log 2>&1
python3 tools/pmc_summary.py $OUT/pb/${TAG}_counter_collection.csv > $OUT/${TAG}_b.txt
rm -f $OUT/p?/*_counter_collection.csv
