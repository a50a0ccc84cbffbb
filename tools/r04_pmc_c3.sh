#!/bin/bash
# Round 4: PMC counters of the narrow C3 kernels (one query at a time, 2 steps): SQ issue / wait, FETCH, WRITE, TCC
# request shapes.  Each counter set in its own pass, each pass under its own time limit.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04/pmc
mkdir -p $OUT
export PGX_INFLIGHT=1
RX="pgxq|pgx_narrow|pgx_trim"
B="python3 bench.py --workload c3 --profile-iters 2"
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
grep -oE "TCC_EA0_[A-Z0-9_]+|TCC_[A-Z_]*WR[A-Z0-9_]*|TCP_TCC_[A-Z_]+" $OUT/counters.txt | sort -u | head -40
pass() {  # pass <name> <counters...>
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "$RX" -d $OUT/$name -o c3 --output-format csv -- $B \
    > $OUT/$name.log 2>&1
  local rc=$?
  echo "[pass $name rc=$rc]"
  if [ $rc -ne 0 ]; then tail -3 $OUT/$name.log; exit $rc; fi
  python3 tools/pmc_summary.py $OUT/$name/c3_counter_collection.csv | tee $OUT/${name}_summary.txt
  rm -f $OUT/$name/c3_counter_collection.csv
}
pass sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU GRBM_GUI_ACTIVE
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass tcc TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum
