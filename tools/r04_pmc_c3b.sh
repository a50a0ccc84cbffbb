#!/bin/bash
# Round 4: PMC FETCH / WRITE / TCC write shapes of the narrow C3 kernels after the ring rework (one query at a time).
# request shapes.  Each counter set in its own pass, each pass under its own time limit.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04/pmc2
mkdir -p $OUT
export PGX_INFLIGHT=1
RX="pgxq|pgx_narrow|pgx_trim"
B="python3 bench.py --workload c3 --profile-iters 2"
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
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass tcc TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum
