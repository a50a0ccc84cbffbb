#!/bin/bash
# Same-box A/B of library builds (run via gpurun from the repo root).  Every (rep, lib, workload) runs bench.py once,
# interleaved, so box-to-box noise cancels; one summary line each.
#   usage: tools/ab.sh <out> "<workloads>" "<lib.so paths>" <reps> [bench args...]
set -o pipefail
O=gpurun_out/$1; WLS=$2; LIBS=$3; REPS=$4; shift 4
mkdir -p $O
for rep in $(seq 1 $REPS); do
  for lib in $LIBS; do
    v=$(basename $lib .so)
    for w in $WLS; do
      PGX_LIB=$lib timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline "$@" > $O/${w}_${v}_$rep.err 2>&1
      rc=$?; echo "[$w $v $rep rc=$rc] $(python tools/bench_summary.py $O/${w}_${v}_$rep.err | tr "\n" " ")"
      [ $rc -ne 0 ] && { tail -5 $O/${w}_${v}_$rep.err; exit $rc; }
    done
  done
done
exit 0
