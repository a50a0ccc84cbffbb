#!/bin/bash
# Round 4: A/B of the generator changes: A = round-4 final, B = uniform segment pointers + carried tile base,
# C = B + 32-bit LDS home-slot hash.  Same box, interleaved.
set -o pipefail
O=gpurun_out/r04/ab
mkdir -p $O
T="timeout -k 10"
for rep in 1 2; do
  for v in A B C; do
    for w in c7 c6; do
      PGX_LIB=pinot_amd/ab/lib$v.so $T 300 python -u bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline > $O/${w}_${v}_$rep.err 2>&1
      rc=$?; echo "[$w $v $rep rc=$rc] $(python tools/bench_summary.py $O/${w}_${v}_$rep.err | head -1)"; [ $rc -ne 0 ] && exit $rc
    done
  done
done
for v in A C; do
  PGX_LIB=pinot_amd/ab/lib$v.so $T 300 python -u bench.py --workload c5 --no-cpu-baseline > $O/c5_$v.err 2>&1
  rc=$?; echo "[c5 $v rc=$rc] $(python tools/bench_summary.py $O/c5_$v.err | head -1)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
