#!/bin/bash
# Round 4: C6 query-kernel variants (rows per lane, value image) and the generated source for offline resource checks.
set -o pipefail
O=gpurun_out/r04/c6b
mkdir -p $O/dump
T="timeout -k 10"
PGX_JIT_DUMP=$O/dump $T 300 python -u bench.py --workload c6 --steps 3 --warmup 1 --no-cpu-baseline > $O/dump.err 2>&1
echo "[dump rc=$?]"
for v in "PGX_FRAC=1" "PGX_NO_IMG=1" "PGX_FRAC=1 PGX_NO_IMG=1" "PGX_COMPACT=1"; do
  env $v $T 300 python -u bench.py --workload c6 --steps 10 --warmup 2 --no-cpu-baseline > $O/v.err 2>&1
  echo "[$v rc=$?] $(python tools/bench_summary.py $O/v.err | head -1)"
done
