#!/bin/bash
# Round 4: C3 kernel times per aggregation-function mix (which part of the narrow aggregation costs what), under
# rocprofv3, plus the C1 bench with the async worker pool.
set -o pipefail
O=gpurun_out/r04/c3h
mkdir -p $O
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in full sum count minmax; do
  VARIANT_QUERY=$v $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o c3 -- \
    python3 tools/c3_variants.py > $O/$v.log 2>&1
  rc=$?
  echo "[variant $v rc=$rc] $(grep kernel_ms $O/$v.log)"
  if [ $rc -ne 0 ]; then tail -3 $O/$v.log; exit $rc; fi
  awk -F'",' 'NR>1 {split($1,a,"("); n=a[1]; gsub(/"/,"",n); split($2,b,","); printf "  %-50.50s calls=%s avg_us=%.1f\n", n, b[1], b[3]/1000}' $O/$v/c3_kernel_stats.csv | grep -v synth | head -5
done
$T 300 python -u bench.py --workload c1 --steps 200 --warmup 20 --no-cpu-baseline > $O/c1.err 2>&1
echo "[c1 rc=$?]"
python tools/bench_summary.py $O/c1.err
