#!/bin/bash
# Round 4: narrow kernels: batched probe misses, 16-byte unit stores; parity, C3 kernel stats, C3 variants.
set -o pipefail
O=gpurun_out/r04/c3i
mkdir -p $O
T="timeout -k 10"
step() {  # step <log> <seconds> <cmd...>
  local log=$1 secs=$2; shift 2
  $T $secs "$@" > $log 2>&1
  local rc=$?
  echo "[step rc=$rc] $*" | cut -c1-160
  tail -2 $log | cut -c1-300
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
PT="python -u -m pytest -v --timeout 300 --timeout-method thread"
step $O/partition.log 600 $PT tests/test_gpu_partition.py -k "narrow or matches_oracle"
step $O/configs.log 600 $PT tests/test_gpu_configs.py -k c3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
prof() {  # prof <name> <env...>
  local name=$1; shift
  env "$@" PGX_INFLIGHT=1 $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$name -o c3 -- \
    python3 bench.py --workload c3 --profile-iters 2 > $O/$name.log 2>&1
  local rc=$?
  echo "[prof $name rc=$rc]"
  if [ $rc -ne 0 ]; then tail -3 $O/$name.log; exit $rc; fi
  awk -F'",' 'NR>1 {split($1,a,"("); n=a[1]; gsub(/"/,"",n); split($2,b,","); printf "  %-50.50s calls=%s avg_us=%.1f\n", n, b[1], b[3]/1000}' $O/$name/c3_kernel_stats.csv | head -8
}
prof ring
for v in count sum; do
  VARIANT_QUERY=$v $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o c3 -- \
    python3 tools/c3_variants.py > $O/$v.log 2>&1
  rc=$?
  echo "[variant $v rc=$rc] $(grep kernel_ms $O/$v.log)"
  if [ $rc -ne 0 ]; then tail -3 $O/$v.log; exit $rc; fi
  awk -F'",' 'NR>1 {split($1,a,"("); n=a[1]; gsub(/"/,"",n); split($2,b,","); printf "  %-50.50s calls=%s avg_us=%.1f\n", n, b[1], b[3]/1000}' $O/$v/c3_kernel_stats.csv | grep -v synth | head -4
done
