#!/bin/bash
# Round 4: split kernel with vector loads (parity + C3 kernel stats), C3 bench (3 in flight), C5 single-query host
# profile (library phases + Python profile).
set -o pipefail
O=gpurun_out/r04/c3j
mkdir -p $O
T="timeout -k 10"
PT="python -u -m pytest -v --timeout 300 --timeout-method thread"
$T 600 $PT tests/test_gpu_partition.py -k "narrow or matches_oracle" > $O/partition.log 2>&1
rc=$?; echo "[partition rc=$rc]"; tail -1 $O/partition.log; [ $rc -ne 0 ] && exit $rc
$T 600 $PT tests/test_gpu_configs.py -k c3 > $O/configs.log 2>&1
rc=$?; echo "[configs rc=$rc]"; tail -1 $O/configs.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
PGX_INFLIGHT=1 $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof1 -o c3 -- \
  python3 bench.py --workload c3 --profile-iters 2 > $O/prof1.log 2>&1
rc=$?; echo "[prof1 rc=$rc]"; [ $rc -ne 0 ] && { tail -3 $O/prof1.log; exit $rc; }
awk -F'",' 'NR>1 {split($1,a,"("); n=a[1]; gsub(/"/,"",n); split($2,b,","); printf "  %-50.50s calls=%s avg_us=%.1f\n", n, b[1], b[3]/1000}' $O/prof1/c3_kernel_stats.csv | grep -v synth | head -8
$T 300 python -u bench.py --workload c3 --steps 10 --warmup 3 --no-cpu-baseline > $O/c3.err 2>&1
echo "[c3 rc=$?]"; python tools/bench_summary.py $O/c3.err
PGX_INFLIGHT=1 PGX_HOST_PROFILE=1 PGX_BENCH_CPROFILE=$O/c5single.prof $T 300 python -u bench.py --workload c5 --steps 6 --warmup 3 --no-cpu-baseline > $O/c5single.err 2>&1
echo "[c5single rc=$?]"; python tools/bench_summary.py $O/c5single.err
grep "pgx host us" $O/c5single.err | tail -2 | cut -c1-400
python -c "
import pstats; pstats.Stats('$O/c5single.prof').sort_stats('tottime').print_stats(14)" | tail -22 | cut -c1-150
