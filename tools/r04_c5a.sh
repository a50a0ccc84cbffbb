#!/bin/bash
# Round 4: C5 state on the current sources: bench (3 in flight), one query at a time under rocprofv3, host phases.
set -o pipefail
O=gpurun_out/r04/c5a
mkdir -p $O
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
$T 300 python -u bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline > $O/bench.err 2>&1
rc=$?; echo "[bench rc=$rc]"; [ $rc -ne 0 ] && { tail -5 $O/bench.err; exit $rc; }
python tools/bench_summary.py $O/bench.err
PGX_INFLIGHT=1 $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof1 -o c5 -- \
  python3 bench.py --workload c5 --profile-iters 3 > $O/prof1.log 2>&1
rc=$?; echo "[prof1 rc=$rc]"; [ $rc -ne 0 ] && { tail -5 $O/prof1.log; exit $rc; }
awk -F'",' 'NR>1 {split($1,a,"("); n=a[1]; gsub(/"/,"",n); split($2,b,","); printf "  %-50.50s calls=%s avg_us=%.1f\n", n, b[1], b[3]/1000}' $O/prof1/c5_kernel_stats.csv | grep -v synth | head -6
PGX_HOST_PROFILE=1 PGX_INFLIGHT=1 $T 300 python -u bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline > $O/host.err 2>&1
rc=$?; echo "[host rc=$rc]"
python tools/bench_summary.py $O/host.err
grep "pgx host us" $O/host.err | tail -2 | cut -c1-600
