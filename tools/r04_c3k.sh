#!/bin/bash
# Round 4: trim with 11-bit digits and aggregation-seeded key ranges: parity (partition, C3 configs, multi-device merges
# + trims), C3 kernel stats one query at a time, PMC FETCH / WRITE per kernel.
set -o pipefail
O=gpurun_out/r04/c3k
mkdir -p $O
T="timeout -k 10"
PT="python -u -m pytest -v --timeout 300 --timeout-method thread"
$T 900 $PT tests/test_gpu_partition.py tests/test_gpu_configs.py tests/test_gpu_multi.py > $O/tests.log 2>&1
rc=$?; echo "[tests rc=$rc]"; tail -1 $O/tests.log; grep -E "FAILED|Error" $O/tests.log | head -5; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
PGX_INFLIGHT=1 $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof1 -o c3 -- \
  python3 bench.py --workload c3 --profile-iters 2 > $O/prof1.log 2>&1
rc=$?; echo "[prof1 rc=$rc]"; [ $rc -ne 0 ] && { tail -3 $O/prof1.log; exit $rc; }
awk -F'",' 'NR>1 {split($1,a,"("); n=a[1]; gsub(/"/,"",n); split($2,b,","); printf "  %-50.50s calls=%s avg_us=%.1f\n", n, b[1], b[3]/1000}' $O/prof1/c3_kernel_stats.csv | grep -v synth | head -9
export PGX_INFLIGHT=1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "pgxq|pgx_narrow|pgx_trim" -d $O/$c -o c3 --output-format csv -- \
    python3 bench.py --workload c3 --profile-iters 2 > $O/$c.log 2>&1
  rc=$?; echo "[pmc $c rc=$rc]"; [ $rc -ne 0 ] && { tail -3 $O/$c.log; exit $rc; }
  python3 tools/pmc_summary.py $O/$c/c3_counter_collection.csv > $O/${c}_summary.txt
  rm -f $O/$c/c3_counter_collection.csv
done
python3 - <<'PY'
import re
tot = 0.0
for c, mul in (("FETCH_SIZE", 2 * 1024), ("WRITE_SIZE", 1024)):
    name = None
    for line in open("gpurun_out/r04/c3k/%s_summary.txt" % c):
        if not line.startswith(" "):
            name = line.strip()[:40]
            continue
        m = re.match(r"\s+(\S+)\s+(\S+)\s+\(n=(\d+)\)", line)
        if m:
            b = float(m.group(2)) * int(m.group(3)) / 2 * mul  # per step (2 steps)
            tot += b
            print("%-10s %-40s %.3f GB" % (c, name, b / 1e9))
print("total per step %.2f GB" % (tot / 1e9))
PY
