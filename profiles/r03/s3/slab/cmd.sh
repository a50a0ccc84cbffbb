set -o pipefail
mkdir -p gpurun_out/slab
timeout -k 10 600 python -u -m pytest tests/test_gpu_partition.py -x -q --timeout 120 --timeout-method thread > gpurun_out/slab/part_tests.log 2>&1 || { echo "tests failed $?"; tail -30 gpurun_out/slab/part_tests.log; exit 1; }
tail -3 gpurun_out/slab/part_tests.log
timeout -k 10 300 python bench.py --workload c3 --no-cpu-baseline > gpurun_out/slab/c3.json 2> gpurun_out/slab/c3.err || exit 1
PGX_PART_SLAB=0 timeout -k 10 300 python bench.py --workload c3 --no-cpu-baseline > gpurun_out/slab/c3_rows.json 2> gpurun_out/slab/c3_rows.err || exit 1
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/slab/prof -o c3 -- python3 $GRAFT_REPO_ROOT/bench.py --workload c3 --no-cpu-baseline --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/slab/c3_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/slab/c3_prof.err
echo done
