set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/exp10
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/exp10/c5.json 2> gpurun_out/exp10/c5.err || exit 1
PGX_INFLIGHT=3 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/exp10/c5_3.json 2> gpurun_out/exp10/c5_3.err || exit 1
PGX_BATCH_SEGS=512 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/exp10/c5_batched.json 2> gpurun_out/exp10/c5_b.err || exit 1
timeout -k 10 300 python bench.py --workload c2 --no-cpu-baseline > gpurun_out/exp10/c2.json 2> gpurun_out/exp10/c2.err || exit 1
