#!/bin/bash
# A/B of the lone C5 replay's first-part size (PGX_DEBUG=head=N: programs and query kernel of the first 1/N of the
# segments, the rest's programs on the side stream): tools/lone_probe.py per N, interleaved twice (run via gpurun)
set -euo pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
for rep in 1 2; do
  for h in 2 4 8 16; do
    PGX_DEBUG=head=$h timeout -k 10 200 python tools/lone_probe.py --workload c5 --n 12 > $OUT/head${h}_$rep.log 2>&1
  done
done
