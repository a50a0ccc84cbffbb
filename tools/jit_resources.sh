#!/bin/bash
# Developer aid: dump the JIT selftest kernels (pgx_jit_selftest) and print hipcc's resource usage per shape
# (VGPRs, scratch spill, occupancy, LDS) for gfx950.  CPU only.
set -euo pipefail
D=$(mktemp -d)
PGX_JIT_DUMP=$D python3 -c "
import ctypes; L=ctypes.CDLL('pinot_amd/libpgx.so')
n=ctypes.c_int(); buf=ctypes.create_string_buffer(1<<16)
L.pgx_jit_selftest(ctypes.byref(n), buf, len(buf))"
for f in $(ls $D/*.hip | sort -V); do
  (echo '#include <hip/hip_runtime.h>'; cat $f) > $D/x.hip
  r=$(hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -c $D/x.hip -o $D/x.o -Rpass-analysis=kernel-resource-usage 2>&1 |
      grep -E "VGPRs:|ScratchSize|Occupancy|LDS Size" | sed 's/.*remark: *//; s/ \[-Rpass.*//' | tr '\n' ' ')
  echo "$(basename $f) T=$(grep -m1 'define PT' $f | awk '{print $3}') R=$(grep -m1 'define PR' $f | awk '{print $3}') $r"
done
rm -rf $D
