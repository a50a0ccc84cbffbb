#!/bin/bash
# Round-end profiles: kernel trace + stats and per-step PMC traffic (tools/profile_wl.sh) for the bench workloads.
#   usage: tools/final_profiles.sh [workloads...]   (default: c5 c3 c2 c6 c7 c3d c3m2 c3f)
set -euo pipefail
WLS=${*:-c5 c3 c2 c6 c7 c3d c3m2 c3f}
for wl in $WLS; do
  case $wl in c3|c3d|c3m2|c3f|c7) steps=5 ;; *) steps=10 ;; esac
  bash tools/profile_wl.sh $wl $steps --no-cpu-baseline
  echo "$wl profiled: $(python3 -c "import json; d=json.load(open('gpurun_out/prof_$wl/traffic_$wl.json')); print(d['hbm_bytes_per_launch'], d['source_hash'])" 2>/dev/null)"
done
