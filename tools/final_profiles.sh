#!/bin/bash
# Round-end profiles: kernel trace + stats and per-step PMC traffic (C5, C3, C2), then the 2-rank gloo rehearsal.
set -euo pipefail
bash tools/profile_wl.sh c5 10
echo "c5 profiled"
bash tools/profile_wl.sh c3 5
echo "c3 profiled"
bash tools/profile_wl.sh c2 10
echo "c2 profiled"
bash tools/rehearse_multi.sh
echo "rehearsal done"
