#!/bin/bash
# In-step A/B of the W^T copy stream's HIP priority (separate processes, alternating).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for i in 1 2; do
  for p in 0 -1; do
    ms=$(ST_WT_STREAM_PRIORITY=$p timeout -k 10 300 python3 bench.py --steps 8 --warmup 3 2>/dev/null | grep -o '"ms_per_step": [0-9.]*') || exit 1
    echo "wt_priority=$p run $i: $ms"
  done
done
