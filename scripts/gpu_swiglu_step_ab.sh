#!/bin/bash
# In-step A/B of the SwiGLU vectors per lane (separate processes, alternating).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for i in 1 2; do
  for u in 2 1; do
    ms=$(ST_SWIGLU_U=$u timeout -k 10 300 python3 bench.py --steps 8 --warmup 3 2>/dev/null | grep -o '"ms_per_step": [0-9.]*') || exit 1
    echo "U=$u run $i: $ms"
  done
done
