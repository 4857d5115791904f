#!/bin/bash
# SwiGLU launch-shape A/B (separate processes: the knobs are read once): vectors per lane
# (ST_SWIGLU_U) and the row cap of the grid (ST_SWIGLU_ROWS), Llama-3-8B I = 14336, 6 x 4096 rows.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for cfg in "2 0" "1 0" "4 0" "7 0" "2 4096" "7 4096" "2 0"; do
  set -- $cfg
  out=$(ST_SWIGLU_U=$1 ST_SWIGLU_ROWS=$2 timeout -k 10 120 python3 tools/bench_kernels.py --only elt --batch 6 --no-ref 2>/dev/null | grep -o '"swiglu_[a-z]*_GBps": [0-9.]*' | tr '\n' ' ') || exit 1
  echo "U=$1 rows=$2: $out"
done
