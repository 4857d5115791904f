#!/bin/bash
# Headline A/B: the per-shape weight-gradient pick with and without csrc/wgrad4.hip (variant 6).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rnd in 1 2; do
  for v in 1 0; do
    ST_WGRAD4=$v ST_WGRAD_TUNE_LOG=1 timeout -k 10 280 python bench.py --steps 8 --warmup 3 > gpurun_out/w4_v${v}_r${rnd}.log 2>&1 || exit $?
    echo "wgrad4=$v round=$rnd $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/w4_v${v}_r${rnd}.log)"
  done
done
