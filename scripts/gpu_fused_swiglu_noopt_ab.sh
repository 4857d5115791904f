#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rnd in 1 2; do
  for v in 1 0; do
    ST_OPT_PROBE_SKIP=1 ST_MLP_FUSED_SWIGLU=$v timeout -k 10 280 python bench.py --steps 8 --warmup 3 > gpurun_out/fsn_v${v}_r${rnd}.log 2>&1 || exit $?
    echo "noopt fused=$v round=$rnd $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fsn_v${v}_r${rnd}.log)"
  done
done
