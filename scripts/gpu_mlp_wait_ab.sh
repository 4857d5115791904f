#!/bin/bash
# MLP optimizer-bucket waits (both projections at MLP entry vs each at its own call) x fused SwiGLU,
# interleaved headline-bench rounds on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rnd in 1 2; do
  for cfg in "1 0" "0 0" "1 1" "0 1"; do
    set -- $cfg
    ST_MLP_WAIT_BOTH=$1 ST_MLP_FUSED_SWIGLU=$2 timeout -k 10 280 python bench.py --steps 8 --warmup 3 > gpurun_out/mw_$1$2_r${rnd}.log 2>&1 || exit $?
    echo "wait_both=$1 fused=$2 round=$rnd $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/mw_$1$2_r${rnd}.log)"
  done
done
