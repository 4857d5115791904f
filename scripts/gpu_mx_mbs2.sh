#!/bin/bash
# Mixtral proxy at round 4's measured config (micro-batch 2, no accumulation; the preset runs
# micro-batch 1 x 2) with the grouped expert wgrad on wgrad4 (default) and on the 4-stage kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rnd in 1 2; do
  for v in 1 0; do
    ST_WGRAD_GROUPED4=$v timeout -k 10 200 python bench.py --layout mixtral_ep8 --layers 4 --micro_batch_size 2 --grad_acc 1 --steps 6 --warmup 2 > gpurun_out/mx2_v${v}_r${rnd}.log 2>&1 || exit $?
    echo "mixtral mbs2 grouped4=$v round=$rnd $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/mx2_v${v}_r${rnd}.log) $(grep -o '"mfu_pct": [0-9.]*' gpurun_out/mx2_v${v}_r${rnd}.log)"
  done
done
exit 0
