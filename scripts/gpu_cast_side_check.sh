#!/bin/bash
# DP8 ZeRO-1 rehearsal (8 gloo ranks on one GPU) with the bucket fp32->bf16 cast on the
# compute stream (ST_CAST_SIDE=0) vs the side stream (1): identical losses expected.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in 0 1; do
  ST_CAST_SIDE=$v LAYOUTS=dp bash scripts/rehearse_layouts_1gpu.sh > gpurun_out/cast_side_$v.log 2>&1 || exit $?
  cp gpurun_out/rehearsal_dp.log gpurun_out/rehearsal_dp_cast$v.log
  echo "ST_CAST_SIDE=$v: $(grep -o '"final_loss": [0-9.]*' gpurun_out/rehearsal_dp_cast$v.log)"
done
