#!/bin/bash
# Alternating A/B of one environment switch on the 1-GPU bench:
#   AB_VAR=ST_SIDE_STREAM_PRIORITY AB_A=0 AB_B=-1 bash scripts/gpu_env_ab.sh
set -u
mkdir -p gpurun_out
for i in 1 2; do
  for v in "$AB_A" "$AB_B"; do
    echo "=== $AB_VAR=$v run $i" >> gpurun_out/env_ab.log
    env "$AB_VAR=$v" timeout -k 10 300 python bench.py --gpus 1 --steps 8 --warmup 2 ${BENCH_ARGS:-} \
        >> gpurun_out/env_ab.log 2>&1 || exit $?
  done
done
