#!/bin/bash
# Single-GPU bench sweep: CFGS="--micro_batch_size 4;--micro_batch_size 2 --grad_acc 2" bash scripts/sweep_micro_batch.sh
# Appends each bench JSON to gpurun_out/sweep.log; stops at the first failing config.
set -u
mkdir -p gpurun_out
IFS=";" read -ra LIST <<< "${CFGS:---micro_batch_size 4}"
for cfg in "${LIST[@]}"; do
  echo "=== $cfg" >> gpurun_out/sweep.log
  timeout -k 10 300 python bench.py --gpus 1 --steps 6 --warmup 2 $cfg >> gpurun_out/sweep.log 2>&1 || exit $?
done
