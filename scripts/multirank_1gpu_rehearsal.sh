#!/bin/bash
# Rehearse the multi-rank bench path (RCCL, ZeRO-1 reduce-scatter / all-gather,
# forward pre-hook waits) with 2 ranks sharing ONE GPU, on a 2-layer Llama-3-8B
# (result marked invalid: debug only).  RCCL may refuse two ranks on one device;
# then the gloo leg still exercises the arena / hook logic on GPU tensors.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 ST_GPU_OVERSUBSCRIBE=1
# RCCL refuses two ranks on one device ("Duplicate GPU detected"), so the rehearsal
# uses gloo on GPU tensors: same arenas, hooks, ZeRO-1 shards and stream ordering.
for zero in 1 0; do
  echo "=== gloo zero=$zero"
  timeout -k 10 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $((29700 + zero)) bench.py --gpus 2 --steps 3 --warmup 1 --layers 2 --seq_len 2048 --zero $zero \
    --backend gloo > gpurun_out/rehearsal_gloo_z$zero.log 2>&1
  rc=$?
  echo "rc=$rc"; grep -E "metric|Error" gpurun_out/rehearsal_gloo_z$zero.log | tail -3
  [ $rc -eq 124 ] || [ $rc -eq 137 ] && exit $rc
done
exit 0
