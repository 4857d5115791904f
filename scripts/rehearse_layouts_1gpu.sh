#!/bin/bash
# Rehearse the 8-GPU bench layouts (bench.py --layout) with 8 ranks sharing ONE MI355X:
# gloo on GPU tensors (RCCL refuses two ranks on one device), 2 decoder layers (result
# marked invalid), real sequence lengths -- so the HIP kernels run on the per-rank shapes
# of each layout (CP8@32K: 4K-query zig-zag chunks at global offsets up to 28K; EP8: one
# expert per rank through the grouped GEMMs; TP2xPP2xDP2: SP + 1F1B + ZeRO-1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 ST_GPU_OVERSUBSCRIBE=1 OMP_NUM_THREADS=2
LAYOUTS=${LAYOUTS:-"tp2pp2dp2 cp8_32k mixtral_ep8 dp"}
port=29810
# heartbeat: a layout can run minutes without printing (gpurun kills silent commands)
( while true; do sleep 50; echo "[rehearse] alive $(date +%T)"; done ) &
hb=$!
trap 'kill $hb 2>/dev/null' EXIT
for lay in $LAYOUTS; do
  port=$((port + 1))
  echo "=== layout $lay"
  layers=2; [ "$lay" = tp2pp2dp2 ] && layers=4  # 2 pipeline stages x 2 interleaved chunks
  timeout -k 10 ${LAYOUT_TIMEOUT:-300} python -m torch.distributed.run --nnodes 1 --nproc-per-node 8 \
    --master-addr 127.0.0.1 --master-port $port bench.py --gpus 8 --layout "$lay" --layers $layers --steps 2 --warmup 1 \
    --backend gloo ${EXTRA:-} > "gpurun_out/rehearsal_$lay.log" 2>&1
  rc=$?
  echo "rc=$rc"; grep -E "HBM estimate|metric|Error|error" "gpurun_out/rehearsal_$lay.log" | head -5
  [ $rc -eq 0 ] || exit $rc
done
exit 0
