# xGMI EP exchange + ZeRO-1, 8 ranks on one GPU: where the first non-finite value appears
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0 ST_GPU_OVERSUBSCRIBE=1 OMP_NUM_THREADS=2 ST_MOE_DEBUG=1 ST_DEBUG_FINITE=1
( while true; do sleep 50; echo "[diag] alive $(date +%T)"; done ) &
hb=$!
trap 'kill $hb 2>/dev/null' EXIT
mkdir -p gpurun_out
echo "== xgmi + zero1"
timeout -k 10 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29961 \
  bench.py --gpus 8 --layout mixtral_ep8 --layers 2 --steps 2 --warmup 1 --backend gloo --ep_comm xgmi > gpurun_out/diag_finite.log 2>&1
echo "rc=$?"; grep '^\[finite\]' gpurun_out/diag_finite.log | sort | head -40
exit 0
