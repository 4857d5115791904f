# Bisect the tp2pp2dp2 8-rank one-GPU rehearsal hang: RCCL TP transport first, then tp2 x dp4 (no PP) on auto.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 ST_GPU_OVERSUBSCRIBE=1 OMP_NUM_THREADS=2
( while true; do sleep 50; echo "[bisect] alive $(date +%T)"; done ) &
hb=$!
trap 'kill $hb 2>/dev/null' EXIT
echo "== tp2pp2dp2 tp_comm=rccl $(date +%T)"
timeout -k 10 400 python -m torch.distributed.run --nnodes 1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29911 \
  bench.py --gpus 8 --layout tp2pp2dp2 --layers 4 --steps 2 --warmup 1 --backend gloo --tp_comm rccl > gpurun_out/bisect_rccl.log 2>&1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/bisect_rccl.log
echo "== tp2 dp4 tp_comm=auto $(date +%T)"
timeout -k 10 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29912 \
  bench.py --gpus 8 --layout dp --tp 2 --sp --layers 2 --steps 2 --warmup 1 --micro_batch_size 2 --backend gloo > gpurun_out/bisect_tp2dp4.log 2>&1
grep -o '"ms_per_step": [0-9.]*\|"tp_transport": {[^}]*' gpurun_out/bisect_tp2dp4.log | head -3
