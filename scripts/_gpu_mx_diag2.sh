# xGMI EP exchange + ZeRO-1, 8 ranks on one GPU (default xGMI timeout), then the xGMI GPU tests
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0 ST_GPU_OVERSUBSCRIBE=1 OMP_NUM_THREADS=2 ST_MOE_DEBUG=1
( while true; do sleep 50; echo "[diag] alive $(date +%T)"; done ) &
hb=$!
trap 'kill $hb 2>/dev/null' EXIT
mkdir -p gpurun_out
echo "== xgmi + zero1, default timeout"
timeout -k 10 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29961 \
  bench.py --gpus 8 --layout mixtral_ep8 --layers 2 --steps 3 --warmup 1 --backend gloo --ep_comm xgmi > gpurun_out/diag_fence.log 2>&1
echo "rc=$?"; grep -o 'RuntimeError: router call [0-9]*: [0-9]*\|"final_loss": [0-9.a-z]*\|"ep_transport": {[^}]*\|"ms_per_step": [0-9.]*' gpurun_out/diag_fence.log | sort | uniq -c | head -5
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_xgmi_gpu.py -m gpu > gpurun_out/xgmi_tests.log 2>&1; echo "xgmi tests rc=$?"; tail -2 gpurun_out/xgmi_tests.log
exit 0
