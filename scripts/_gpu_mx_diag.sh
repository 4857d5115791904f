# Mixtral 8-rank one-GPU rehearsal NaN diagnosis: vary one setting per run (routing checks on).
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0 ST_GPU_OVERSUBSCRIBE=1 OMP_NUM_THREADS=2 ST_MOE_DEBUG=1
( while true; do sleep 50; echo "[diag] alive $(date +%T)"; done ) &
hb=$!
trap 'kill $hb 2>/dev/null' EXIT
mkdir -p gpurun_out
port=29950
for arm in ${ARMS:-"rccl:--ep_comm rccl" "zero0:--ep_comm xgmi --zero 0"}; do
  n=${arm%%:*}; extra=${arm#*:}; port=$((port + 1))
  echo "== $n ($extra)"
  timeout -k 10 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port $port \
    bench.py --gpus 8 --layout mixtral_ep8 --layers 2 --steps 2 --warmup 1 --backend gloo $extra > gpurun_out/diag_$n.log 2>&1
  rc=$?
  echo "rc=$rc"; grep -o 'RuntimeError: router call [0-9]*: [0-9]*\|"final_loss": [0-9.a-z]*' gpurun_out/diag_$n.log | sort | uniq -c | head -3
  [ $rc -eq 124 ] || [ $rc -eq 137 ] && exit $rc
done
exit 0
