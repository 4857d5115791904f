# Headline micro-batch A/B on one box: 6 (default) vs 7 (fits by the estimate since bf16 moments)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for m in 6 7 6 7; do
  echo "== mbs $m $(date +%T)"
  timeout -k 10 400 python bench.py --steps 10 --warmup 3 --micro_batch_size $m > gpurun_out/mbs_$m.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/mbs_$m.log; exit 1; }
  grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"max_mem_gb": [0-9.]*\|HBM estimate [0-9.]* GB' gpurun_out/mbs_$m.log | tr '\n' ' '; echo
done
