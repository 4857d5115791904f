# Mixtral EP8 slice variants (micro-batch x expert GEMM path) + both pipeline stages of tp2pp2dp2.
set -e
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/slices
mkdir -p $O
run() {  # name, env..., -- bench args
  local n=$1; shift
  echo "== $n $(date +%T)"
  timeout -k 10 420 env "$@" > $O/$n.json 2> $O/$n.err || { tail -30 $O/$n.err; exit 1; }
  tail -1 $O/$n.json | python -c "import json,sys; r=json.loads(sys.stdin.read()); print({k: r[k] for k in ('ms_per_step','mfu_pct_per_rank_upper_bound','peak_hbm_gb','hbm_estimate_gb','hbm_estimate_err_pct','hbm_estimate_8gpu_worst_rank_gb')})"
}
for V in ${VARIANTS:-mb1_vendor mb2_vendor mb2_grouped mb1_grouped}; do
  mb=${V%%_*}; mb=${mb#mb}; ga=$((2 / mb)); g=auto; [ "${V#*_}" = grouped ] && g=0
  run mixtral_$V ST_MOE_VENDOR_GEMM=$g python bench.py --layout mixtral_ep8 --slice --micro_batch_size $mb --grad_acc $ga --steps 3 --warmup 2
done
if [ "${PP:-1}" = "1" ]; then
  run tp2pp2dp2_first python bench.py --layout tp2pp2dp2 --slice --slice_stage first --steps 2 --warmup 2
  run tp2pp2dp2 python bench.py --layout tp2pp2dp2 --slice --steps 3 --warmup 2
fi
