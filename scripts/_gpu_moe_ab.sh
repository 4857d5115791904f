# Mixtral EP8 slice A/B over environment settings: ARMS="name:VAR=val,VAR=val ..." (mb1 unless MB=2)
set -e
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/moe_ab
mkdir -p $O
MB=${MB:-1}
for arm in ${ARMS:-base:ST_MOE_BWD_OVERLAP=0 overlap:ST_MOE_BWD_OVERLAP=1}; do
  n=${arm%%:*}; envs=${arm#*:}
  echo "== $n ($envs) $(date +%T)"
  timeout -k 10 420 env ${envs//,/ } python bench.py --layout mixtral_ep8 --slice --micro_batch_size $MB --grad_acc $((2 / MB)) --steps ${STEPS:-4} --warmup 2 > $O/$n.json 2> $O/$n.err || { tail -30 $O/$n.err; exit 1; }
  tail -1 $O/$n.json | python -c "import json,sys; r=json.loads(sys.stdin.read()); print({k: r[k] for k in ('ms_per_step','mfu_pct_per_rank_upper_bound','peak_hbm_gb')})"
done
