# Per-rank slice A/B over environment settings, same box: LAYOUT=dp ARMS="name:VAR=val,..."
set -e
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/slice_ab
mkdir -p $O
for arm in $ARMS; do
  n=${arm%%:*}; envs=${arm#*:}
  echo "== $n ($envs) $(date +%T)"
  timeout -k 10 420 env ${envs//,/ } python bench.py --layout ${LAYOUT:-dp} --slice --steps ${STEPS:-4} --warmup 2 > $O/$n.json 2> $O/$n.err || { tail -30 $O/$n.err; exit 1; }
  tail -1 $O/$n.json | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['ms_per_step'], r['mfu_pct_per_rank_upper_bound'])"
done
