# Headline bench A/B over environment settings, same box: ARMS="name:VAR=val,VAR=val ..."
set -e
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/env_ab
mkdir -p $O
for arm in $ARMS; do
  n=${arm%%:*}; envs=${arm#*:}
  echo "== $n ($envs) $(date +%T)"
  timeout -k 10 300 env ${envs//,/ } python bench.py --steps ${STEPS:-10} --warmup 3 ${BENCH_ARGS:-} > $O/$n.json 2> $O/$n.err || { tail -30 $O/$n.err; exit 1; }
  tail -1 $O/$n.json | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['ms_per_step'], r['value'])"
done
