# tp2pp2dp2 per-stage slices with the even split and with an uneven chunk distribution.
set -e
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/pp_balance
mkdir -p $O
for D in even 9,8,8,7; do
  for S in first last; do
    n=${D//,/_}_$S
    extra=""; [ $D != even ] && extra="--layer_distribution $D"
    echo "== $n $(date +%T)"
    timeout -k 10 420 python bench.py --layout tp2pp2dp2 --slice --slice_stage $S --steps 3 --warmup 2 $extra > $O/$n.json 2> $O/$n.err || { tail -30 $O/$n.err; exit 1; }
    tail -1 $O/$n.json | python -c "import json,sys; r=json.loads(sys.stdin.read()); print({k: r.get(k) for k in ('layers_on_rank','ms_per_step','peak_hbm_gb','hbm_estimate_gb','hbm_estimate_err_pct')})"
  done
done
