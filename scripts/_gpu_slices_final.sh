# Final per-rank slices (current defaults) with the resident-memory fields, incl. the first PP stage.
set -e
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/slices_final
mkdir -p $O
for spec in dp tp2pp2dp2 tp2pp2dp2:first cp8_32k mixtral_ep8; do
  L=${spec%%:*}; S=last; [ "$spec" != "$L" ] && S=${spec#*:}
  n=$L; [ $S = first ] && n=${L}_first
  echo "== $n $(date +%T)"
  timeout -k 10 420 python bench.py --layout $L --slice --slice_stage $S --steps ${STEPS:-3} --warmup 2 > $O/$n.json 2> $O/$n.err || { tail -30 $O/$n.err; exit 1; }
  tail -1 $O/$n.json | python -c "import json,sys; r=json.loads(sys.stdin.read()); print({k: r.get(k) for k in ('ms_per_step','mfu_pct_per_rank_upper_bound','peak_hbm_gb','hbm_estimate_gb','hbm_estimate_err_pct','hbm_after_build_gb','hbm_resident_between_steps_gb','hbm_estimate_resident_gb')})"
done
