# Per-rank compute slices of the four 8-GPU BASELINE layouts on one GPU (bench.py --slice),
# then a kernel-trace breakdown of each.
set -e
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/slices
mkdir -p $O
for L in $([ "${SKIP_RUN:-0}" = "1" ] || echo ${SLICES:-dp tp2pp2dp2 cp8_32k mixtral_ep8}); do
  echo "== slice $L $(date +%T)"
  timeout -k 10 420 python bench.py --layout $L --slice --steps ${STEPS:-3} --warmup ${WARMUP:-2} > $O/$L.json 2> $O/$L.err || { tail -30 $O/$L.err; exit 1; }
  tail -1 $O/$L.json
done
if [ "${PROF:-1}" = "1" ]; then
  for L in ${SLICES:-dp tp2pp2dp2 cp8_32k mixtral_ep8}; do
    echo "== prof $L $(date +%T)"
    timeout -k 10 420 rocprofv3 --kernel-trace -d $O/prof_$L -o run -- python3 bench.py --layout $L --slice --steps 2 --warmup 1 > $O/prof_$L.log 2>&1 || { tail -20 $O/prof_$L.log; exit 1; }
    DB=$(ls $O/prof_$L/*/run_results.db 2>/dev/null | head -1 || true)
    [ -z "$DB" ] && DB=$(find $O/prof_$L -name "*results.db" | head -1)
    python tools/rocpd_summary.py $DB --steps 2 --csv $O/kernels_$L.csv > $O/breakdown_$L.txt || true
    head -25 $O/breakdown_$L.txt
    rm -rf $O/prof_$L
  done
fi
