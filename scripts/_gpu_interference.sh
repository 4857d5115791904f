# Side-stream interference: kernel traces of the headline step with the
# unfused MLP (default) and the fused gate|up + SwiGLU GEMM, same process image, breakdown +
# which main-stream kernels grow under the side-stream AdamW (tools/trace_overlap.py).
set -e
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/interf
mkdir -p $O
for arm in ${ARMS:-unfused fused fused_np}; do
  F=0; P=1
  [ $arm = fused ] && F=1
  [ $arm = fused_np ] && F=1 && P=0
  echo "== $arm $(date +%T)"
  ST_MLP_FUSED_SWIGLU=$F ST_GEMM4W_PERSIST=$P timeout -k 10 400 rocprofv3 --kernel-trace -d $O/prof_$arm -o run -- python3 bench.py --steps 3 --warmup 2 > $O/bench_$arm.log 2>&1 || { tail -20 $O/bench_$arm.log; exit 1; }
  tail -1 $O/bench_$arm.log
  DB=$(find $O/prof_$arm -name "*results.db" | head -1)
  python tools/rocpd_summary.py $DB --steps 3 --csv $O/kernels_$arm.csv > $O/breakdown_$arm.txt
  python tools/trace_overlap.py $DB --steps 3 > $O/overlap_$arm.txt
  head -20 $O/breakdown_$arm.txt; head -30 $O/overlap_$arm.txt
  rm -rf $O/prof_$arm
done
