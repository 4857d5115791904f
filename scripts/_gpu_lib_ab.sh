# Flash kernel A/B across library variants (ab_libs/*.so vs the default), interleaved.
set -e
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/lib_ab
mkdir -p $O
for r in a b; do
  for v in ${LIBS:-default}; do
    if [ $v = default ]; then L=""; else L=ab_libs/$v.so; fi
    ST_KERNEL_LIB=$L timeout -k 10 200 python tools/bench_flash_shapes.py ${SHAPE_ARGS:-} > $O/${v}_$r.jsonl
    echo "== $v $r"; grep "${PASS:-bwd}" $O/${v}_$r.jsonl | cut -c1-100
  done
done
