# Static s_setprio in the flash forward: default vs odd-workgroup priority; 8-wave ping-pong vs its priority variant.
set -e
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/prio
mkdir -p $O
for r in a b; do
  for arm in "def::0" "odd:ab_libs/prio_ODD.so:0" "pp::1" "pp_prio:ab_libs/prio_PP.so:1"; do
    n=${arm%%:*}; rest=${arm#*:}; L=${rest%%:*}; PPV=${rest#*:}
    ST_KERNEL_LIB=$L ST_FLASH_PP=$PPV timeout -k 10 200 python tools/bench_flash_shapes.py --no-bwd > $O/${n}_$r.jsonl
    echo "== $n $r"; grep '"fwd"' $O/${n}_$r.jsonl | cut -c1-100
  done
done
