# Non-temporal dS stores/loads in the dS-materialising flash backward: kernel A/B + step A/B.
set -e
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/nt
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash and (bwd or backward)" > $O/tests0.log 2>&1 || { tail -30 $O/tests0.log; exit 1; }
ST_FLASH_DS_NT=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash and (bwd or backward)" > $O/tests1.log 2>&1 || { tail -30 $O/tests1.log; exit 1; }
tail -1 $O/tests0.log; tail -1 $O/tests1.log
for r in a b; do
  for v in 0 1; do
    ST_FLASH_DS_NT=$v timeout -k 10 200 python tools/bench_flash_shapes.py > $O/shapes_${v}_$r.jsonl
    echo "== nt=$v $r"; grep '"bwd"' $O/shapes_${v}_$r.jsonl | cut -c1-120
  done
done
STEPS=10 ARMS="n0:ST_FLASH_DS_NT=0 n1:ST_FLASH_DS_NT=1 n0b:ST_FLASH_DS_NT=0 n1b:ST_FLASH_DS_NT=1" bash scripts/_gpu_env_ab.sh
