set -e
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/pw2
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash_fwd_pw or rescale_spikes" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in base pw pwf; do
  if [ $v = base ]; then unset ST_FLASH_FWD; else export ST_FLASH_FWD=$v; fi
  timeout -k 10 200 python tools/bench_flash_shapes.py --no-bwd --shapes bench,cp8_32k_r3 > $O/$v.jsonl
  echo $v; cat $O/$v.jsonl
done
unset ST_FLASH_FWD
PROF=0 STEPS=3 WARMUP=2 bash scripts/_gpu_slices.sh
