set -e
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/pw1
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash_fwd_pw or rescale_spikes or flash_long_sequence or cp_chunk_at_global" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 200 python tools/bench_flash_shapes.py --no-bwd > $O/base.jsonl
ST_FLASH_FWD=pw timeout -k 10 200 python tools/bench_flash_shapes.py --no-bwd > $O/pw.jsonl
cat $O/base.jsonl $O/pw.jsonl
ST_FLASH_FWD=pwf timeout -k 10 200 python tools/bench_flash_shapes.py --no-bwd > $O/pwf.jsonl
cat $O/pwf.jsonl
