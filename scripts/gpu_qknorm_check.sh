cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k qknorm > gpurun_out/qk_test.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/qk_test.log; exit 1; }
tail -3 gpurun_out/qk_test.log
timeout -k 10 300 python bench.py --model qwen3-0.6b --micro_batch_size 2 --seq_len 2048 --steps 6 --warmup 2 > gpurun_out/q06_fused.log 2>&1 && grep '^{' gpurun_out/q06_fused.log | cut -c1-200
ST_FUSED_QKNORM=0 timeout -k 10 300 python bench.py --model qwen3-0.6b --micro_batch_size 2 --seq_len 2048 --steps 6 --warmup 2 > gpurun_out/q06_unfused.log 2>&1 && grep '^{' gpurun_out/q06_unfused.log | cut -c1-200
