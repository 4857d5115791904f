#!/bin/bash
# Grouped expert weight gradient on csrc/wgrad4.hip vs the 4-stage grouped kernel: tests,
# microbench, then interleaved Mixtral / Qwen3-30B-A3B proxy rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "wgrad" > gpurun_out/wg4g_tests.log 2>&1 || exit $?
tail -1 gpurun_out/wg4g_tests.log
timeout -k 10 200 python -u tools/bench_wgrad_grouped.py > gpurun_out/wg4g_bench.log 2>&1 || exit $?
cat gpurun_out/wg4g_bench.log
for rnd in 1 2; do
  for v in 1 0; do
    ST_WGRAD_GROUPED4=$v timeout -k 10 200 python bench.py --layout mixtral_ep8 --layers 4 --steps 6 --warmup 2 > gpurun_out/mxw4_v${v}_r${rnd}.log 2>&1 || exit $?
    echo "mixtral grouped4=$v round=$rnd $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/mxw4_v${v}_r${rnd}.log) $(grep -o '"mfu_pct": [0-9.]*' gpurun_out/mxw4_v${v}_r${rnd}.log)"
    ST_WGRAD_GROUPED4=$v timeout -k 10 200 python bench.py --model qwen3-30b-a3b --layers 4 --micro_batch_size 2 --steps 6 --warmup 2 > gpurun_out/q3w4_v${v}_r${rnd}.log 2>&1 || exit $?
    echo "qwen3 grouped4=$v round=$rnd $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/q3w4_v${v}_r${rnd}.log) $(grep -o '"mfu_pct": [0-9.]*' gpurun_out/q3w4_v${v}_r${rnd}.log)"
  done
done
exit 0
