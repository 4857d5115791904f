#!/bin/bash
# Long-K MoE forward GEMMs on csrc/gemm4w.hip vs the 8-phase grouped kernel: numerics, then
# interleaved Mixtral (and Qwen3-30B-A3B, which stays on the grouped kernel) proxy rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm4w or expert_ffn or grouped" > gpurun_out/moe_g4_tests.log 2>&1 || exit $?
tail -1 gpurun_out/moe_g4_tests.log
for rnd in 1 2; do
  for v in 1 0; do
    ST_MOE_GEMM4W=$v timeout -k 10 200 python bench.py --layout mixtral_ep8 --layers 4 --steps 6 --warmup 2 > gpurun_out/mxg4_v${v}_r${rnd}.log 2>&1 || exit $?
    echo "mixtral gemm4w=$v round=$rnd $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/mxg4_v${v}_r${rnd}.log) $(grep -o '"mfu_pct": [0-9.]*' gpurun_out/mxg4_v${v}_r${rnd}.log)"
  done
done
timeout -k 10 200 python bench.py --model qwen3-30b-a3b --layers 4 --micro_batch_size 2 --steps 6 --warmup 2 > gpurun_out/q3g4.log 2>&1 || exit $?
echo "qwen3 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/q3g4.log) $(grep -o '"mfu_pct": [0-9.]*' gpurun_out/q3g4.log)"
