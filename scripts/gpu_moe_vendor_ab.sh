#!/bin/bash
# MoE expert GEMMs: one-launch HIP grouped kernel vs one hipBLASLt GEMM per expert (host counts),
# interleaved A/B on the Mixtral and Qwen3-30B-A3B 4-layer proxies, plus the numerics test.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "expert_ffn" > gpurun_out/moe_vendor_test.log 2>&1 || exit $?
for rnd in 1 2; do
  for v in 0 1; do
    ST_MOE_VENDOR_GEMM=$v timeout -k 10 200 python bench.py --layout mixtral_ep8 --layers 4 --steps 6 --warmup 2 > gpurun_out/mx_v${v}_r${rnd}.log 2>&1 || exit $?
    echo "mx vendor=$v round=$rnd $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/mx_v${v}_r${rnd}.log)"
    ST_MOE_VENDOR_GEMM=$v timeout -k 10 200 python bench.py --model qwen3-30b-a3b --layers 4 --micro_batch_size 2 --steps 6 --warmup 2 > gpurun_out/q3_v${v}_r${rnd}.log 2>&1 || exit $?
    echo "q3 vendor=$v round=$rnd $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/q3_v${v}_r${rnd}.log)"
  done
done
exit 0
