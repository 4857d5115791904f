#!/bin/bash
# Fused gate|up GEMM + SwiGLU epilogue (csrc/gemm4w.hip) vs hipBLASLt + swiglu kernel: numerics,
# then interleaved headline-bench A/B rounds (each step time-limited; first failure ends the run).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "swiglu or gemm4w" > gpurun_out/fused_swiglu_tests.log 2>&1 || exit $?
tail -2 gpurun_out/fused_swiglu_tests.log
for rnd in 1 2; do
  for v in 1 0; do
    ST_MLP_FUSED_SWIGLU=$v timeout -k 10 280 python bench.py --steps 8 --warmup 3 > gpurun_out/fs_v${v}_r${rnd}.log 2>&1 || exit $?
    echo "fused=$v round=$rnd $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fs_v${v}_r${rnd}.log)"
  done
done
exit 0
