#!/bin/bash
# Elementwise-kernel check: numerics, isolated bandwidth, then the headline step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "swiglu or rmsnorm" > gpurun_out/elt_test.log 2>&1 || { tail -30 gpurun_out/elt_test.log; exit 1; }
tail -1 gpurun_out/elt_test.log
timeout -k 10 300 python tools/bench_kernels.py --only elt --no-ref > gpurun_out/elt_bench.log 2>&1 || { tail -20 gpurun_out/elt_bench.log; exit 1; }
grep -i "gbps\|swiglu\|rms" gpurun_out/elt_bench.log | head -20
timeout -k 10 600 python bench.py --steps 8 --warmup 2 ${BENCH_ARGS:-} > gpurun_out/elt_step.log 2>&1 && grep '^{' gpurun_out/elt_step.log | cut -c1-220
