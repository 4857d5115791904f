#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; grep -v "^{" "gpurun_out/$name.log" | tail -n 12 | cut -c1-330; echo "=== $name rc=$rc"; return $rc; }
step gmm_tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_train_gpu.py -k "grouped or moe or swiglu_linear" || exit $?
ST_GMM_ORDER=1 step gmm_bench_order1 300 python tools/bench_grouped_gemm.py || exit $?
ST_GMM_ORDER=0 step gmm_bench_order0 300 python tools/bench_grouped_gemm.py || exit $?
step wgrad_layouts 300 python tools/bench_wgrad_layouts.py || exit $?
exit 0
