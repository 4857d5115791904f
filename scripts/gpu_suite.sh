#!/bin/bash
# Full GPU test suite + grouped-GEMM microbench + q3 proxy profile (each step time-limited).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; tail -n 3 "gpurun_out/$name.log" | cut -c1-300; echo "=== $name rc=$rc"; return $rc; }
step gmm_tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_train_gpu.py -k "grouped or moe" || exit $?
step gmm_bench 300 python tools/bench_grouped_gemm.py || exit $?
step mx_proxy 300 python bench.py --layout mixtral_ep8 --layers 4 --steps 5 --warmup 2 || exit $?
step q3_proxy 300 python bench.py --model qwen3-30b-a3b --layers 4 --micro_batch_size 2 --steps 5 --warmup 2 || exit $?
step q3_prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_q3 -o run --output-format csv -- python bench.py --model qwen3-30b-a3b --layers 4 --micro_batch_size 2 --steps 4 --warmup 2 || exit $?
step gpu_all 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu || exit $?
exit 0
