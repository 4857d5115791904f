#!/bin/bash
# 8-phase grouped expert GEMM: numerics tests, microbench (8-phase vs 2-phase arms in one
# process) and the MoE proxies with the 8-phase kernel vs ST_GMM_8PHASE=0.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; tail -n 3 "gpurun_out/$name.log" | cut -c1-300; echo "=== $name rc=$rc"; return $rc; }
step gmm_tests 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_train_gpu.py -k "grouped or moe or expert" || exit $?
step gmm_bench 300 python -u tools/bench_grouped_gemm.py || exit $?
step mx_proxy_8ph 300 python -u bench.py --layout mixtral_ep8 --layers 4 --steps 5 --warmup 2 || exit $?
step mx_proxy_2ph 300 env ST_GMM_8PHASE=0 python -u bench.py --layout mixtral_ep8 --layers 4 --steps 5 --warmup 2 || exit $?
step q3_proxy_8ph 300 python -u bench.py --model qwen3-30b-a3b --layers 4 --micro_batch_size 2 --steps 5 --warmup 2 || exit $?
step q3_proxy_2ph 300 env ST_GMM_8PHASE=0 python -u bench.py --model qwen3-30b-a3b --layers 4 --micro_batch_size 2 --steps 5 --warmup 2 || exit $?
exit 0
