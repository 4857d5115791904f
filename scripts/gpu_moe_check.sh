#!/bin/bash
# MoE session on one GPU: grouped-wgrad + expert numerics, then the Mixtral and
# Qwen3-30B-A3B 4-layer proxies (all experts local) and a kernel trace of the Mixtral one.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; tail -n 4 "gpurun_out/$name.log"; echo "=== $name rc=$rc"; return $rc; }
step moe_tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_train_gpu.py -k "wgrad_grouped or moe or embedding" || exit $?
step mixtral_proxy 600 python bench.py --layout mixtral_ep8 --layers 4 --steps 5 --warmup 2 || exit $?
step mixtral_proxy_mbs4 600 python bench.py --layout mixtral_ep8 --layers 4 --steps 5 --warmup 2 --micro_batch_size 4 || exit $?
step qwen3moe_proxy 600 python bench.py --model qwen3-30b-a3b --layers 4 --micro_batch_size 2 --steps 5 --warmup 2 || exit $?
step moe_prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_moe -o run --output-format csv -- python bench.py --layout mixtral_ep8 --layers 4 --steps 4 --warmup 2 || exit $?
exit 0
