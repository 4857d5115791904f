#!/bin/bash
# Grouped vs per-expert MoE weight gradient, same box (Mixtral 4-layer proxy, all experts local).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; tail -n 2 "gpurun_out/$name.log" | cut -c1-220; echo "=== $name rc=$rc"; return $rc; }
step wg_tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_train_gpu.py -k "wgrad_grouped or moe" || exit $?
for r in 1 2; do
  ST_MOE_GROUPED_WGRAD=1 step grouped_$r 300 python bench.py --layout mixtral_ep8 --layers 4 --steps 5 --warmup 2 || exit $?
  ST_MOE_GROUPED_WGRAD=0 step loop_$r 300 python bench.py --layout mixtral_ep8 --layers 4 --steps 5 --warmup 2 || exit $?
done
step q3_grouped 300 python bench.py --model qwen3-30b-a3b --layers 4 --micro_batch_size 2 --steps 5 --warmup 2 || exit $?
ST_MOE_GROUPED_WGRAD=0 step q3_loop 300 python bench.py --model qwen3-30b-a3b --layers 4 --micro_batch_size 2 --steps 5 --warmup 2 || exit $?
step q3_prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_q3 -o run --output-format csv -- python bench.py --model qwen3-30b-a3b --layers 4 --micro_batch_size 2 --steps 4 --warmup 2 || exit $?
step mx_prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_moe -o run --output-format csv -- python bench.py --layout mixtral_ep8 --layers 4 --steps 4 --warmup 2 || exit $?
exit 0
