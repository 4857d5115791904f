#!/bin/bash
# Weight gradients on a side stream (ST_WGRAD_STREAM=side) vs the compute stream: numerics + step A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; tail -n 6 "gpurun_out/$name.log" | cut -c1-300; echo "=== $name rc=$rc"; return $rc; }
ST_WGRAD_STREAM=side step train_tests_side 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_train_gpu.py || exit $?
step ab_wgrad_side 900 python tools/ab_step.py --variants ST_WGRAD_STREAM=main,ST_WGRAD_STREAM=side --rounds 4 --steps 3 --micro_batch_size 6 --fused_head 1 || exit $?
exit 0
