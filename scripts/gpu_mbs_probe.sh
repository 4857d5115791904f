#!/bin/bash
# SwiGLU-activation recompute: same-box A/B at micro-batch 6, then micro-batch 7 / 8 (memory + speed).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; grep -E '^\{' "gpurun_out/$name.log" | python3 -c "import json,sys; [print(d['ms_per_step'], d['value'], d['mfu_pct'], d['max_mem_gb']) for d in map(json.loads, sys.stdin)]"; tail -n 2 "gpurun_out/$name.log" | cut -c1-200; echo "=== $name rc=$rc"; return $rc; }
step swiglu_tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_train_gpu.py tests/test_kernels_gpu.py -k "swiglu or mlp or train_step or parity" || exit $?
step mbs6_recompute 400 python bench.py --steps 8 --warmup 3 || exit $?
ST_MLP_RECOMPUTE_ACT=0 step mbs6_keep 400 python bench.py --steps 8 --warmup 3 || exit $?
step mbs7_recompute 400 python bench.py --steps 8 --warmup 3 --micro_batch_size 7 || exit $?
ST_HBM_HEADROOM_GB=4 step mbs8_recompute 400 python bench.py --steps 8 --warmup 3 --micro_batch_size 8 || exit $?
exit 0
