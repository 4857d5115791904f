#!/bin/bash
# Flash backward with dQ on a second stream beside dK/dV: numerics, then a same-process step A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; tail -n 6 "gpurun_out/$name.log" | cut -c1-300; echo "=== $name rc=$rc"; return $rc; }
ST_FLASH_BWD_CONCURRENT=1 step flash_tests_conc 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash or attn" || exit $?
step ab_flash_conc 900 python tools/ab_step.py --variants ST_FLASH_BWD_CONCURRENT=0,ST_FLASH_BWD_CONCURRENT=1 --rounds 4 --steps 3 --micro_batch_size 6 --fused_head 1 || exit $?
exit 0
