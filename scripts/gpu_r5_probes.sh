#!/bin/bash
# Round-5 measurements: CP chunk-shape backward A/B (two-phase dS vs one-shot) and the
# in-step upper bound of producer-written transposed wgrad operands (ST_WGRAD_TN_PROBE).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; tail -n 3 "gpurun_out/$name.log" | cut -c1-400; echo "=== $name rc=$rc"; return $rc; }
step cp_flash_bwd_ab 400 python -u tools/bench_cp_flash_bwd.py || exit $?
step wgrad_tn_probe_ab 600 python -u tools/ab_step.py --variants ST_WGRAD_TN_PROBE=0,ST_WGRAD_TN_PROBE=1 --rounds 3 --steps 3 --micro_batch_size 6 --fused_head 1 --opt_state_dtype bf16 --gemm_tuning use || exit $?
exit 0
