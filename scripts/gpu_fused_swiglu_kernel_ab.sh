#!/bin/bash
# Fused gate|up + SwiGLU in the headline step by kernel: unfused (hipBLASLt + swiglu pass) vs the
# fused kind-5 kernel persistent (e), kind 5 one tile per workgroup (e, ST_GEMM4W_PERSIST=0) and
# the stream-persistent kind 6 (f).  Interleaved rounds; first failure ends the run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
  local tag=$1 rnd=$2; shift 2
  env "$@" timeout -k 10 280 python bench.py --steps 8 --warmup 3 > gpurun_out/fk_${tag}_r${rnd}.log 2>&1 || exit $?
  echo "$tag round=$rnd $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fk_${tag}_r${rnd}.log)"
}
for rnd in 1 2; do
  run unfused $rnd ST_MLP_FUSED_SWIGLU=0
  run fused_e_persist $rnd ST_MLP_FUSED_SWIGLU=1 ST_GEMM4W_SWIGLU_KERNEL=e ST_GEMM4W_PERSIST=1
  run fused_e_tiles $rnd ST_MLP_FUSED_SWIGLU=1 ST_GEMM4W_SWIGLU_KERNEL=e ST_GEMM4W_PERSIST=0
  run fused_f $rnd ST_MLP_FUSED_SWIGLU=1 ST_GEMM4W_SWIGLU_KERNEL=f
done
exit 0
