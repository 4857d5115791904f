#!/bin/bash
# Qwen3-30B-A3B proxy: grouped expert wgrad on the 4-stage kernel vs csrc/wgrad4.hip persistent /
# one unit per workgroup; Mixtral proxy with the non-persistent grid.  Interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
q3() {
  local tag=$1 rnd=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --model qwen3-30b-a3b --layers 4 --micro_batch_size 2 --steps 6 --warmup 2 > gpurun_out/q3p_${tag}_r${rnd}.log 2>&1 || exit $?
  echo "qwen3 $tag round=$rnd $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/q3p_${tag}_r${rnd}.log)"
}
for rnd in 1 2; do
  q3 4stage $rnd ST_WGRAD_GROUPED4=0
  q3 w4_persist $rnd ST_WGRAD_GROUPED4=1 ST_WGRAD4_GROUPED_PERSIST=1
  q3 w4_units $rnd ST_WGRAD_GROUPED4=1 ST_WGRAD4_GROUPED_PERSIST=0
  ST_WGRAD_GROUPED4=1 ST_WGRAD4_GROUPED_PERSIST=0 timeout -k 10 200 python bench.py --layout mixtral_ep8 --layers 4 --steps 6 --warmup 2 > gpurun_out/mxp_units_r${rnd}.log 2>&1 || exit $?
  echo "mixtral w4_units round=$rnd $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/mxp_units_r${rnd}.log)"
done
exit 0
