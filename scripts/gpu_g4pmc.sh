#!/bin/bash
# PMC passes over the one-wave-per-SIMD GEMM (two tile orders) vs hipBLASLt (dense gate|up shape).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum GRBM_GUI_ACTIVE -d gpurun_out/g4pmc3 -o run --output-format csv -- python tools/_g4prof.py > gpurun_out/g4pmc3.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d gpurun_out/g4pmc4 -o run --output-format csv -- python tools/_g4prof.py > gpurun_out/g4pmc4.log 2>&1 || exit $?
exit 0
