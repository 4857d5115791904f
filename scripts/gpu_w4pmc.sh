#!/bin/bash
# PMC passes (one counter group per run, kernel trace only) over wgrad4 / the 8-phase kernel /
# hipBLASLt at the gate|up weight-gradient shape.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/w4pmc1 -o run --output-format csv -- python tools/_w4prof.py > gpurun_out/w4pmc1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d gpurun_out/w4pmc2 -o run --output-format csv -- python tools/_w4prof.py > gpurun_out/w4pmc2.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d gpurun_out/w4pmc3 -o run --output-format csv -- python tools/_w4prof.py > gpurun_out/w4pmc3.log 2>&1 || exit $?
exit 0
