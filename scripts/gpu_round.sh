#!/bin/bash
# One GPU-box session: kernel numerics -> integration tests -> smoke -> short bench -> rocprof stats.
# Each GPU step has its own time limit; a crash/timeout (exit > 1) stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
STEPS=${STEPS:-8}
WARMUP=${WARMUP:-2}
STAGES=${STAGES:-"kernels train smoke bench prof"}
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/summary.log
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/summary.log
  tail -15 "gpurun_out/$name.log" | tee -a gpurun_out/summary.log
  return $rc
}
has() { [[ " $STAGES " == *" $1 "* ]]; }
rc_ok() { [ "$1" -eq 0 ]; }
if has kernels; then run pytest_kernels 600 python -m pytest tests/test_kernels_gpu.py tests/test_xgmi_gpu.py -x -q -m gpu; rc=$?; rc_ok $rc || exit $rc; fi
if has train; then HIP_LAUNCH_BLOCKING=1 run pytest_train 400 python -m pytest tests/test_train_gpu.py -x -q -m gpu; rc=$?; rc_ok $rc || exit $rc; fi
if has smoke; then run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"; rc=$?; [ $rc -eq 0 ] || exit $rc; fi
if has bench; then run bench 900 python bench.py --gpus 1 --steps "$STEPS" --warmup "$WARMUP" ${BENCH_ARGS:-}; rc=$?; [ $rc -eq 0 ] || exit $rc; fi
if has opt; then run optimize_mfu 900 python tools/optimize_mfu.py --rounds 3 --steps 3; rc=$?; [ $rc -eq 0 ] || exit $rc; fi
if has prof; then
  export TMPDIR=/tmp
  run rocprof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
      python bench.py --gpus 1 --steps 3 --warmup 1 ${BENCH_ARGS:-}; rc=$?
  [ $rc -eq 0 ] || exit $rc
fi
if has pmc; then
  # hardware counters: one rocprofv3 run per counter group, --pmc with --kernel-trace only
  export TMPDIR=/tmp
  KB="python3 tools/bench_kernels.py --only attn,elt --no-ref --iters 3"
  run pmc_mfma 240 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16 \
      -d gpurun_out/pmc_mfma -o run --output-format csv -- $KB || exit $?
  run pmc_lds 240 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
      -d gpurun_out/pmc_lds -o run --output-format csv -- $KB || exit $?
  # (derived FETCH_SIZE/WRITE_SIZE hung rocprofv3 on this pool: raw TCC request counts instead)
  run pmc_hbm 240 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum \
      -d gpurun_out/pmc_hbm -o run --output-format csv -- $KB || exit $?
  run pmc_step 400 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16 \
      -d gpurun_out/pmc_step -o run --output-format csv -- python3 bench.py --gpus 1 --steps 1 --warmup 1 || exit $?
fi
exit 0
