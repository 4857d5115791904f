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
if has kernels; then run pytest_kernels 600 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu; rc=$?; rc_ok $rc || exit $rc; fi
if has train; then HIP_LAUNCH_BLOCKING=1 run pytest_train 400 python -m pytest tests/test_train_gpu.py -x -q -m gpu; rc=$?; rc_ok $rc || exit $rc; fi
if has smoke; then run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"; rc=$?; [ $rc -eq 0 ] || exit $rc; fi
if has bench; then run bench 900 python bench.py --gpus 1 --steps "$STEPS" --warmup "$WARMUP" ${BENCH_ARGS:-}; rc=$?; [ $rc -eq 0 ] || exit $rc; fi
if has prof; then
  export TMPDIR=/tmp
  run rocprof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
      python bench.py --gpus 1 --steps 3 --warmup 1 ${BENCH_ARGS:-}; rc=$?
fi
exit 0
