#!/bin/bash
# One GPU-box session: kernel numerics -> smoke -> short bench -> rocprof stats.
# Each GPU step has its own time limit; a crash/timeout (exit >1) stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
STEPS=${STEPS:-8}
WARMUP=${WARMUP:-2}
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/summary.log
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/summary.log
  tail -5 "gpurun_out/$name.log" | tee -a gpurun_out/summary.log
  return $rc
}
rc_ok() { [ "$1" -le 1 ]; }
run pytest_gpu 900 python -m pytest tests -x -q -m gpu; rc=$?; rc_ok $rc || exit $rc
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"; rc=$?; rc_ok $rc || exit $rc
run bench 900 python bench.py --gpus 1 --steps "$STEPS" --warmup "$WARMUP"; rc=$?; rc_ok $rc || exit $rc
if [ "${PROFILE:-1}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
  run rocprof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
      python bench.py --gpus 1 --steps 3 --warmup 1; rc=$?
fi
exit 0
