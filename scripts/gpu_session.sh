#!/bin/bash
# One GPU-box session: the steps named in $STEPS (space separated), each time-limited;
# the first failure ends the run.  Step names: sp_gemm tests bench prof gmm flash wgrad
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
STEPS=${STEPS:-"tests bench"}
step() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; tail -n 4 "gpurun_out/$name.log" | cut -c1-400; echo "=== $name rc=$rc"; return $rc; }
for s in $STEPS; do
  case $s in
    sp_gemm) step sp_gemm 240 python tools/bench_sp_gemm.py || exit $? ;;
    tests) step gpu_tests 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu || exit $? ;;
    bench) step bench 600 python bench.py --steps 10 --warmup 3 || exit $? ;;
    prof) step step_prof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_step -o run --output-format csv -- python bench.py --steps 3 --warmup 2 || exit $? ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
exit 0
