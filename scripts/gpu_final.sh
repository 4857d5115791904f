#!/bin/bash
# Round-end check on one GPU: full GPU test suite, the headline bench, and a kernel trace of
# the headline step (each step time-limited; the first failure ends the run).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; tail -n 3 "gpurun_out/$name.log" | cut -c1-300; echo "=== $name rc=$rc"; return $rc; }
step gpu_all 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu || exit $?
step bench 600 python bench.py --steps 10 --warmup 3 || exit $?
step step_prof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_step -o run --output-format csv -- python bench.py --steps 3 --warmup 2 || exit $?
exit 0
