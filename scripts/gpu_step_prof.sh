#!/bin/bash
# Kernel trace of the headline step (Llama-3-8B, mbs 6) + a short bench, for profiles/r03.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; tail -n 3 "gpurun_out/$name.log" | cut -c1-300; echo "=== $name rc=$rc"; return $rc; }
step bench 600 python bench.py --steps 10 --warmup 3 || exit $?
step step_prof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_step -o run --output-format csv -- python bench.py --steps 3 --warmup 2 || exit $?
exit 0
