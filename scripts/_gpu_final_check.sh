# Final check of the committed tree: GPU suite, smoke, headline bench.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; tail -n 3 "gpurun_out/$name.log" | cut -c1-300; echo "=== $name rc=$rc"; return $rc; }
step gpu_all 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu || exit $?
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
step bench 600 python bench.py --steps 10 --warmup 3 || exit $?
