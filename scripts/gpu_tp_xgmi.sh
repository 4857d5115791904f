#!/bin/bash
# tp 4 / 8 xGMI transport: same-GPU multi-process decoder-layer tests + 8-rank 1-GPU rehearsal
# of the reference's Qwen3-32B TP8 rows (auto transport, production-sized IPC areas).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; tail -n 3 "gpurun_out/$name.log" | cut -c1-300; echo "=== $name rc=$rc"; return $rc; }
step tp_xgmi_tests 600 python -u -m pytest -v --timeout 400 --timeout-method thread tests/test_xgmi_gpu.py -k "tp_decoder or sp_decoder or ipc" || exit $?
step tp8_rehearsal 900 python -u scripts/bench_reference_rows_8gpu.py --rehearse --filter "qwen3-32b-(sp-)?tp8-mbs1-ga1-s2048$" --steps 2 --warmup 1 --timeout 300 --out gpurun_out/rehearsal_tp8.jsonl || exit $?
exit 0
