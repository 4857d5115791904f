#!/bin/bash
# Single-node launcher (reference: scripts/torch_dist/launch_single_node.sh).
#
#   scripts/launch_single_node.sh [NPROC] -- <train.py args...>
#
# * one process per GPU via torchrun on 127.0.0.1, RCCL over xGMI;
# * a lock file keeps two jobs from sharing the node's GPUs;
# * --max-restarts (default 0, env MAX_RESTARTS) + --auto_resume turns a
#   watchdog exit (75) or a crashed rank into a resume from the newest checkpoint.
set -euo pipefail
NPROC=${1:-8}
shift || true
[ "${1:-}" = "--" ] && shift
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
LOCK="${LOCK_FILE:-/tmp/scaletorch_amd_node.lock}"
PORT="${MASTER_PORT:-29500}"
exec 9>"$LOCK"
if ! flock -n 9; then
  echo "another scaletorch_amd job holds $LOCK; refusing to oversubscribe the GPUs" >&2
  exit 1
fi
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TORCH_NCCL_ASYNC_ERROR_HANDLING=${TORCH_NCCL_ASYNC_ERROR_HANDLING:-1}
export OMP_NUM_THREADS=${OMP_NUM_THREADS:-8}
python -m torch.distributed.run --nnodes=1 --nproc-per-node="$NPROC" \
  --master-addr 127.0.0.1 --master-port "$PORT" --max-restarts "${MAX_RESTARTS:-0}" \
  "$ROOT/train.py" "$@"
