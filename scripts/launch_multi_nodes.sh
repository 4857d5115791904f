#!/bin/bash
# Multi-node launcher (reference: scripts/torch_dist/launch_multi_nodes.sh).
#
#   NODE_LIST=node_list.txt scripts/launch_multi_nodes.sh [NPROC_PER_NODE] -- <train.py args...>
#
# node_list.txt: one hostname per line, the first is the rendezvous master.
# ssh-fans out one torchrun per node (static rendezvous: node_rank = line
# number), writes per-node logs under $LOG_DIR, and forwards SIGINT/SIGTERM to
# every remote job so a cancelled launch does not leave ranks holding GPUs.
set -euo pipefail
NPROC=${1:-8}
shift || true
[ "${1:-}" = "--" ] && shift
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
NODE_LIST=${NODE_LIST:-node_list.txt}
LOG_DIR=${LOG_DIR:-$ROOT/work_dir/logs}
PORT=${MASTER_PORT:-29500}
mapfile -t NODES < <(grep -v '^\s*#' "$NODE_LIST" | grep -v '^\s*$')
NNODES=${#NODES[@]}
[ "$NNODES" -ge 1 ] || { echo "no nodes in $NODE_LIST" >&2; exit 1; }
MASTER=${NODES[0]}
mkdir -p "$LOG_DIR"
PIDS=()
cleanup() {
  echo "stopping remote jobs..." >&2
  for n in "${NODES[@]}"; do
    ssh -o BatchMode=yes "$n" "pkill -INT -u \$(id -u) -f 'torch.distributed.run.*--master-port $PORT'" 2>/dev/null || true
  done
  for p in "${PIDS[@]}"; do kill "$p" 2>/dev/null || true; done
}
trap cleanup INT TERM
ARGS=$(printf ' %q' "$@")
for i in "${!NODES[@]}"; do
  n=${NODES[$i]}
  ssh -o BatchMode=yes "$n" "cd $ROOT && HSA_ENABLE_IPC_MODE_LEGACY=0 TORCH_NCCL_ASYNC_ERROR_HANDLING=1 \
    python -m torch.distributed.run --nnodes=$NNODES --node-rank=$i --nproc-per-node=$NPROC \
    --master-addr $MASTER --master-port $PORT $ROOT/train.py $ARGS" > "$LOG_DIR/node_${i}_${n}.log" 2>&1 &
  PIDS+=($!)
done
rc=0
for p in "${PIDS[@]}"; do wait "$p" || rc=$?; done
exit $rc
