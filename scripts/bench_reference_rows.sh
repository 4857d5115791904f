#!/bin/bash
# The reference's single-device table (README.md:30-36 of the
# reference: Qwen3 0.6B / 1.7B / 4B on 1x Ascend 910B) re-run on ONE MI355X with
# the same model, micro-batch, sequence length and activation checkpointing.
# Our timing is the FULL step (incl. clip + AdamW), the reference's was fwd+bwd.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/reference_rows.jsonl
: > $OUT
run() {  # model mbs seq gc ref_tok_s
  local extra=""; [ "$4" = "1" ] && extra="--gc"
  timeout -k 10 600 python bench.py --model "$1" --micro_batch_size "$2" --seq_len "$3" --steps 6 --warmup 2 $extra \
      > gpurun_out/ref_row.log 2>&1
  local rc=$?
  local line; line=$(grep '^{' gpurun_out/ref_row.log | tail -1)
  echo "{\"model\": \"$1\", \"mbs\": $2, \"seq\": $3, \"gc\": $4, \"reference_tok_s\": $5, \"rc\": $rc, \"ours\": ${line:-null}}" >> $OUT
  echo "$1 mbs=$2 seq=$3 gc=$4 rc=$rc $(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read() or "{}"); print(d.get("tokens_per_s_per_gpu"), d.get("mfu_pct"), d.get("max_mem_gb"))' 2>/dev/null)"
  [ $rc -eq 124 ] || [ $rc -eq 137 ] && exit $rc
  return 0
}
run qwen3-0.6b 2 2048 0 9731
run qwen3-0.6b 1 8192 1 9834
run qwen3-0.6b 1 16384 1 9079
run qwen3-1.7b 1 2048 0 4685
run qwen3-1.7b 1 2048 1 3162
run qwen3-1.7b 1 8192 1 7396
run qwen3-4b 1 2048 1 2415
exit 0
