#!/bin/bash
# Kernel traces of the MoE proxies (Mixtral EP layout on 1 GPU, Qwen3-30B-A3B), 4 layers each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mx -o run --output-format csv -- python bench.py --layout mixtral_ep8 --layers 4 --steps 3 --warmup 2 > gpurun_out/prof_mx.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_q3 -o run --output-format csv -- python bench.py --model qwen3-30b-a3b --layers 4 --micro_batch_size 2 --steps 3 --warmup 2 > gpurun_out/prof_q3.log 2>&1 || exit $?
exit 0
