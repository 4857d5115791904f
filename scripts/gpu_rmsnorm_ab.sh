#!/bin/bash
# RMSNorm backward block-cap A/B: numerics, then isolated bandwidth per cap (B4 S4096 h4096).
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k rmsnorm > gpurun_out/rms_test.log 2>&1 || exit $?
for cap in ${CAPS:-256 512 1024 2048}; do
  echo "cap=$cap" >> gpurun_out/rms_ab.log
  ST_RMSNORM_BWD_BLOCKS=$cap timeout -k 10 200 python tools/bench_kernels.py --only elt --no-ref --batch 4 \
      >> gpurun_out/rms_ab.log 2>&1 || exit $?
done
