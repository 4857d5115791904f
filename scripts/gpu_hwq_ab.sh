set -u
mkdir -p gpurun_out
for i in 1 2; do
  for q in 4 8; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --steps 8 --warmup 3 > gpurun_out/hwq_${q}_$i.log 2>&1 || exit $?
    echo "q=$q run $i: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/hwq_${q}_$i.log)"
  done
done
