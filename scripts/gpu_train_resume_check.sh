#!/bin/bash
# tools/train.py on one GPU: 20 steps with checkpoints every 10, then --auto_resume to 30;
# the resumed run must start from step 20 and keep training (HIP kernels, async save).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
W=/tmp/st_resume_check
rm -rf $W
common="--model_name_or_path tiny-llama --synthetic_data True --micro_batch_size 4 --sequence_length 256
        --learning_rate 1e-3 --log_interval 5 --save_model_checkpoint True --save_frequency 10 --work_dir $W"
timeout -k 10 300 python tools/train.py $common --total_train_steps 20 > gpurun_out/resume_a.log 2>&1 || exit $?
timeout -k 10 300 python tools/train.py $common --total_train_steps 30 --auto_resume True > gpurun_out/resume_b.log 2>&1 || exit $?
ls $W
grep -h "Step:" gpurun_out/resume_a.log | tail -2
grep -h -i "resum" gpurun_out/resume_b.log | head -3
grep -h "Step:" gpurun_out/resume_b.log | head -3
