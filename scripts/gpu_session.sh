#!/bin/bash
# One GPU-box session: the steps named in $STEPS (space separated), each time-limited;
# the first failure ends the run.  Step names: sp_gemm tests bench prof gmm flash wgrad
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
STEPS=${STEPS:-"tests bench"}
step() {
  local name=$1 to=$2; shift 2; echo "=== $name"
  # heartbeat: a slow-but-live step (the GPU test suite, a multi-process test) must not
  # look hung to gpurun's 180-s silence check; each step's own timeout bounds real hangs
  ( while true; do sleep 60; echo "[$name] alive $(date +%T) $(wc -l < "gpurun_out/$name.log" 2>/dev/null) lines"; done ) & local hb=$!
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  kill $hb 2>/dev/null; wait $hb 2>/dev/null
  tail -n 4 "gpurun_out/$name.log" | cut -c1-400; echo "=== $name rc=$rc"; return $rc
}
for s in $STEPS; do
  case $s in
    sp_gemm) step sp_gemm 240 python tools/bench_sp_gemm.py || exit $? ;;
    newk) step new_kernels 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_xgmi_gpu.py -m gpu -k "swiglu_epilogue or fused_matches or ep_exchange or ipc or grouped" || exit $? ;;
    wside_ab) step wgrad_side_ab 900 python tools/ab_step.py --variants ST_WGRAD_STREAM=main,ST_WGRAD_STREAM=side --rounds 3 --steps 3 --micro_batch_size 6 --fused_head 1 || exit $? ;;
    large_ab) step wgrad_large_ab 900 python tools/ab_step.py --variants ST_WGRAD_TUNE_LARGE=1,ST_WGRAD_TUNE_LARGE=0 --rounds 3 --steps 3 --micro_batch_size 6 --fused_head 1 || exit $? ;;
    tuned_ab) step wgrad_tuned_ab 900 python tools/ab_step.py --variants ST_WGRAD_TUNED=1,ST_WGRAD_TUNED=0 --rounds 3 --steps 3 --micro_batch_size 6 --fused_head 1 || exit $? ;;
    onet_ab) step onet_ab 900 python tools/ab_step.py --variants ST_WGRAD_ONE_T=1,ST_WGRAD_ONE_T=0 --rounds 3 --steps 3 --micro_batch_size 6 --fused_head 1 || exit $? ;;
    adamw_ab) step adamw_ab 900 python tools/ab_step.py --variants ST_ADAMW_BLOCKS=0,ST_ADAMW_BLOCKS=1024,ST_ADAMW_BLOCKS=256,ST_ADAMW_BLOCKS=64 --rounds 3 --steps 3 --micro_batch_size 6 --fused_head 1 || exit $? ;;
    cp_reorder) step cp_reorder 240 python tools/bench_cp_reorder.py || exit $? ;;
    opt_probe) step opt_probe 900 python tools/ab_step.py --variants ST_OPT_PROBE_SKIP=0,ST_OPT_PROBE_SKIP=1 --rounds 4 --steps 3 --micro_batch_size 6 --fused_head 1 || exit $? ;;
    moe) step mx_proxy 400 python bench.py --layout mixtral_ep8 --micro_batch_size 2 --grad_acc 1 --layers 4 --steps 5 --warmup 2 || exit $?
         step q3_proxy 400 python bench.py --model qwen3-30b-a3b --layers 4 --micro_batch_size 2 --steps 5 --warmup 2 || exit $? ;;
    q3_prof) step q3_prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_q3 -o run --output-format csv -- python bench.py --model qwen3-30b-a3b --layers 4 --micro_batch_size 2 --steps 3 --warmup 2 || exit $? ;;
    moe_prof) step mx_prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mx -o run --output-format csv -- python bench.py --layout mixtral_ep8 --micro_batch_size 2 --grad_acc 1 --layers 4 --steps 3 --warmup 2 || exit $? ;;
    gmm) step grouped_gemm_bench 300 python tools/bench_grouped_gemm.py || exit $? ;;
    rmsbwd) step rmsnorm_bwd_caps 300 bash -c 'for b in 256 512 768 1024; do ST_RMSNORM_BWD_BLOCKS=$b timeout -k 5 60 python tools/bench_rmsnorm_bwd.py || exit $?; done' || exit $? ;;
    rmspf) step rmsnorm_pf 400 bash -c 'for v in 0 1 0 1; do ST_RMSNORM_BWD_PF=$v timeout -k 5 60 python tools/bench_rmsnorm_bwd.py || exit $?; done && ST_RMSNORM_BWD_PF=1 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_train_gpu.py -m gpu -k "rmsnorm or deterministic or native_vs_reference"' || exit $? ;;
    dswiglu) step dense_swiglu 240 python tools/bench_dense_swiglu.py || exit $? ;;
    sptest) step sp_pair_test 400 python -u -m pytest -x -v --timeout 330 --timeout-method thread tests/test_xgmi_gpu.py -m gpu -k sp_decoder || exit $? ;;
    xtests) step xgmi_tests 700 python -u -m pytest -x -v --timeout 330 --timeout-method thread tests/test_xgmi_gpu.py -m gpu || exit $? ;;
    tests) step gpu_tests 1000 python -u -m pytest -x -v --timeout 330 --timeout-method thread tests -m gpu || exit $? ;;
    bench) step bench 600 python bench.py --steps 10 --warmup 3 || exit $? ;;
    bench16) step bench16 600 python bench.py --steps 10 --warmup 3 --opt_state_dtype bf16 || exit $? ;;
    hc8k) step bench_hc8k 600 python bench.py --steps 10 --warmup 3 --head_chunk 8192 || exit $? ;;
    hc12k) step bench_hc12k 600 python bench.py --steps 10 --warmup 3 --head_chunk 12288 || exit $? ;;
    prio) step bench_prio_default 600 python bench.py --steps 10 --warmup 3 || exit $?
          step bench_prio_high 600 env ST_COMPUTE_STREAM_PRIORITY=-1 python bench.py --steps 10 --warmup 3 || exit $?
          step bench_prio_default2 600 python bench.py --steps 10 --warmup 3 || exit $?
          step bench_prio_high2 600 env ST_COMPUTE_STREAM_PRIORITY=-1 python bench.py --steps 10 --warmup 3 || exit $? ;;
    mbs7) step bench_mbs7 600 python bench.py --steps 10 --warmup 3 --micro_batch_size 7 || exit $? ;;
    mbs8) step bench_mbs8 600 env ST_HBM_HEADROOM_GB=8 python bench.py --steps 10 --warmup 3 --micro_batch_size 8 || exit $? ;;
    bench32) step bench32 600 python bench.py --steps 10 --warmup 3 --opt_state_dtype fp32 || exit $? ;;
    adamk) step adamw_kernels 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_train_gpu.py -m gpu -k "adamw or overlapped or delayed or deterministic or rmsnorm" || exit $? ;;
    wt_ab) step wt_ab 900 python tools/ab_step.py --variants ST_ADAMW_WT=1,ST_ADAMW_WT=0 --rounds 3 --steps 3 --micro_batch_size 6 --fused_head 1 || exit $? ;;
    prof) step step_prof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_step -o run --output-format csv -- python bench.py --steps 3 --warmup 2 || exit $? ;;
    rehearse) step rehearse 1000 env LAYOUTS="${LAYOUTS:-mixtral_ep8 tp2pp2dp2}" LAYOUT_TIMEOUT=400 bash scripts/rehearse_layouts_1gpu.sh || exit $? ;;
    rehearse_mx) step rehearse_mx 600 env LAYOUTS=mixtral_ep8 LAYOUT_TIMEOUT=420 EXTRA="--seq_len 512" ST_XGMI_EP_MAX_MB=48 bash scripts/rehearse_layouts_1gpu.sh || exit $? ;;
    flash_pmc) step flash_pmc 200 timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE -d gpurun_out/flash_pmc -o run --output-format csv -- python tools/bench_flash_bwd_ds.py || exit $? ;;
    rehearse_mx4k) step rehearse_mx4k 600 env LAYOUTS=mixtral_ep8 LAYOUT_TIMEOUT=500 ST_XGMI_EP_MAX_MB=48 bash scripts/rehearse_layouts_1gpu.sh || exit $? ;;
    rehearse_dp) step rehearse_dp 600 env LAYOUTS=dp LAYOUT_TIMEOUT=500 bash scripts/rehearse_layouts_1gpu.sh || exit $? ;;
    gmm_pmc) step gmm_pmc 250 timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE -d gpurun_out/gmm_pmc -o run --output-format csv -- python tools/bench_grouped_gemm.py || exit $? ;;
    replay) step replay 1100 env ST_XGMI_EP_MAX_MB=48 python scripts/bench_reference_rows_8gpu.py --rehearse --steps 2 --warmup 1 --timeout 300 \
              --out gpurun_out/reference_rows_rehearsal.jsonl --filter "${REPLAY_FILTER:-.}" || exit $? ;;
    # the table is written under gpurun_out/ (merged back) and copied into scaletorch_amd/tuning/ by hand
    gtune) step gemm_tune 900 env ST_GEMM_TUNING_FILE=gpurun_out/gemm_gfx950.csv python bench.py --steps 1 --warmup 2 --gemm_tuning tune || exit $? ;;
    gtune_rot) step gemm_tune_rot 900 env ST_GEMM_TUNING_FILE=gpurun_out/gemm_gfx950_rot.csv PYTORCH_TUNABLEOP_ROTATING_BUFFER_SIZE=512 PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=60 python bench.py --steps 1 --warmup 2 --gemm_tuning tune || exit $? ;;
    gtune_rot_ab) step gemm_tune_rot_ab 900 env ST_GEMM_TUNING_FILE=gpurun_out/gemm_gfx950_rot.csv python tools/ab_step.py --variants TUNABLE=1,TUNABLE=0 --rounds 3 --steps 3 --micro_batch_size 6 --fused_head 1 --gemm_tuning use || exit $? ;;
    gtune_ab) step gemm_tune_ab 900 python tools/ab_step.py --variants TUNABLE=1,TUNABLE=0 --rounds 3 --steps 3 --micro_batch_size 6 --fused_head 1 --gemm_tuning use || exit $? ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
exit 0
