set -e
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/flash_r6
mkdir -p $O
timeout -k 10 300 python tools/bench_flash_shapes.py > $O/base.jsonl
cat $O/base.jsonl
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE -d $O/pmc_mfma -o run --output-format csv -- python3 tools/bench_flash_shapes.py --iters 3 > /dev/null
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 tools/bench_flash_shapes.py --iters 3 > /dev/null
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d $O/pmc_write -o run --output-format csv -- python3 tools/bench_flash_shapes.py --iters 3 > /dev/null
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $O/pmc_lds -o run --output-format csv -- python3 tools/bench_flash_shapes.py --iters 3 > /dev/null
python tools/pmc_summary.py $O/pmc_mfma $O/pmc_fetch $O/pmc_write $O/pmc_lds > $O/pmc.md
python tools/pmc_by_grid.py $O flash > $O/pmc_by_grid.txt
cat $O/pmc_by_grid.txt
rm -rf $O/pmc_mfma $O/pmc_fetch $O/pmc_write $O/pmc_lds  # raw passes: keep gpurun_out small
