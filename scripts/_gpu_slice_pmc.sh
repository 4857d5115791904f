# PMC row of the heaviest kernel of each per-rank slice: three counter
# passes per slice, counters only on the kernels matching the slice's regex.
set -e
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/slice_pmc
mkdir -p $O
declare -A RX=(
  [dp]='Custom_Cijk_Alik_Bljk_BBS_BH_MT256x256x64'
  [tp2pp2dp2]='Custom_Cijk_Alik_Bljk_BBS_BH_Bias_HA_S_SAV_NTD_SK3'
  [cp8_32k]='flash_bwd_dkdv_kernel'
  [mixtral_ep8]='wgrad4_kernel|grouped8_kernel|gemm4e_kernel'
)
for L in ${SLICES:-dp tp2pp2dp2 cp8_32k mixtral_ep8}; do
  echo "== $L $(date +%T)"
  i=0
  for set in "SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i + 1))
    timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $set --kernel-include-regex "${RX[$L]}" -d $O/$L/pmc_$i -o run --output-format csv -- python3 bench.py --layout $L --slice --steps 1 --warmup 1 > $O/$L.log$i 2>&1 || { tail -20 $O/$L.log$i; exit 1; }
  done
  python tools/pmc_by_grid.py $O/$L "${RX[$L]}" > $O/pmc_$L.txt
  cat $O/pmc_$L.txt
  rm -rf $O/$L
done
