set -e
bash scripts/_gpu_flash_pmc.sh
PROF=0 STEPS=3 WARMUP=2 bash scripts/_gpu_slices.sh
