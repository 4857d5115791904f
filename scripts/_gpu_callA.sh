set -e
bash scripts/_gpu_call2.sh
bash scripts/_gpu_flash_pmc.sh
