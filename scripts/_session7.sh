set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu.sh "probe s7_final --preset final --width 800 --height 800 --spp 64 --reps 3 --commit-env HRT_GWALK_BIG=1,HRT_GWALK_MED=1/HRT_GWALK_BIG=0,HRT_GWALK_MED=1/HRT_GWALK_BIG=1,HRT_GWALK_MED=0/HRT_GWALK_BIG=0,HRT_GWALK_MED=0" "probe s7_fcount --preset final --width 800 --height 800 --spp 64 --reps 1 --count" "tests general or final or gwalk or smoke or medium"
