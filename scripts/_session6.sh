set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu.sh "libs s6_one_final '--preset final --width 800 --height 800 --spp 64 --reps 3' prevone cur prevone cur" "libs s6_one_c5 '--preset cornell --width 2048 --height 2048 --spp 1250 --share 8 --reps 2' prevone cur" "libs s6_one_smoke '--preset cornell_smoke --width 800 --height 800 --spp 200 --reps 2' prevone cur" "probe s6_fcount --preset final --width 800 --height 800 --spp 64 --reps 1 --count" "probe s6_c2count --preset random --width 1920 --height 1080 --spp 100 --reps 1 --count" "tests"
