set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu.sh "libs s16_c2 '--preset random --width 1920 --height 1080 --spp 500 --reps 3' prev cur prev cur" "libs s16_c4 '--preset random_10k --width 3840 --height 2160 --spp 2000 --share 8 --reps 1' prev cur" "libs s16_c5 '--preset cornell --width 2048 --height 2048 --spp 10000 --share 8 --reps 1' prev cur" "libs s16_final '--preset final --width 800 --height 800 --spp 64 --reps 3' prev cur" "libs s16_c3 '--preset earth_perlin --width 1920 --height 1080 --spp 1000 --reps 2' prev cur"
