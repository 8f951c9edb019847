set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu.sh "profile r04h_c2 random 1920 1080 500" "profile r04h_c3 earth_perlin 1920 1080 1000" "profile r04h_c4s8 random_10k 3840 2160 2000 8" "profile r04h_c5s8 cornell 2048 2048 10000 8" "profile r04h_final final 800 800 64"
