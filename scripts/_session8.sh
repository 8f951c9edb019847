set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu.sh "profile r04f_final final 800 800 64" "profile r04f_c4s8 random_10k 3840 2160 2000 8"
