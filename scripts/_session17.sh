set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu.sh "profile r04h_c4 random_10k 3840 2160 2000"
