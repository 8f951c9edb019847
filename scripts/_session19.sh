set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu.sh "tests" "smoke"
