set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu.sh "tests" "smoke" "probe s13_final --preset final --width 800 --height 800 --spp 64 --reps 3 --count" "bench s13_bench"
