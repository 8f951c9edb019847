set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu.sh "tests" "smoke" "bench r04h_bench" "configs r04h" "rehearsal r04h_reh"
