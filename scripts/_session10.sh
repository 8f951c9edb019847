set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu.sh "probe s10_final_chunk --preset final --width 800 --height 800 --spp 64 --reps 3 --env HRT_CHUNK_MIN=16/HRT_CHUNK_MIN=8/HRT_CHUNK_MIN=32/HRT_CHUNK_TAIL=0/HRT_CHUNK_MIN=8,HRT_CHUNK_DIV=16" "probe s10_final_knobs --preset final --width 800 --height 800 --spp 64 --reps 3 --env HRT_PRIM_BATCH=8,HRT_POSTPONE=32/HRT_PRIM_BATCH=8,HRT_POSTPONE=28/HRT_PRIM_BATCH=12,HRT_POSTPONE=32/HRT_PRIM_BATCH=6,HRT_POSTPONE=36" "probe s10_final256 --preset final --width 800 --height 800 --spp 256 --reps 2 --count"
