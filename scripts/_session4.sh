set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu.sh "tests" "probe s4_final_batch --preset final --width 800 --height 800 --spp 64 --reps 2 --env HRT_PRIM_BATCH=32/HRT_PRIM_BATCH=16/HRT_PRIM_BATCH=8/HRT_PRIM_BATCH=4" "probe s4_final_post --preset final --width 800 --height 800 --spp 64 --reps 2 --env HRT_POSTPONE=44/HRT_POSTPONE=52/HRT_POSTPONE=32" "probe s4_c5_batch --preset cornell --width 2048 --height 2048 --spp 1250 --share 8 --reps 2 --env HRT_PRIM_BATCH=32/HRT_PRIM_BATCH=16" "rehearsal s4_reh --steps 3 --warmup 1 --no-cpu-baseline"
