set -e
E=""
for pp in 48 56 60; do for pb in 6 8 12; do E="$E/HRT_POSTPONE=$pp,HRT_PRIM_BATCH=$pb"; done; done
timeout -k 10 300 python scripts/probe.py --spp 100 --reps 3 --env "${E#/}" > gpurun_out/sweep_env.log 2>&1
bash scripts/sweep_build.sh "--spp 100 --reps 3" "-DHRT_WALK_UNROLL=4" "-DHRT_WALK_UNROLL=8" "-DHRT_WALK_UNROLL=6 -DHRT_PRIM_EVERY=3" "-DHRT_BASIC_WAVES=5" "-DHRT_BASIC_WAVES=7" "" > gpurun_out/sweep_build.log 2>&1
