#!/bin/bash
# general-kernel waves/SIMD A/B (HRT_GEN_WAVES_RT 4 / 5 / 6), alternated in one process per scene
set -u
E="HRT_GEN_WAVES_RT=4/HRT_GEN_WAVES_RT=5/HRT_GEN_WAVES_RT=6"
timeout -k 10 200 python -u scripts/probe.py --preset cornell --width 2048 --height 2048 --spp 64 --reps 3 --env "$E" > gpurun_out/gw_cornell.log 2>&1 && \
timeout -k 10 200 python -u scripts/probe.py --preset final --width 800 --height 800 --spp 64 --reps 3 --env "$E" > gpurun_out/gw_final.log 2>&1 && \
timeout -k 10 200 python -u scripts/probe.py --preset cornell_smoke --width 800 --height 800 --spp 64 --reps 3 --env "$E" > gpurun_out/gw_smoke.log 2>&1
