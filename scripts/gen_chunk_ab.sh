#!/bin/bash
# general-scene chunk rule at low spp: (min, div) = (64, 8) default / (16, 8) / (16, 32), one process per scene
set -u
E="HRT_CHUNK_MIN=64,HRT_CHUNK_DIV=8/HRT_CHUNK_MIN=16,HRT_CHUNK_DIV=8/HRT_CHUNK_MIN=16,HRT_CHUNK_DIV=32/HRT_CHUNK_MIN=32,HRT_CHUNK_DIV=8"
timeout -k 10 200 python -u scripts/probe.py --preset final --width 800 --height 800 --spp 64 --reps 3 --env "$E" > gpurun_out/gc_final.log 2>&1 && \
timeout -k 10 200 python -u scripts/probe.py --preset cornell --width 2048 --height 2048 --spp 64 --reps 3 --env "$E" > gpurun_out/gc_cornell.log 2>&1 && \
timeout -k 10 200 python -u scripts/probe.py --preset cornell_smoke --width 800 --height 800 --spp 200 --reps 3 --env "$E" > gpurun_out/gc_smoke.log 2>&1 && \
timeout -k 10 200 python -u scripts/probe.py --preset earth_perlin --width 1920 --height 1080 --spp 128 --reps 3 --env "$E" > gpurun_out/gc_earth.log 2>&1
