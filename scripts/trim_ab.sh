#!/bin/bash
# general-kernel TRIM instantiations A/B: default / HRT_GEN_TRIM=0 (all features) / 4 waves per SIMD
set -u
E="/HRT_GEN_TRIM=0/HRT_GEN_WAVES_RT=4"
: > gpurun_out/trim_ab.log
for spec in "earth_perlin 1920 1080 128" "simple_light 1920 1080 128" "cornell_smoke 800 800 200" "cornell 2048 2048 64"; do
  set -- $spec
  timeout -k 10 200 python -u scripts/probe.py --preset $1 --width $2 --height $3 --spp $4 --reps 3 --env "$E" >> gpurun_out/trim_ab.log 2>&1 || exit $?
done
