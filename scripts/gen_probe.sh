#!/bin/bash
# general scenes at low spp, default knobs (probe.py) -> gpurun_out/gen_probe.log
set -u
: > gpurun_out/gen_probe.log
for spec in "final 800 800 64" "cornell 2048 2048 64" "cornell_smoke 800 800 200" "earth_perlin 1920 1080 128" "simple_light 1920 1080 128"; do
  set -- $spec
  timeout -k 10 200 python -u scripts/probe.py --preset $1 --width $2 --height $3 --spp $4 --reps 3 >> gpurun_out/gen_probe.log 2>&1 || exit $?
done
