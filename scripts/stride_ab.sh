#!/bin/bash
# tile-stride A/B (HRT_TILE_STRIDE=0: binary search over the tile table) on C2 shares 1 / 2 / 8
set -u
E="/HRT_TILE_STRIDE=0"
: > gpurun_out/stride_ab.log
for n in 1 2 8; do
  timeout -k 10 150 python -u scripts/probe.py --spp 500 --reps 3 --share $n --env "$E" >> gpurun_out/stride_ab.log 2>&1 || exit $?
done
