#!/bin/bash
# BASELINE configs 3-5 on one GPU (bench.py lines, one per config) -> gpurun_out/configs.jsonl
set -u
OUT=gpurun_out/configs.jsonl
: > $OUT
run() { timeout -k 10 "$1" python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline "${@:2}" >> $OUT 2>> gpurun_out/configs.err; }
run 120 --preset earth_perlin --spp 1000 && \
run 200 --preset random_10k --width 3840 --height 2160 --spp 2000 && \
run 200 --preset cornell --width 2048 --height 2048 --spp 1250
