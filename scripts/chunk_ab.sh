#!/bin/bash
# General-scene chunk-rule A/B (HRT_CHUNK_MIN / HRT_CHUNK_DIV) on C3 and C5 -> gpurun_out/chunk_ab.jsonl
set -u
OUT=gpurun_out/chunk_ab.jsonl
: > $OUT
run() { echo "{\"ab\": \"$1 $2\"}" >> $OUT; HRT_CHUNK_MIN=$1 HRT_CHUNK_DIV=$2 timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-parity "${@:3}" >> $OUT 2>> gpurun_out/chunk_ab.err; }
for ab in "32 16" "128 4"; do
  run $ab --preset earth_perlin --spp 1000 && run $ab --preset cornell --width 2048 --height 2048 --spp 1250 || exit 1
done
