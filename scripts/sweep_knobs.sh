#!/bin/bash
# HRT_POSTPONE x HRT_PRIM_BATCH on the sphere kernel, alternated in one process per scene (probe.py --env)
set -u
envs=""
for p in 40 44 48 52 56; do for b in 4 6 8; do envs="$envs/HRT_POSTPONE=$p,HRT_PRIM_BATCH=$b"; done; done
envs=${envs#/}
timeout -k 10 200 python -u scripts/probe.py --spp 500 --reps 3 --env "$envs" > gpurun_out/sweep_c2.log 2>&1 && \
timeout -k 10 300 python -u scripts/probe.py --preset random_10k --width 3840 --height 2160 --spp 64 --reps 3 --env "$envs" > gpurun_out/sweep_c4.log 2>&1
