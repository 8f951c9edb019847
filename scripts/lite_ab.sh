#!/bin/bash
# general-kernel LITE instantiation A/B (HRT_GEN_TRIM=0 = the all-feature build) on Cornell
set -u
timeout -k 10 200 python -u scripts/probe.py --preset cornell --width 2048 --height 2048 --spp 64 --reps 3 --env "/HRT_GEN_TRIM=0" > gpurun_out/lite_cornell.log 2>&1
