#!/bin/bash
# rank 0's share of an N-way tile split on one GPU (what each GPU of an N-GPU bench renders)
set -u
: > gpurun_out/share_probe.log
for n in 1 2 4 8; do
  timeout -k 10 120 python -u scripts/probe.py --spp 500 --reps 3 --share $n >> gpurun_out/share_probe.log 2>&1 || exit $?
done
for n in 1 8; do
  timeout -k 10 200 python -u scripts/probe.py --preset random_10k --width 3840 --height 2160 --spp 250 --reps 2 --share $n >> gpurun_out/share_probe.log 2>&1 || exit $?
done
