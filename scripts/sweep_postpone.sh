#!/bin/bash
# HRT_POSTPONE sweep on the headline scene (one process per value; 64 spp probe frames)
for v in ${@:-8 16 24 32 40 48 64}; do
  echo "== postpone $v"
  HRT_POSTPONE=$v timeout -k 10 120 python scripts/probe.py --spp 64 --reps 2 | grep -E "rep 1|median" || exit $?
done
