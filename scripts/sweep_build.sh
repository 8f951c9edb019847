#!/bin/bash
# Rebuild libhrt with each EXTRA define set and probe (same box, back to back).
#   bash scripts/sweep_build.sh "<probe args>" "-DA=1" "-DA=2 -DB=3" ...
set -e
ARGS=$1; shift
for ex in "$@"; do
  echo "== EXTRA=$ex"
  make -s -C hyper-ray-tracer_amd -B EXTRA="$ex" > /dev/null
  timeout -k 10 200 python scripts/probe.py $ARGS | grep -E "median|count:"
done
make -s -C hyper-ray-tracer_amd -B > /dev/null
