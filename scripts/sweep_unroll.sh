#!/bin/bash
# rebuild libhrt with each walk unroll factor and probe the headline scene (postpone 64/32/24)
set -e
for u in ${@:-1 2 4}; do
  echo "== unroll $u"
  make -s -C hyper-ray-tracer_amd -B EXTRA=-DHRT_WALK_UNROLL=$u > /dev/null
  timeout -k 10 200 python scripts/probe.py --spp 64 --reps 2 --env "HRT_KERNEL=general/HRT_POSTPONE=64/HRT_POSTPONE=32/HRT_POSTPONE=24" | grep -E "median"
done
make -s -C hyper-ray-tracer_amd -B > /dev/null
