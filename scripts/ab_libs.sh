#!/bin/bash
# A/B of prebuilt library variants (ab/libhrt_<name>.so, built on the CPU side) on one GPU box, back to
# back: bash scripts/ab_libs.sh "<probe args>" name1 name2 ...   (each in its own process, 200 s limit)
set -u
ARGS=$1; shift
mkdir -p gpurun_out
for n in "$@"; do
  echo "== $n" >> gpurun_out/ab.log
  HRT_LIB=ab/libhrt_$n.so timeout -k 10 200 python scripts/probe.py $ARGS >> gpurun_out/ab.log 2>&1 || { echo "== $n failed rc $?" >> gpurun_out/ab.log; exit 1; }
done
grep -E "^==|median" gpurun_out/ab.log
