#!/bin/bash
# Build an A/B variant of libhrt here (CPU container) into ab/libhrt_<name>.so, from a copy of the sources so
# the in-tree build stays the default one; scripts/gpu.sh "libs <tag> '<probe args>' <name>..." runs them.
#   bash scripts/ablib.sh <name> [EXTRA defines, e.g. -DHRT_PERLIN_SELECT=1]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
tmp=/tmp/hrt_ab_$name
rm -rf "$tmp" && mkdir -p "$tmp/pkg"
cp -r "$ROOT/include" "$tmp/"
cp -r "$ROOT/hyper-ray-tracer_amd/csrc" "$ROOT/hyper-ray-tracer_amd/Makefile" "$tmp/pkg/"
make -s -j8 -C "$tmp/pkg" EXTRA="$*" COMMON="-O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-parameter -I../include -Icsrc $*" lib/libhrt.so
mkdir -p "$ROOT/ab"
cp "$tmp/pkg/lib/libhrt.so" "$ROOT/ab/libhrt_$name.so"
echo "ab/libhrt_$name.so"
