#!/bin/bash
# CPU sanitizer run (race detection / sanitizers).  CPU only: never run on a GPU box.
#   1. ThreadSanitizer over the oracle's thread pools (oracle/tsan_check.cpp: every preset on 8 threads,
#      frames equal to the one-thread frames bit for bit);
#   2. the CPU test suite (-m "not gpu") with the host library's sources (scene lowering, BvhNode::new,
#      walk-stream builders, presets, image writer, knobs), the oracle and the host lane simulator built under
#      clang AddressSanitizer + UndefinedBehaviorSanitizer and loaded in place of the ordinary builds
#      (HRT_LIB, ORACLE_LIB, LANE_SIM_CFLAGS), the clang ASan runtime preloaded into Python.
# Output: $SAN_OUT (default /tmp/hrt_sanitize)/sanitize_*.log; the summary goes into DESIGN.md.
set -u
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd "$ROOT"
OUT=${SAN_OUT:-/tmp/hrt_sanitize}
mkdir -p "$OUT"
RT=/opt/rocm/lib/llvm/lib/clang/22/lib/linux/libclang_rt.asan-x86_64.so

make -s -C oracle tsan > "$OUT/sanitize_tsan.log" 2>&1
echo "tsan exit $? ($(grep -c 'WARNING: ThreadSanitizer' "$OUT/sanitize_tsan.log") reports)"

make -s -C hyper-ray-tracer_amd asan && make -s -C oracle asan || exit 1
# detect_leaks=0: Python and torch hold their allocations to exit; the suite's own leaks are not the target
LD_PRELOAD=$RT ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1 \
UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
HRT_LIB=$ROOT/hyper-ray-tracer_amd/lib/asan/libhrt.so ORACLE_LIB=$ROOT/oracle/_asan/liboracle.so \
LANE_SIM_CFLAGS="-g -fsanitize=address,undefined -fno-sanitize-recover=undefined -shared-libsan" \
  timeout -k 10 3600 python -m pytest tests -m "not gpu" -q -p no:cacheprovider "$@" > "$OUT/sanitize_asan.log" 2>&1
rc=$?
echo "asan+ubsan suite exit $rc: $(tail -1 "$OUT/sanitize_asan.log")"
grep -E "ERROR: AddressSanitizer|runtime error:" "$OUT/sanitize_asan.log" | head -20
exit $rc
