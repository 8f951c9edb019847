#!/bin/bash
# rocprofv3 passes over one bench run (one timed frame): kernel trace + stats, then PMC passes in
# their own runs (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950; no trace domains mixed
# with --pmc).  Outputs under gpurun_out/prof_<tag>_*.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}
ARGS=${2:-"--steps 1 --warmup 1 --no-cpu-baseline"}
export TMPDIR=/tmp
cd /tmp
OUT=$ROOT/gpurun_out
run() {  # run <name> <seconds> <rocprof args...>
  local name=$1 secs=$2; shift 2
  echo "== $name" >> $OUT/profile.log
  timeout -k 10 $secs rocprofv3 "$@" -d $OUT/prof_${TAG}_$name -o run --output-format csv -- python3 $ROOT/bench.py $ARGS >> $OUT/profile.log 2>&1
  local rc=$?
  echo "== $name exit $rc" >> $OUT/profile.log
  return $rc
}
: > $OUT/profile.log
run kt 300 --kernel-trace --stats && \
run fetch 300 --pmc FETCH_SIZE && \
run write 300 --pmc WRITE_SIZE && \
run sq 300 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE
