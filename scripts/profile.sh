#!/bin/bash
# rocprofv3 passes over one bench run: kernel trace + stats, then PMC passes in their own runs
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950; no trace domains mixed with --pmc; at most
# 8 SQ + 2 GRBM counters per pass).  Outputs under gpurun_out/prof_<tag>_*; summarise with
#   python scripts/summarize_profile.py <tag> <preset> <W> <H> <spp>
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02}
ARGS=${2:-"--steps 1 --warmup 1 --no-cpu-baseline --no-parity"}
export TMPDIR=/tmp
cd /tmp
OUT=$ROOT/gpurun_out
mkdir -p $OUT
run() {  # run <name> <seconds> <rocprof args...>
  local name=$1 secs=$2; shift 2
  echo "== $name" >> $OUT/profile_$TAG.log
  timeout -k 10 $secs rocprofv3 "$@" -d $OUT/prof_${TAG}_$name -o run --output-format csv -- python3 $ROOT/bench.py $ARGS >> $OUT/profile_$TAG.log 2>&1
  local rc=$?
  echo "== $name exit $rc" >> $OUT/profile_$TAG.log
  return $rc
}
: > $OUT/profile_$TAG.log
run kt 300 --kernel-trace --stats && \
run fetch 300 --pmc FETCH_SIZE && \
run write 300 --pmc WRITE_SIZE && \
run sq 300 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE && \
run sq2 300 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE
