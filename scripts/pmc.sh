#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, no trace domains) over one probe/bench command.
#   bash scripts/pmc.sh <tag> <python script + args...>
# Outputs gpurun_out/pmc_<tag>_<pass>/run_counter_collection.csv; summarise with scripts/pmc_summary.py <tag>.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
export TMPDIR=/tmp
cd /tmp
OUT=$ROOT/gpurun_out
PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU"
  "SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_INSTS_SMEM"
  "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_INSTS_VSKIPPED SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_FLAT"
)
i=0
for p in "${PASSES[@]}"; do
  echo "== pass $i: $p" >> $OUT/pmc_$TAG.log
  timeout -k 10 300 rocprofv3 --pmc $p -d $OUT/pmc_${TAG}_$i -o run --output-format csv -- python3 $ROOT/"$@" >> $OUT/pmc_$TAG.log 2>&1
  rc=$?
  echo "== pass $i exit $rc" >> $OUT/pmc_$TAG.log
  [ $rc -eq 0 ] || exit $rc
  i=$((i+1))
done
