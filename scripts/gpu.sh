#!/bin/bash
# One GPU-box session driver: every step under its own time limit, output under gpurun_out/, a step that
# crashes, aborts or times out ends the session (exit 1 = ordinary test failures lets later steps run).
#
#   bash scripts/gpu.sh <step> [<step> ...]      each step one quoted word list:
#     "tests [pytest -k expr]"                   pytest -m gpu (verbose, per-test timeout)      -> tests.log
#     "smoke"                                    __graft_entry__.smoke()                        -> smoke.log
#     "bench <tag> [bench args]"                 one bench.py line                              -> <tag>.jsonl
#     "rehearsal <tag> [bench args]"             2 ranks sharing GPU 0 (--one-device)           -> <tag>.jsonl
#     "rehearsaln <tag> <N> [bench args]"        N ranks (N <= 4) sharing GPU 0 (--one-device)  -> <tag>.jsonl
#     "rehtrace <tag> [bench args]"              the same under rocprofv3 --kernel-trace         -> prof_<tag>/
#     "configs <tag>"                            BASELINE configs 3-5 lines (C4 / C5 also as an 8-way share)
#     "profile <tag> <preset> <W> <H> <spp> [share] [bench args]"
#                                                rocprofv3 kernel trace + PMC passes over one bench run,
#                                                summarised into profiles/<tag>_summary.md + roofline_pmc.json
#     "probe <tag> [probe.py args]"              scripts/probe.py (A/B of env knobs: --env "A=1/A=2")
#     "libs <tag> <probe args> <name>..."        probe.py against prebuilt ab/libhrt_<name>.so variants
# Example:  gpurun -- 'bash scripts/gpu.sh "tests" "bench r03a" "configs r03a"'
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
LOG=$OUT/session.log

run() {  # run <name> <seconds> <cmd...>: output appended to gpurun_out/<name>.log
  local name=$1 secs=$2; shift 2
  echo "== $name: $*" >> "$LOG"
  timeout -k 10 "$secs" "$@" >> "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name exit $rc" >> "$LOG"
  return $rc
}
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }

bench_line() {  # bench_line <tag> <seconds> <bench args...>: the JSON line to <tag>.jsonl
  local tag=$1 secs=$2; shift 2
  echo "== $tag: bench.py $*" >> "$LOG"
  timeout -k 10 "$secs" python -u bench.py "$@" >> "$OUT/$tag.jsonl" 2>> "$OUT/$tag.err"
  local rc=$?
  echo "== $tag exit $rc" >> "$LOG"
  return $rc
}

profile() {  # profile <tag> <preset> <W> <H> <spp> [share] [bench args...]
  local tag=$1 preset=$2 W=$3 H=$4 spp=$5; shift 5
  local share=1
  if [ $# -gt 0 ] && [[ $1 =~ ^[0-9]+$ ]]; then share=$1; shift; fi
  local args="--preset $preset --width $W --height $H --spp $spp --share $share --steps 1 --warmup 1 --no-cpu-baseline --no-parity --no-delivery $*"
  local rc=0
  export TMPDIR=/tmp
  pushd /tmp > /dev/null
  prof() {  # prof <pass> <rocprofv3 args...>
    local pass=$1; shift
    echo "== profile $tag $pass" >> "$LOG"
    timeout -k 10 400 rocprofv3 "$@" -d "$OUT/prof_${tag}_$pass" -o run --output-format csv -- python3 "$ROOT/bench.py" $args \
      --launch-record "$OUT/prof_${tag}_$pass/launch.json" \
      >> "$OUT/profile_$tag.log" 2>&1
    local r=$?
    echo "== profile $tag $pass exit $r" >> "$LOG"
    return $r
  }
  prof kt --kernel-trace --stats && \
  prof fetch --pmc FETCH_SIZE && \
  prof write --pmc WRITE_SIZE && \
  prof sq --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE && \
  prof sq2 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE
  rc=$?
  popd > /dev/null
  [ $rc -eq 0 ] && python scripts/summarize_profile.py "$tag" "$preset" "$W" "$H" "$spp" "$share" >> "$OUT/profile_$tag.log" 2>&1
  return $rc
}

step() {
  local kind=$1; shift
  case $kind in
    tests)
      if [ $# -gt 0 ]; then run tests 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "$*"
      else run tests 900 python -u -m pytest tests -m gpu -x -v --durations=25 --timeout 200 --timeout-method thread -p no:cacheprovider; fi ;;
    smoke) run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) local tag=$1; shift; bench_line "$tag" 600 "$@" ;;
    rehearsal)  # bench.py starts its own ranks (hrt/launcher.py): no torchrun
      local tag=$1; shift
      echo "== $tag: 2-rank rehearsal $*" >> "$LOG"
      timeout -k 10 240 python -u bench.py --gpus 2 --one-device "$@" >> "$OUT/$tag.jsonl" 2>> "$OUT/$tag.err"
      local rc=$?; echo "== $tag exit $rc" >> "$LOG"; return $rc ;;
    rehearsaln)  # N ranks on one GPU (the N > 1 code paths: split, delivery, parity and CPU leg on the N-GPU frame)
      local tag=$1 n=$2; shift 2
      [ "$n" -le 4 ] || { echo "rehearsaln: at most 4 ranks" >> "$LOG"; return 2; }
      echo "== $tag: $n-rank rehearsal $*" >> "$LOG"
      timeout -k 10 400 python -u bench.py --gpus "$n" --one-device "$@" >> "$OUT/$tag.jsonl" 2>> "$OUT/$tag.err"
      local rc=$?; echo "== $tag exit $rc" >> "$LOG"; return $rc ;;
    rehtrace)  # kernel timeline of a concurrent 2-rank rehearsal: one rocprofv3 per rank (each rank its own
      # profiled program with the process-group variables set, so bench.py never spawns under the profiler's preload)
      local tag=$1; shift
      echo "== $tag: rocprofv3 kernel trace of a 2-rank rehearsal $*" >> "$LOG"
      export TMPDIR=/tmp
      local port=$(( 29500 + RANDOM % 2000 )) pids=() r rc=0
      for r in 0 1; do
        RANK=$r LOCAL_RANK=$r WORLD_SIZE=2 LOCAL_WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=$port \
          timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/prof_${tag}/rank$r" -o run --output-format csv -- \
          python3 "$ROOT/bench.py" --gpus 2 --one-device "$@" >> "$OUT/$tag.r$r.out" 2>> "$OUT/$tag.err" &
        pids+=($!)
      done
      for r in 0 1; do wait "${pids[$r]}" || rc=$?; done
      cat "$OUT/$tag.r0.out" >> "$OUT/$tag.jsonl"
      echo "== $tag exit $rc" >> "$LOG"; return $rc ;;
    configs)
      local tag=$1
      # C3 with its parity rows and CPU baseline; C4's whole frame with the fewest rows the CPU budget allows (a 4K
      # row at 2000 spp is ~20 s of the oracle's reference culling on 16 threads); C4's and C5's 1/8 shares with
      # parity tiles and a CPU baseline on tiles
      bench_line "${tag}_configs" 300 --steps 1 --warmup 1 --no-delivery --preset earth_perlin --spp 1000 && \
      bench_line "${tag}_configs" 500 --steps 1 --warmup 1 --no-delivery --preset random_10k --width 3840 --height 2160 --spp 2000 && \
      bench_line "${tag}_configs" 300 --steps 1 --warmup 1 --no-delivery --preset random_10k --width 3840 --height 2160 --spp 2000 --share 8 && \
      bench_line "${tag}_configs" 300 --steps 1 --warmup 1 --no-delivery --preset cornell --width 2048 --height 2048 --spp 10000 --share 8 ;;
    profile) profile "$@" ;;
    probe) local tag=$1; shift; run "$tag" 600 python -u scripts/probe.py "$@" ;;
    libs)
      local tag=$1 args=$2; shift 2
      for n in "$@"; do
        echo "== lib $n" >> "$OUT/$tag.log"
        HRT_LIB=ab/libhrt_$n.so run "$tag" 300 python -u scripts/probe.py $args || return $?
      done ;;
    *) echo "unknown step $kind" >> "$LOG"; return 2 ;;
  esac
}

: > "$LOG"
for spec in "$@"; do
  eval "step $spec"
  rc=$?
  if fatal $rc; then echo "stopping after '$spec' (rc $rc)" >> "$LOG"; cat "$LOG"; exit $rc; fi
done
cat "$LOG"
