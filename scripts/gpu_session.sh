#!/bin/bash
# One GPU-box session: each GPU step under its own time limit; a step that crashes, aborts or times
# out ends the session (pytest exit 1 = ordinary test failures, which still lets later steps run).
mkdir -p gpurun_out
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name: $*" >> gpurun_out/session.log
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name exit $rc" >> gpurun_out/session.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc $rc)" >> gpurun_out/session.log; exit $rc; fi
  return 0
}
: > gpurun_out/session.log
for spec in "$@"; do
  eval "step $spec" || exit $?
done
cat gpurun_out/session.log
