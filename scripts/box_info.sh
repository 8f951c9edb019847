#!/bin/bash
# What the GPU box gives one job: CPUs (affinity / cgroup quota), memory, GPU.
echo "nproc: $(nproc)"
python3 -c "import os; print('affinity:', len(os.sched_getaffinity(0)), 'cpu_count:', os.cpu_count())"
for f in /sys/fs/cgroup/cpu.max /sys/fs/cgroup/cpuset.cpus.effective /sys/fs/cgroup/memory.max; do
  [ -r $f ] && echo "$f: $(cat $f)"
done
grep -m1 "model name" /proc/cpuinfo
echo "OMP_NUM_THREADS=${OMP_NUM_THREADS:-unset} MAX_JOBS=${MAX_JOBS:-unset}"
ldd --version | head -1
