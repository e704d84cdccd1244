#!/bin/bash
# Box facts for the CPU-baseline report: CPU quota / affinity / memory (no GPU use).
mkdir -p gpurun_out
{ echo "nproc=$(nproc)"; cat /sys/fs/cgroup/cpu.max 2>/dev/null || echo "no cpu.max";
  python3 -c "import os; print('aff', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())"; free -g; } \
  > gpurun_out/probe.txt 2>&1
