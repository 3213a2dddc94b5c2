#!/bin/bash
# Box diagnostics next to a bench run: CPU share / throttling, GPU clocks and queues, so a
# slow run can be told apart from a slow box.  Writes gpurun_out/box_diag_<tag>.txt.
tag=${1:-now}
out=gpurun_out/box_diag_$tag.txt
mkdir -p gpurun_out
{
  echo "== date"; date -u
  echo "== nproc / affinity"; nproc; python3 -c 'import os; print(len(os.sched_getaffinity(0)))'
  echo "== cgroup cpu.max"; cat /sys/fs/cgroup/cpu.max 2>/dev/null || true
  echo "== cgroup cpu.stat"; cat /sys/fs/cgroup/cpu.stat 2>/dev/null || true
  echo "== lscpu"; lscpu 2>/dev/null | grep -E 'Model name|Socket|NUMA node|L3' || true
  echo "== loadavg"; cat /proc/loadavg
  echo "== rocm-smi clocks"; timeout 20 rocm-smi --showclocks 2>/dev/null || true
  echo "== rocm-smi perf level"; timeout 20 rocm-smi --showperflevel 2>/dev/null || true
  echo "== rocm-smi power"; timeout 20 rocm-smi --showpower 2>/dev/null || true
  echo "== compute partition"; timeout 20 rocm-smi --showcomputepartition 2>/dev/null || true
  echo "== memory partition"; timeout 20 rocm-smi --showmemorypartition 2>/dev/null || true
  echo "== gpu processes"; timeout 20 rocm-smi --showpids 2>/dev/null || true
} > "$out" 2>&1
exit 0
