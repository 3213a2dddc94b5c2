#!/bin/bash
# Measurement only: the AQL packet's agent-scope acquire vs none (DORA_GPU_AQL_ACQUIRE=none) on
# C3, the 40.96 MB headline and the native 4 MB ladder, interleaved.  The bench's sources are
# written once before any pack reads them, so no stale line can be read here.
# Output: gpurun_out/acquire_ab.jsonl.
export TMPDIR=/tmp
out=gpurun_out/acquire_ab.jsonl
mkdir -p gpurun_out
for rep in 1 2 3; do
  for acq in agent none; do
    line=$(DORA_GPU_AQL_ACQUIRE=$acq timeout -k 10 120 python bench.py --workload c3 --no-cpu-baseline --no-ladder --steps 1000) || exit $?
    echo "{\"acquire\": \"$acq\", \"wl\": \"c3\", \"bench\": $line}" >> $out
    line=$(DORA_GPU_AQL_ACQUIRE=$acq timeout -k 10 120 python bench.py --no-cpu-baseline --no-ladder --steps 1000) || exit $?
    echo "{\"acquire\": \"$acq\", \"wl\": \"c2\", \"bench\": $line}" >> $out
    timeout -k 10 180 python scripts/native_tp.py --sizes 4096000 --n 3000 \
      --env DORA_GPU_AQL_ACQUIRE=$acq | sed "s/^/{\"acquire\": \"$acq\", \"r\": /; s/\$/}/" >> $out || exit $?
  done
done
