#!/bin/bash
# 4 MB native ladder: per-dispatch GPU costs (acquire fence, queue count, signalling grid).
out=${1:-gpurun_out/sweep_4mb_b.jsonl}
: > "$out"
for r in 1 2; do
  for e in "" "DORA_GPU_AQL_ACQUIRE=none" "DORA_GPU_AQL_QUEUES=2" "DORA_GPU_AQL_QUEUES=1" \
           "DORA_GPU_SIGNAL_GRID=256" "DORA_GPU_AQL_PRELOAD=0"; do
    args=""
    [ -n "$e" ] && args="--env $e"
    timeout -k 10 60 python scripts/native_tp.py --sizes 4096000 --n 3000 $args >> "$out" 2>&1 || exit 1
  done
done
