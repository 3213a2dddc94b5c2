#!/bin/bash
# 4 MB native-ladder knob sweep (interleaved, 2 rounds): in-flight cap, chunk shape, AQL queues.
out=${1:-gpurun_out/sweep_4mb.jsonl}
: > "$out"
for r in 1 2; do
  for e in "" "DORA_GPU_MAX_IN_FLIGHT=16" "DORA_GPU_MAX_IN_FLIGHT=24" "DORA_GPU_PACK_CHUNK=16384" \
           "DORA_GPU_PACK_CHUNK=32768" "DORA_GPU_AQL_QUEUES=6" "DORA_GPU_AQL_QUEUES=8"; do
    args=""
    [ -n "$e" ] && args="--env $e"
    timeout -k 10 60 python scripts/native_tp.py --sizes 4096000 --n 3000 $args >> "$out" 2>&1 || exit 1
  done
done
