#!/bin/bash
# Queue count and in-flight cap on the coherent-load build (4 MB / 16 MB, sources rotated past
# the caches), two interleaved rounds.  Output: gpurun_out/coherent_knobs_ab.jsonl
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/coherent_knobs_ab.jsonl
: > "$out"
for r in 1 2; do
  for spec in "DORA_GPU_AQL_QUEUES=4" "DORA_GPU_AQL_QUEUES=3" "DORA_GPU_AQL_QUEUES=5" \
              "DORA_GPU_MAX_IN_FLIGHT=8" "DORA_GPU_MAX_IN_FLIGHT=16"; do
    for sz in "4096000 64" "16777216 40"; do
      read -r size ns <<< "$sz"
      timeout -k 10 120 python scripts/native_tp.py --sizes $size --n 10000 \
        --env DORA_BENCH_TP_SOURCES=$ns --env "$spec" >> "$out" || exit 1
    done
  done
done
