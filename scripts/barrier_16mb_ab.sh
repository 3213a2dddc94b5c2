#!/bin/bash
# 16 MB on the coherent build: barrier bit from 16 MB (in order per queue, <= 3 queues, as the
# 40.96 MB packs) vs overlapping packs on 4 queues; sources rotated past the caches, 3 rounds.
# Output: gpurun_out/barrier_16mb_ab.jsonl
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/barrier_16mb_ab.jsonl
: > "$out"
for r in 1 2 3; do
  for b in 33554432 16000000 8000000; do
    for sz in "16777216 40" "13000068 50"; do
      read -r size ns <<< "$sz"
      timeout -k 10 120 python scripts/native_tp.py --sizes $size --n 3000 \
        --env DORA_BENCH_TP_SOURCES=$ns --env DORA_GPU_AQL_BARRIER_BYTES=$b >> "$out" || exit 1
    done
  done
done
