#!/bin/bash
# Coherent-load single-segment packs without the dispatch acquire fence (DORA_GPU_AQL_COHERENT=1)
# vs the default (plain nt loads + agent acquire): native ladder with sources rotated past the
# caches, 3 interleaved rounds, then the bench headline both ways.
# Output: gpurun_out/coherent_ab.jsonl
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/coherent_ab.jsonl
: > "$out"
for r in 1 2 3; do
  for c in 0 1; do
    for sz in "4096 64" "1048576 64" "4096000 64" "16777216 40"; do
      read -r size ns <<< "$sz"
      timeout -k 10 120 python scripts/native_tp.py --sizes $size --n 10000 \
        --env DORA_BENCH_TP_SOURCES=$ns --env DORA_GPU_AQL_COHERENT=$c >> "$out" || exit 1
    done
  done
done
for c in 0 1 0 1; do
  line=$(DORA_GPU_AQL_COHERENT=$c timeout -k 10 120 python bench.py --steps 1000 --no-ladder --no-cpu-baseline) || exit 1
  echo "{\"coherent\": $c, \"bench\": $line}" >> "$out"
done
