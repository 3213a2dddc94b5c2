#!/bin/bash
# AQL queue count around the default 4 (3 / 4 / 5 / 6) at 4 MB and 16 MB, native node, sources
# rotated past the caches, two interleaved rounds.  Output: gpurun_out/queues_4mb_hbm_ab.jsonl
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/queues_4mb_hbm_ab.jsonl
: > "$out"
for r in 1 2; do
  for q in 3 4 5 6; do
    for spec in "4096000 64" "16777216 40"; do
      set -- $spec
      timeout -k 10 120 python scripts/native_tp.py --sizes $1 --n 10000 \
        --env DORA_BENCH_TP_SOURCES=$2 --env DORA_GPU_AQL_QUEUES=$q >> "$out" || exit 1
    done
  done
done
