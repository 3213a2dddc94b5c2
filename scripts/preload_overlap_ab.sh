#!/bin/bash
# Kernarg preload (arguments from the host ring, preloaded into SGPRs) vs the device argument
# ring, on 1 and 4 AQL queues: does preloading serialise consecutive packs of a queue?  4 MB,
# sources rotated past the caches, two interleaved rounds.  Output: gpurun_out/preload_overlap_ab.jsonl
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/preload_overlap_ab.jsonl
: > "$out"
for r in 1 2; do
  for spec in "1 1" "1 0" "4 1" "4 0"; do
    set -- $spec
    timeout -k 10 120 python scripts/native_tp.py --sizes 4096000 --n 5000 \
      --env DORA_BENCH_TP_SOURCES=64 --env DORA_GPU_AQL_QUEUES=$1 \
      --env DORA_GPU_AQL_PRELOAD=$2 >> "$out" || exit 1
  done
done
