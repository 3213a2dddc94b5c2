#!/bin/bash
# 4 MB chunk bytes on the coherent kernel (sources rotated past the caches): 8 KiB (default,
# 500 workgroups) vs 16 KiB (250, one load batch each) vs 12 KiB, interleaved x3.
# Output: gpurun_out/chunk_4mb_coherent_ab.jsonl
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/chunk_4mb_coherent_ab.jsonl
: > "$out"
for r in 1 2 3; do
  for c in 8192 16384 12288; do
    timeout -k 10 120 python scripts/native_tp.py --sizes 4096000,1048576 --n 10000 \
      --env DORA_BENCH_TP_SOURCES=64 --env DORA_GPU_PACK_CHUNK=$c >> "$out" || exit 1
  done
done
