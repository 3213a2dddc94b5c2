#!/bin/bash
# Headline (40.96 MB, 1000 steps) pack shape on the coherent-load kernel: chunk bytes and
# signalling grid, interleaved x2 (knobs in the process environment, inherited by every node).
# Output: gpurun_out/headline_coherent_ab.jsonl
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/headline_coherent_ab.jsonl
: > "$out"
for r in 1 2; do
  for v in "X=1" "DORA_GPU_PACK_CHUNK=16384" "DORA_GPU_PACK_CHUNK=4096" "DORA_GPU_SIGNAL_GRID=2048" \
           "DORA_GPU_SIGNAL_GRID=512" "DORA_GPU_AQL_COHERENT=0"; do
    line=$(env $v timeout -k 10 120 python bench.py --steps 1000 --no-ladder --no-cpu-baseline) || exit 1
    echo "{\"variant\": \"$v\", \"bench\": $line}" >> "$out"
  done
done
