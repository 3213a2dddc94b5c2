#!/bin/bash
# C3 (multi-segment packs): coherent argument + source loads without the acquire fence
# (DORA_GPU_AQL_COHERENT=all; the default before this A/B) vs the fenced kernel, bench.py 1000 steps, interleaved x3.
# Output: gpurun_out/coherent_c3_ab.jsonl
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/coherent_c3_ab.jsonl
: > "$out"
for r in 1 2 3; do
  for c in all 1; do
    line=$(DORA_GPU_AQL_COHERENT=$c timeout -k 10 120 python bench.py --workload c3 --steps 1000 \
      --no-ladder --no-cpu-baseline) || exit 1
    echo "{\"coherent\": \"$c\", \"bench\": $line}" >> "$out"
  done
done
