#!/bin/bash
# Release fence none (default) vs agent on the C2 headline (40.96 MB, barrier packets), 1000 and
# 20 steps, interleaved.  Output: gpurun_out/release_headline_ab.jsonl.
export TMPDIR=/tmp
out=gpurun_out/release_headline_ab.jsonl
mkdir -p gpurun_out
for rep in 1 2 3; do
  for rel in none agent; do
    for steps in 1000 20; do
      line=$(DORA_GPU_AQL_RELEASE=$rel timeout -k 10 120 python bench.py --no-cpu-baseline --no-ladder --steps $steps --warmup 5) || exit $?
      echo "{\"release\": \"$rel\", \"steps\": $steps, \"bench\": $line}" >> $out
    done
  done
done
