#!/bin/bash
# AQL packet release fence: agent scope (default) vs none (DORA_GPU_AQL_RELEASE=none), on the
# native ladder at 4 MB / 16 MB and the C3 bench, interleaved.
# Output: gpurun_out/release_ab.jsonl.
export TMPDIR=/tmp
out=gpurun_out/release_ab.jsonl
mkdir -p gpurun_out
for rep in 1 2 3; do
  for rel in agent none; do
    timeout -k 10 180 python scripts/native_tp.py --sizes 4096000,16777216 --n 3000 \
      --env DORA_GPU_AQL_RELEASE=$rel | sed "s/^/{\"release\": \"$rel\", \"r\": /; s/\$/}/" >> $out || exit $?
    line=$(DORA_GPU_AQL_RELEASE=$rel timeout -k 10 120 python bench.py --workload c3 --no-cpu-baseline --no-ladder --steps 1000) || exit $?
    echo "{\"release\": \"$rel\", \"c3\": $line}" >> $out
  done
done
