#!/bin/bash
# In-flight cap for mid-size messages: native ladder at 4 MB / 13 MB / 16 MB and the C3 bench,
# caps 8 / 12 / 16 / 24, interleaved.  Output: gpurun_out/inflight_mid_ab.jsonl.
export TMPDIR=/tmp
out=gpurun_out/inflight_mid_ab.jsonl
mkdir -p gpurun_out
for rep in 1 2; do
  for cap in 8 12 16 24; do
    timeout -k 10 180 python scripts/native_tp.py --sizes 4096000,13000068,16777216 --n 3000 \
      --env DORA_GPU_MAX_IN_FLIGHT=$cap | sed "s/^/{\"cap\": $cap, \"r\": /; s/\$/}/" >> $out || exit $?
    line=$(DORA_GPU_MAX_IN_FLIGHT=$cap timeout -k 10 120 python bench.py --workload c3 --no-cpu-baseline --no-ladder --steps 1000) || exit $?
    echo "{\"cap\": $cap, \"c3\": $line}" >> $out
  done
done
