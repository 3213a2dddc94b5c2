#!/bin/bash
# In-flight cap 8 vs 12 at 1 MB / 4 MB (native node ladder), interleaved, one box.
mkdir -p gpurun_out
for rep in 1 2 3; do
  for f in 8 12; do
    DORA_GPU_MAX_IN_FLIGHT=$f timeout -k 10 120 python scripts/native_tp.py --sizes 1048576,4096000 --n 5000 \
      | sed "s/^{/{\"in_flight\": $f, /" >> gpurun_out/inflight_ab2.jsonl || exit $?
  done
done
