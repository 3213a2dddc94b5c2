#!/bin/bash
# Latency ladder p50/p99 with kernel arguments preloaded from the host ring (default) vs read from
# the device ring (DORA_GPU_AQL_PRELOAD=0): does the command processor's PCIe read of the
# preload arguments show up in small-message latency?  Two interleaved rounds, 300 messages.
# Output: gpurun_out/lat_preload_ab.jsonl
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/lat_preload_ab.jsonl
: > "$out"
for r in 1 2; do
  for p in 1 0; do
    line=$(DORA_GPU_AQL_PRELOAD=$p timeout -k 10 180 python bench.py --steps 50 --warmup 5 --tp-n 0 \
      --lat-n 300 --no-cpu-baseline) || exit 1
    echo "{\"preload\": $p, \"bench\": $line}" >> "$out"
  done
done
