#!/bin/bash
# Latency ladder (1 ms between messages) with consumers that sleep after the default 200 us of
# spinning vs consumers that keep spinning through the gap (DORA_GPU_SPIN_US=5000), interleaved.
# Output: gpurun_out/spin_latency_ab.jsonl.
export TMPDIR=/tmp
out=gpurun_out/spin_latency_ab.jsonl
mkdir -p gpurun_out
for rep in 1 2; do
  for spin in 200 5000; do
    line=$(DORA_GPU_SPIN_US=$spin timeout -k 10 200 python bench.py --no-cpu-baseline --tp-n 0 --steps 100) || exit $?
    echo "{\"spin_us\": $spin, \"bench\": $line}" >> $out
  done
done
