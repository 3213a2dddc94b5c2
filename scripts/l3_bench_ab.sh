#!/bin/bash
# bench.py (headline, latency ladder, native ladder) with and without L3-domain placement,
# interleaved on one box.  Output: gpurun_out/l3_bench_ab.jsonl
mkdir -p gpurun_out
for v in 1 0 1 0; do
  DORA_GPU_PIN_L3=$v timeout -k 10 200 python bench.py --no-cpu-baseline \
    | sed "s/^{/{\"pin_l3\": $v, /" >> gpurun_out/l3_bench_ab.jsonl || exit $?
done
