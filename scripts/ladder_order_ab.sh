#!/bin/bash
# bench.py with the native ladder before (default) / after (DORA_BENCH_LADDER_LATE=1) this
# process opens the GPU, interleaved.  Output: gpurun_out/ladder_order_ab.jsonl
mkdir -p gpurun_out
for late in 0 1 0 1; do
  DORA_BENCH_LADDER_LATE=$late timeout -k 10 200 python bench.py --no-cpu-baseline \
    | sed "s/^{/{\"ladder_late\": $late, /" >> gpurun_out/ladder_order_ab.jsonl || exit $?
done
