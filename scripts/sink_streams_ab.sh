#!/bin/bash
# Bench sink with its default 3 fill streams vs one (DORA_GPU_FILL_STREAMS=1 in the sink only:
# fewer hardware queues on the GPU), C2 headline and C3, interleaved.
mkdir -p gpurun_out
for fs in 3 1 3 1; do
  for w in c2 c3; do
    DORA_BENCH_SINK_DORA_GPU_FILL_STREAMS=$fs timeout -k 10 200 python bench.py --no-cpu-baseline --no-ladder --workload $w \
      | sed "s/^{/{\"sink_fill_streams\": $fs, /" >> gpurun_out/sink_streams_ab.jsonl || exit $?
  done
done
