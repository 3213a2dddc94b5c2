#!/bin/bash
# bench.py headline + ladders and the C3 workload at in-flight caps 12 and 8, interleaved.
# Output: gpurun_out/inflight_bench_ab.jsonl
mkdir -p gpurun_out
for f in 12 8 12 8; do
  DORA_GPU_MAX_IN_FLIGHT=$f timeout -k 10 200 python bench.py --no-cpu-baseline \
    | sed "s/^{/{\"in_flight\": $f, /" >> gpurun_out/inflight_bench_ab.jsonl || exit $?
  DORA_GPU_MAX_IN_FLIGHT=$f timeout -k 10 200 python bench.py --no-cpu-baseline --workload c3 \
    | sed "s/^{/{\"in_flight\": $f, /" >> gpurun_out/inflight_bench_ab.jsonl || exit $?
done
