#!/bin/bash
# Size-dependent in-flight cap (default: 12 below 8 MiB, 8 above) vs a flat 8, interleaved:
# native node ladder and bench.py (headline + ladders).  Output: gpurun_out/inflight_size_ab.jsonl
mkdir -p gpurun_out
for cap in default 8 default 8; do
  if [ $cap = default ]; then unset DORA_GPU_MAX_IN_FLIGHT; else export DORA_GPU_MAX_IN_FLIGHT=$cap; fi
  timeout -k 10 120 python scripts/native_tp.py --sizes 65536,1048576,4096000 --n 5000 \
    | sed "s/^{/{\"cap\": \"$cap\", /" >> gpurun_out/inflight_size_ab.jsonl || exit $?
  timeout -k 10 200 python bench.py --no-cpu-baseline \
    | sed "s/^{/{\"cap\": \"$cap\", /" >> gpurun_out/inflight_size_ab.jsonl || exit $?
done
