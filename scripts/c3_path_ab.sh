#!/bin/bash
# C3 (13 MB nested packs) on the AQL queues (default, < 32 MiB) vs the HIP fill streams
# (DORA_GPU_AQL_MAX_BYTES=8 MiB), interleaved.  Output: gpurun_out/c3_path_ab.jsonl
mkdir -p gpurun_out
for m in default 8388608 default 8388608; do
  if [ $m = default ]; then unset DORA_GPU_AQL_MAX_BYTES; else export DORA_GPU_AQL_MAX_BYTES=$m; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-ladder --workload c3 \
    | sed "s/^{/{\"aql_max\": \"$m\", /" >> gpurun_out/c3_path_ab.jsonl || exit $?
done
