#!/bin/bash
# 4 MB concurrency A/B on the native node ladder (20000 messages): overlapping packs (default)
# vs packs in order per queue (barrier bit from 4 MB: at most 3 concurrent) vs lower in-flight
# caps.  The 40.96 MB pack is faster with fewer concurrent copies; is 4 MB too?
# Output: gpurun_out/conc_4mb_ab.jsonl
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/conc_4mb_ab.jsonl
for r in 1 2 3; do
  for spec in "x" "DORA_GPU_AQL_BARRIER_BYTES=4000000" "DORA_GPU_MAX_IN_FLIGHT=4" \
              "DORA_GPU_MAX_IN_FLIGHT=6" "DORA_GPU_AQL_BARRIER_BYTES=4000000 DORA_GPU_MAX_IN_FLIGHT=6"; do
    args=()
    for kv in $spec; do [ "$kv" = x ] || args+=(--env "$kv"); done
    timeout -k 10 120 python scripts/native_tp.py --sizes 4096000,16777216 --n 20000 "${args[@]}" \
      >> gpurun_out/conc_4mb_ab.jsonl || exit $?
  done
done
