#!/bin/bash
# 4 MB packs in order per queue (barrier bit, 3 queues) vs overlapping, x in-flight cap, native
# node ladder, 5000 messages.  Output: gpurun_out/barrier_4mb_ab.jsonl
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in "0 12" "4000000 12" "4000000 24" "0 24" "0 12" "4000000 12"; do
  set -- $spec
  timeout -k 10 150 python scripts/native_tp.py --sizes 1048576,4194304 --n 5000 \
    --env DORA_GPU_AQL_BARRIER_BYTES=$1 --env DORA_GPU_MAX_IN_FLIGHT=$2 \
    >> gpurun_out/barrier_4mb_ab.jsonl || exit $?
done
