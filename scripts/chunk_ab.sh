#!/bin/bash
# 4 MB pack shape under a deep pipeline: chunk bytes per workgroup (DORA_GPU_PACK_CHUNK) x
# in-flight cap, native node ladder, 5000 messages.  Output: gpurun_out/chunk_ab.jsonl
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in "8192 24" "16384 24" "32768 24" "65536 24" "16384 32" "32768 32" "8192 24" "16384 24"; do
  set -- $spec
  timeout -k 10 150 python scripts/native_tp.py --sizes 1048576,4194304 --n 5000 \
    --env DORA_GPU_PACK_CHUNK=$1 --env DORA_GPU_MAX_IN_FLIGHT=$2 \
    >> gpurun_out/chunk_ab.jsonl || exit $?
done
