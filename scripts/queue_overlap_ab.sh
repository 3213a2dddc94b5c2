#!/bin/bash
# Do packs on one AQL queue overlap?  4 MB native ladder (sources rotated past the caches) on 1
# or 2 queues, without / with the barrier bit, with / without the acquire fence.  If the
# barrier bit changes nothing, consecutive packets of a queue already run one at a time.
# Output: gpurun_out/queue_overlap_ab.jsonl
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/queue_overlap_ab.jsonl
: > "$out"
for r in 1 2; do
  for spec in "1 0 agent" "1 4000000 agent" "1 0 none" "2 0 agent" "2 4000000 agent"; do
    set -- $spec
    timeout -k 10 120 python scripts/native_tp.py --sizes 4096000 --n 5000 \
      --env DORA_BENCH_TP_SOURCES=64 --env DORA_GPU_AQL_QUEUES=$1 \
      --env DORA_GPU_AQL_BARRIER_BYTES=$2 --env DORA_GPU_AQL_ACQUIRE=$3 >> "$out" || exit 1
  done
done
