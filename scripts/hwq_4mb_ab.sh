#!/bin/bash
# HIP hardware queues per process (GPU_MAX_HW_QUEUES, HIP's default 4) x AQL queues per sender:
# the 4 MB / 16 MB native ladder (sources rotated past the caches) falls 2-3x from 5 AQL queues up
# (r02_queues_4mb_hbm_ab.jsonl), as if the dataflow's queues then outnumber the hardware queue
# slots.  Two interleaved rounds.  Output: gpurun_out/hwq_4mb_ab.jsonl
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/hwq_4mb_ab.jsonl
: > "$out"
for r in 1 2; do
  for spec in "d 4" "1 4" "1 6" "1 8" "2 4" "2 6"; do
    set -- $spec
    for sz in "4096000 64" "16777216 40"; do
      read -r size ns <<< "$sz"
      if [ "$1" = d ]; then
        timeout -k 10 120 python scripts/native_tp.py --sizes $size --n 10000 \
          --env DORA_BENCH_TP_SOURCES=$ns --env DORA_GPU_AQL_QUEUES=$2 \
          | sed "s/^{/{\"hwq\": \"default\", /" >> "$out" || exit 1
      else
        GPU_MAX_HW_QUEUES=$1 timeout -k 10 120 python scripts/native_tp.py --sizes $size --n 10000 \
          --env DORA_BENCH_TP_SOURCES=$ns --env DORA_GPU_AQL_QUEUES=$2 \
          | sed "s/^{/{\"hwq\": $1, /" >> "$out" || exit 1
      fi
    done
  done
done
