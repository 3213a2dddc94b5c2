#!/bin/bash
# 4 MB sender knobs on the native node with 16 rotating (HBM-resident) sources, interleaved.
# Earlier native_tp.py sweeps passed --env to the sinks only (fixed): their sender knobs were
# never applied.  Output: gpurun_out/knobs_4mb_hbm_ab.jsonl
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/knobs_4mb_hbm_ab.jsonl
: > "$out"
for r in 1 2; do
  for spec in "x" "DORA_BENCH_TP_SOURCES=1" "DORA_GPU_MAX_IN_FLIGHT=6" "DORA_GPU_MAX_IN_FLIGHT=20" \
              "DORA_GPU_AQL_QUEUES=2" "DORA_GPU_AQL_QUEUES=8" "DORA_GPU_AQL_BARRIER_BYTES=4000000" \
              "DORA_GPU_PACK_CHUNK=32768" "DORA_GPU_PACK_CHUNK=4096" "DORA_GPU_SIGNAL_GRID=256" \
              "DORA_GPU_AQL_ACQUIRE=none"; do
    args=(--env DORA_BENCH_TP_SOURCES=16)
    for kv in $spec; do [ "$kv" = x ] || args+=(--env "$kv"); done
    timeout -k 10 120 python scripts/native_tp.py --sizes 4096000 --n 20000 "${args[@]}" \
      >> "$out" || exit 1
  done
done
