#!/bin/bash
# Native ladder: one resident source vs 16 rotating copies (beyond what L2 holds), 4 MB and 16 MB.
out=${1:-gpurun_out/sources_4mb.jsonl}
: > "$out"
for r in 1 2; do
  for e in "DORA_BENCH_TP_SOURCES=1" "DORA_BENCH_TP_SOURCES=16"; do
    timeout -k 10 90 python scripts/native_tp.py --sizes 4096000,16777216 --n 10000 --env $e >> "$out" 2>&1 || exit 1
  done
done
