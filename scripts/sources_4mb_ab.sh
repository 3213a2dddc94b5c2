#!/bin/bash
# 4 MB source residency A/B on one box, interleaved: native node and Python node, one resident
# source (Infinity-Cache resident after the first pass) vs 16 / 64 rotating sources
# (64 MB / 256 MB).  Output: gpurun_out/sources_4mb_ab.jsonl
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/sources_4mb_ab.jsonl
: > "$out"
for r in 1 2; do
  for n in 1 16 64; do
    timeout -k 10 120 python scripts/native_tp.py --sizes 4096000 --n 20000 \
      --env DORA_BENCH_TP_SOURCES=$n | sed "s/^{/{\"who\": \"native\", \"sources\": $n, /" >> "$out" || exit 1
    timeout -k 10 120 python scripts/py_tp.py --sizes 4096000 --n 20000 --sources $n \
      | sed "s/^{/{\"who\": \"python\", \"sources\": $n, /" >> "$out" || exit 1
  done
done
