#!/bin/bash
# Round-5 probes, third set (each GPU step under its own limit; the first failure ends it):
#  1. native 1 MiB throughput from 1 and 64 rotating sources and the Python node from 64,
#     interleaved twice (is the 64-source native gap the sources or the box?);
#  2. C3 blocks under multi-segment CP grid caps 1280/1024/768/512 x in-flight caps 8/12.
# usage: bash scripts/r05_probe3.sh <out dir under gpurun_out>
set -euo pipefail
out=${1:?out dir}
mkdir -p "$out"
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 120 python -u scripts/native_tp.py --sizes 1048576 --n 20000 \
    --env DORA_GPU_TRACE=subphases >> "$out/tp_native_src1.jsonl" 2>> "$out/tp.err"
  timeout -k 10 120 python -u scripts/native_tp.py --sizes 1048576 --n 20000 \
    --env DORA_GPU_TRACE=subphases --env DORA_BENCH_TP_SOURCES=64 >> "$out/tp_native_src64.jsonl" \
    2>> "$out/tp.err"
  DORA_GPU_TRACE=subphases timeout -k 10 120 python -u scripts/py_tp.py --sizes 1048576 \
    --sources 64 --n 20000 >> "$out/tp_py_src64.jsonl" 2>> "$out/tp.err"
done
timeout -k 10 400 python -u scripts/c3_burst_probe.py --reps 2 --multi-grids 1280,1024,768,512 \
  --caps 8,12 > "$out/c3_combo.jsonl" 2> "$out/c3_combo.err"
echo done
