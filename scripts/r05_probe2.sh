#!/bin/bash
# Round-5 probes, second set (each GPU step under its own limit; the first failure ends it):
#  1. the native node's throughput mode at 1 MiB from one resident source and from 64 rotating
#     sources (the bench ladder's), with the host sub-phase profile;
#  2. small device messages' latency by stage in bench.py's shape (scripts/small_lat_probe.py);
#  3. C3 blocks under multi-segment CP grid caps x in-flight caps from 8 MiB, interleaved.
# usage: bash scripts/r05_probe2.sh <out dir under gpurun_out>
set -euo pipefail
out=${1:?out dir}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/native_tp.py --sizes 1048576 --n 20000 \
  --env DORA_GPU_TRACE=subphases > "$out/native_tp_src1.jsonl" 2> "$out/native_tp_src1.err"
timeout -k 10 200 python -u scripts/native_tp.py --sizes 1048576 --n 20000 \
  --env DORA_GPU_TRACE=subphases --env DORA_BENCH_TP_SOURCES=64 > "$out/native_tp_src64.jsonl" \
  2> "$out/native_tp_src64.err"
timeout -k 10 150 python -u scripts/small_lat_probe.py --n 400 > "$out/small_lat.jsonl" \
  2> "$out/small_lat.err"
timeout -k 10 300 python -u scripts/c3_burst_probe.py --reps 2 --multi-grids 0,1024,1536 \
  --caps 8,12 > "$out/c3_combo.jsonl" 2> "$out/c3_combo.err"
echo done
