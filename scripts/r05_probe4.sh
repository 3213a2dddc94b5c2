#!/bin/bash
# Round-5 probes, fourth set (each GPU step under its own limit; the first failure ends it):
#  1. the host's other ways to read a device sample < 4096 B (scripts/small_path_probe.py);
#  2. C3 blocks under multi-segment CP grid caps 640/768/896, with and without the full grid
#     for a multi-segment pack dispatched onto idle queues (the burst's first cloud).
# usage: bash scripts/r05_probe4.sh <out dir under gpurun_out>
set -euo pipefail
out=${1:?out dir}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 60 python -u scripts/small_path_probe.py --n 300 > "$out/small_path.jsonl" \
  2> "$out/small_path.err"
timeout -k 10 400 python -u scripts/c3_burst_probe.py --reps 2 --multi-grids 640,768,896 \
  --lone-grids 0,3584 > "$out/c3_combo.jsonl" 2> "$out/c3_combo.err"
echo done
