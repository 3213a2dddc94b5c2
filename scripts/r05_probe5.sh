#!/bin/bash
# Round-5 probes, fifth set: C3 blocks under multi-segment CP grid caps 640/704/768 (three
# interleaved reps), then one rep with the sender's host sub-phase profile (per-cloud host cost).
# usage: bash scripts/r05_probe5.sh <out dir under gpurun_out>
set -euo pipefail
out=${1:?out dir}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/c3_burst_probe.py --reps 3 --multi-grids 640,704,768 \
  > "$out/c3_combo.jsonl" 2> "$out/c3_combo.err"
DORA_GPU_TRACE=subphases timeout -k 10 120 python -u scripts/c3_burst_probe.py --reps 1 \
  --multi-grids 704 > "$out/c3_subphases.jsonl" 2> "$out/c3_subphases.err"
echo done
