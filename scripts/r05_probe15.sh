#!/bin/bash
# Round-5 probes, fifteenth set: C3 blocks (three reps) and one with the sender's sub-phase
# profile, after trimming the flag-line loads of a multi-segment pack's dispatch.
# usage: bash scripts/r05_probe15.sh <out dir under gpurun_out>
set -euo pipefail
out=${1:?out dir}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/c3_burst_probe.py --reps 3 > "$out/c3.jsonl" 2> "$out/c3.err"
DORA_GPU_TRACE=subphases timeout -k 10 120 python -u scripts/c3_burst_probe.py --reps 1 \
  > "$out/c3_subphases.jsonl" 2> "$out/c3_subphases.err"
echo done
