#!/bin/bash
# Round-5 probes, twelfth set: C3 blocks with 4 / 5 / 6 AQL queues taking the 13 MB clouds
# (three interleaved reps; 6 queues created).
# usage: bash scripts/r05_probe12.sh <out dir under gpurun_out>
set -euo pipefail
out=${1:?out dir}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/c3_burst_probe.py --reps 3 --mid-queues 4,5,6 \
  > "$out/c3_queues.jsonl" 2> "$out/c3_queues.err"
echo done
