#!/bin/bash
# Round-5 probes, thirteenth set: C3 blocks with the sender's in-flight cap from 8 MiB at 8 (the
# default) or 11 (the small-sample cap: queue_size + 1), four interleaved reps.
# usage: bash scripts/r05_probe13.sh <out dir under gpurun_out>
set -euo pipefail
out=${1:?out dir}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/c3_burst_probe.py --reps 4 --caps 8,11 \
  > "$out/c3_caps.jsonl" 2> "$out/c3_caps.err"
echo done
