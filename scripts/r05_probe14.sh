#!/bin/bash
# Round-5 probes, fourteenth set: small-message latency by stage with the GPU idle between
# messages (default) and kept awake by one resident sleeping wave (--warm), twice each.
# usage: bash scripts/r05_probe14.sh <out dir under gpurun_out>
set -euo pipefail
out=${1:?out dir}
mkdir -p "$out"
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 150 python -u scripts/small_lat_probe.py --n 300 >> "$out/small_lat.jsonl" \
    2>> "$out/small_lat.err"
  timeout -k 10 150 python -u scripts/small_lat_probe.py --n 300 --warm >> "$out/small_lat.jsonl" \
    2>> "$out/small_lat.err"
done
echo done
