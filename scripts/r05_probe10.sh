#!/bin/bash
# Round-5 probes, tenth set: the synchronous 40.96 MB send's completion path (scripts/sync_probe.py).
# usage: bash scripts/r05_probe10.sh <out dir under gpurun_out>
set -euo pipefail
out=${1:?out dir}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/sync_probe.py --reps 3 --n 200 --modes cp,k1024,k2048,k3584 \
  > "$out/sync_probe.jsonl" 2> "$out/sync_probe.err"
echo done
