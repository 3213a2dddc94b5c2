#!/bin/bash
# Round-5 distribution: the driver's bench command N times back to back on one box (each run
# under its own limit).   usage: bash scripts/r05_dist.sh <out dir under gpurun_out> [N]
set -euo pipefail
out=${1:?out dir}
n=${2:-5}
mkdir -p "$out"
export TMPDIR=/tmp
for r in $(seq 1 "$n"); do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --detail "$out/d_head_$r.json" \
    > "$out/b_head_$r.json" 2> "$out/b_head_$r.err"
done
echo done
