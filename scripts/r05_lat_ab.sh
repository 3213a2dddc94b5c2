#!/bin/bash
# Round-5 A/B: the round-4 tree (git worktree ./wt04 at db00df7, built in place) against HEAD,
# full bench runs interleaved three times on one box: the latency ladder (device 8 B / 4 KB
# p50), the headline and the ladders.   usage: bash scripts/r05_lat_ab.sh <out dir under gpurun_out>
set -euo pipefail
out=$(cd "$(dirname "$1")" && pwd)/$(basename "$1")
mkdir -p "$out"
export TMPDIR=/tmp
root=$(pwd)
for r in 1 2 3; do
  (cd "$root/wt04" && timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline \
    --lat-n 300 --detail "$out/d_r04_$r.json" > "$out/b_r04_$r.json" 2> "$out/b_r04_$r.err")
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --lat-n 300 \
    --detail "$out/d_r05_$r.json" > "$out/b_r05_$r.json" 2> "$out/b_r05_$r.err"
done
echo done
