#!/bin/bash
# The sender's in-flight cap below 8 MiB (node.cpp max_in_flight): 10 (= the default queue_size,
# a receiver can never hold more ready inputs than it keeps) against r03's 11, on the native
# benchmark node's throughput mode, interleaved.  usage: bash scripts/cap_ab.sh <out dir> [rounds]
set -euo pipefail
out=${1:?out dir}; rounds=${2:-4}
mkdir -p "$out"
export TMPDIR=/tmp
for r in $(seq 1 "$rounds"); do
  for cap in 10 11; do
    timeout -k 10 200 python -u scripts/native_tp.py --sizes 4096,1048576,4096000 --n 2000 \
      --env DORA_GPU_MAX_IN_FLIGHT=$cap:8 > "$out/r${r}_cap$cap.jsonl" 2> "$out/r${r}_cap$cap.err"
    sed "s/^{/{\"run\": \"r${r}_cap$cap\", /" "$out/r${r}_cap$cap.jsonl" >> "$out/summary.jsonl"
  done
done
echo done
