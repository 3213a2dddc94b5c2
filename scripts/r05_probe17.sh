#!/bin/bash
# Round-5 probes, seventeenth set: does a periodic touch keep the GPU's dispatch side awake
# between small messages 1 ms apart?  scripts/small_lat_probe.py without (0) and with a host
# thread that every 40 us publishes an empty AQL packet (1), reads (2) or writes (3) a word of
# device memory over PCIe; two interleaved rounds.
# usage: bash scripts/r05_probe17.sh <out dir under gpurun_out>
set -euo pipefail
out=${1:?out dir}
mkdir -p "$out"
export TMPDIR=/tmp
for r in 0 1; do
  for m in 0 1 2 3; do
    timeout -k 10 120 python -u scripts/small_lat_probe.py --n 300 --heartbeat $m \
      >> "$out/small_lat.jsonl" 2>> "$out/small_lat.err"
  done
done
echo done
