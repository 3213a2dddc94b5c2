#!/bin/bash
# Round-5 probes, eleventh set: one C3 block under the message trace, reduced to per-send host
# stages of its 20-cloud burst (scripts/c3_send_trace.py).
# usage: bash scripts/r05_probe11.sh <out dir under gpurun_out>
set -euo pipefail
out=${1:?out dir}
mkdir -p "$out/trace"
export TMPDIR=/tmp
DORA_GPU_TRACE="$out/trace" timeout -k 10 150 python -u scripts/c3_burst_probe.py --reps 1 \
  > "$out/c3.jsonl" 2> "$out/c3.err"
python scripts/c3_send_trace.py "$out/trace" --n 20 > "$out/burst_sends.jsonl"
python scripts/c3_send_trace.py "$out/trace" --n 222 > "$out/steady_sends.jsonl"
echo done
