#!/bin/bash
# Kernel trace of the Python 4 MiB throughput run with and without CP-signalled packs: per AQL
# queue, how a packet's start relates to the previous packet's end (negative: they overlap).
#   usage: bash scripts/cp_queue_overlap.sh <out dir>; then python scripts/queue_gap_report.py <out dir>
set -euo pipefail
out=${1:?out dir}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d "$out/cp" -o run -- \
  python scripts/py_tp.py --sizes 4194304 --n 2000 > "$out/cp_tp.json" 2> "$out/cp.err"
DORA_GPU_AQL_CP_SIGNAL=0 timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d "$out/kernel" -o run -- \
  python scripts/py_tp.py --sizes 4194304 --n 2000 > "$out/kernel_tp.json" 2> "$out/kernel.err"
echo done
