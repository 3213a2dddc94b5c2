#!/bin/bash
# Round-5 probes, sixteenth set: C3 blocks with the packs' packets published before (0) or after
# (1) their descriptors (dora_gpu_test_defer_doorbell), interleaved, six reps each.
# usage: bash scripts/r05_probe16.sh <out dir under gpurun_out>
set -euo pipefail
out=${1:?out dir}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_dataflow.py -k big_multi_segment_async > "$out/tests.log" 2>&1
timeout -k 10 400 python -u scripts/c3_burst_probe.py --reps 6 --defer 0,1 > "$out/c3.jsonl" 2> "$out/c3.err"
echo done
