#!/bin/bash
# Round-5 probes, twentieth set: the keep-awake test, the warm thread against a HIP stream with
# the process's CPU time (scripts/warm_copy_probe.py, off / on, two rounds), and the driver's
# bench command at the default.
# usage: bash scripts/r05_probe20.sh <out dir under gpurun_out>
set -euo pipefail
out=${1:?out dir}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_keep_awake.py -x -v --timeout 120 --timeout-method thread > "$out/tests.log" 2>&1
for r in 0 1; do
  for w in 0 25; do
    timeout -k 10 120 python -u scripts/warm_copy_probe.py --n 300 --keep-awake-us $w \
      >> "$out/warm_copy.jsonl" 2>> "$out/warm_copy.err"
  done
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --detail "$out/bench_detail.json" > "$out/bench.json" 2> "$out/bench.err"
echo done
