#!/bin/bash
# Round-5 probes, nineteenth set: the warm thread against a HIP stream of the same process
# (scripts/warm_copy_probe.py, off / on, two rounds), then the GPU tests with it on.
# (profiles/r05_warm_copy_zd.jsonl was run at commit 395dc61, where an environment variable set
# the period; --keep-awake-us does the same.)
# usage: bash scripts/r05_probe19.sh <out dir under gpurun_out>
set -euo pipefail
out=${1:?out dir}
mkdir -p "$out"
export TMPDIR=/tmp
for r in 0 1; do
  for w in 0 25; do
    timeout -k 10 120 python -u scripts/warm_copy_probe.py --n 300 --keep-awake-us $w \
      >> "$out/warm_copy.jsonl" 2>> "$out/warm_copy.err"
  done
done
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1
echo done
