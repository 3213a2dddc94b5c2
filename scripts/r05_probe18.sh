#!/bin/bash
# Round-5 probes, eighteenth set: the warm thread (aql.cpp warm_main) on (25 us) and off (0): the
# GPU tests with it on, then three interleaved rounds of the driver's bench command and of
# scripts/small_lat_probe.py per side.  (profiles/r05_keep_awake_ab_ze.jsonl was run at commit
# 395dc61, where an environment variable set the period; these flags do the same.)
# usage: bash scripts/r05_probe18.sh <out dir under gpurun_out>
set -euo pipefail
out=${1:?out dir}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1
for r in 0 1 2; do
  for tag in off on; do
    if [ $tag = off ]; then w=0; else w=25; fi
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --keep-awake-us $w \
      --detail "$out/d_${tag}_$r.json" > "$out/b_${tag}_$r.json" 2> "$out/e_${tag}_$r.log"
    timeout -k 10 120 python -u scripts/small_lat_probe.py --n 300 --keep-awake-us $w \
      >> "$out/small_lat.jsonl" 2>> "$out/small_lat.err"
  done
done
echo done
