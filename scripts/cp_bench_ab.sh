#!/bin/bash
# Interleaved full bench.py runs over fill-signal configurations (name=ENV pairs): the C3 block
# and the ladders of one box.   usage: bash scripts/cp_bench_ab.sh <out dir> <rounds> cfg...
set -o pipefail
out=${1:-gpurun_out/cpb}; rounds=${2:-2}; shift 2
mkdir -p "$out"
for r in $(seq 1 $rounds); do
  for cfg in "$@"; do
    name=${cfg%%=*}; kv=${cfg#*=}
    env $kv timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$out/bench_${name}_$r.json" 2> "$out/bench_${name}_$r.err" || { echo BENCH FAILED; exit 1; }
  done
done
echo ok
