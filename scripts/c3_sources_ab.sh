#!/bin/bash
# C3 vs a flat 13,000,068-B pack with the same number of rotating sources (16: 208 MB, inside
# the 256 MB Infinity Cache; 24: 312 MB, beyond it), interleaved.
# Output: gpurun_out/c3_sources_ab.jsonl.
export TMPDIR=/tmp
out=gpurun_out/c3_sources_ab.jsonl
mkdir -p gpurun_out
run() {
  tag=$1; shift
  line=$(timeout -k 10 120 python bench.py --no-cpu-baseline --no-ladder --steps 1000 "$@") || exit $?
  echo "{\"tag\": \"$tag\", \"bench\": $line}" >> $out
}
for rep in 1 2 3; do
  run c3_src24 --workload c3 --sources 24
  run flat_src24 --size 13000068 --sources 24
  run c3_src16 --workload c3 --sources 16
  run flat_src16 --size 13000068 --sources 16
  run c3_src48 --workload c3 --sources 48
done
