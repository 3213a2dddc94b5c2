#!/bin/bash
# C3 with 16 lists (the config: x/y/z/intensity at sample offsets 4 mod 16, so every segment has
# byte-stored head/tail bytes and loads from the dword-shift path) against 15 lists (offsets
# 64 B: every buffer at 0 mod 16, no head/tail bytes), interleaved.
# Output: gpurun_out/c3_edges_ab.jsonl.
export TMPDIR=/tmp
out=gpurun_out/c3_edges_ab.jsonl
mkdir -p gpurun_out
run() {
  tag=$1; shift
  line=$(timeout -k 10 120 python bench.py --no-cpu-baseline --no-ladder --steps 1000 --workload c3 "$@") || exit $?
  echo "{\"tag\": \"$tag\", \"bench\": $line}" >> $out
}
for rep in 1 2 3; do
  run lists16 --c3-lists 16
  run lists15 --c3-lists 15
done
