#!/bin/bash
# C3 (16 lists: bodies at 16 mod 64) and the same cloud with 15 lists (bodies at 0 mod 64),
# chunks from the body's cache line (default) vs from its first aligned unit
# (DORA_GPU_LINE_CHUNKS=0, the r01 layout), interleaved.  Output: gpurun_out/c3_line_ab.jsonl.
export TMPDIR=/tmp
out=gpurun_out/c3_line_ab.jsonl
mkdir -p gpurun_out
run() {
  tag=$1; envv=$2; lists=$3
  line=$(timeout -k 10 120 env $envv python bench.py --no-cpu-baseline --no-ladder --steps 1000 --workload c3 --c3-lists $lists) || exit $?
  echo "{\"tag\": \"$tag\", \"bench\": $line}" >> $out
}
for rep in 1 2 3; do
  run lists16_line DORA_X=1 16
  run lists16_unit DORA_GPU_LINE_CHUNKS=0 16
  run lists15_line DORA_X=1 15
  run lists15_unit DORA_GPU_LINE_CHUNKS=0 15
done
