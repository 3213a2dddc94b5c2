#!/bin/bash
# Where the C3 pack's extra device time comes from: a flat 13,000,068-B pack through the
# multi-segment kernel (device argument ring, DORA_GPU_AQL_PRELOAD=0) and C3 without the
# validity tail segments (DORA_GPU_VALIDITY=inline), against the defaults, interleaved.
# Output: gpurun_out/c3_overhead_ab.jsonl.
export TMPDIR=/tmp
out=gpurun_out/c3_overhead_ab.jsonl
mkdir -p gpurun_out
run() {
  tag=$1; shift
  line=$(timeout -k 10 120 env "$@") || exit $?
  echo "{\"tag\": \"$tag\", \"bench\": $line}" >> $out
}
B="python bench.py --no-cpu-baseline --no-ladder --steps 1000"
for rep in 1 2 3; do
  run c3 DORA_X=1 $B --workload c3
  run c3_inline DORA_GPU_VALIDITY=inline $B --workload c3
  run flat DORA_X=1 $B --size 13000068
  run flat_devargs DORA_GPU_AQL_PRELOAD=0 $B --size 13000068
  run flat_off4_devargs DORA_GPU_AQL_PRELOAD=0 $B --size 13000068 --src-offset 4
done
