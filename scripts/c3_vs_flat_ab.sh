#!/bin/bash
# Where C3's GPU time goes: the 13,000,068-B C3 sample (7 segments, f32 buffers at 4 mod 16)
# against one flat 13,000,068-B UInt8 pack from an aligned source, a source at 4 mod 16 (the
# dword-shift load path) and at 1 mod 16 (the byte funnel), interleaved.
# Output: gpurun_out/c3_vs_flat_ab.jsonl.
export TMPDIR=/tmp
out=gpurun_out/c3_vs_flat_ab.jsonl
mkdir -p gpurun_out
run() {
  tag=$1; shift
  line=$(timeout -k 10 120 python bench.py --no-cpu-baseline --no-ladder --steps 1000 "$@") || exit $?
  echo "{\"tag\": \"$tag\", \"bench\": $line}" >> $out
}
for rep in 1 2 3; do
  run c3 --workload c3
  run flat_off0 --size 13000068
  run flat_off4 --size 13000068 --src-offset 4
  run flat_off1 --size 13000068 --src-offset 1
done
