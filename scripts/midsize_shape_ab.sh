#!/bin/bash
# Mid-size packs (13 MB: the C3 cloud and one flat UInt8 sample of the same size) under
# overlapping AQL dispatch: chunk shape, loads in flight per lane, signalling grid, barrier.
# Output: gpurun_out/midsize_shape_ab.jsonl.
export TMPDIR=/tmp
out=gpurun_out/midsize_shape_ab.jsonl
mkdir -p gpurun_out
run() {
  tag=$1; wl=$2; shift 2
  if [ "$wl" = c3 ]; then a="--workload c3"; else a="--size 13000068"; fi
  line=$(env "$@" timeout -k 10 120 python bench.py --no-cpu-baseline --no-ladder --steps 1000 $a) || exit $?
  echo "{\"tag\": \"$tag\", \"wl\": \"$wl\", \"bench\": $line}" >> $out
}
for rep in 1 2; do
  for wl in c3 flat; do
    run default $wl DORA_NOTHING=1
    run u4_8k $wl DORA_GPU_PACK_VARIANT=u4nt DORA_GPU_PACK_CHUNK=8192
    run u4_16k $wl DORA_GPU_PACK_VARIANT=u4nt DORA_GPU_PACK_CHUNK=16384
    run u8_32k_g256 $wl DORA_GPU_SIGNAL_GRID=256
    run u4_8k_g2048 $wl DORA_GPU_PACK_VARIANT=u4nt DORA_GPU_PACK_CHUNK=8192 DORA_GPU_SIGNAL_GRID=2048
    run u4_8k_g512 $wl DORA_GPU_PACK_VARIANT=u4nt DORA_GPU_PACK_CHUNK=8192 DORA_GPU_SIGNAL_GRID=512
  done
done
