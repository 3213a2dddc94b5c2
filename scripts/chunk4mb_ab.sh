#!/bin/bash
# 4 MB native ladder under overlapping AQL packs: chunk bytes per workgroup (8 KiB default ->
# 512 workgroups; 16 KiB; 32 KiB with 8 loads in flight) and the signalling grid, interleaved.
# Output: gpurun_out/chunk4mb_ab.jsonl.
export TMPDIR=/tmp
out=gpurun_out/chunk4mb_ab.jsonl
mkdir -p gpurun_out
run() {
  tag=$1; shift
  args=""
  for kv in "$@"; do args="$args --env $kv"; done
  timeout -k 10 180 python scripts/native_tp.py --sizes 4096000 --n 3000 $args \
    | sed "s/^/{\"tag\": \"$tag\", \"r\": /; s/\$/}/" >> $out || exit $?
}
for rep in 1 2 3; do
  run default DORA_X=1
  run c16k DORA_GPU_PACK_CHUNK=16384
  run c32k_u8 DORA_GPU_PACK_CHUNK=32768 DORA_GPU_PACK_VARIANT=u8nt
  run c4k DORA_GPU_PACK_CHUNK=4096
done
