#!/bin/bash
# 8-32 MB packs: 8 loads in flight per lane over 32 KiB chunks (the r01 default for that range)
# vs 4 loads over 8 KiB chunks (the >= 32 MB shape), on C3, a flat 13 MB pack and the native
# 16 MB ladder, interleaved.  Output: gpurun_out/u4_mid_ab.jsonl.
export TMPDIR=/tmp
out=gpurun_out/u4_mid_ab.jsonl
mkdir -p gpurun_out
run() {
  tag=$1; envv=$2; shift 2
  line=$(timeout -k 10 120 env $envv python bench.py --no-cpu-baseline --no-ladder --steps 1000 "$@") || exit $?
  echo "{\"tag\": \"$tag\", \"bench\": $line}" >> $out
}
nat() {
  tag=$1; envv=$2
  timeout -k 10 180 python scripts/native_tp.py --sizes 16777216 --n 2000 --env $envv \
    | sed "s/^/{\"tag\": \"$tag\", \"r\": /; s/\$/}/" >> $out || exit $?
}
for rep in 1 2; do
  run c3_u8 DORA_X=1 --workload c3
  run c3_u4 DORA_GPU_PACK_VARIANT=u4nt --workload c3
  run c3_u4_c16k "DORA_GPU_PACK_VARIANT=u4nt DORA_GPU_PACK_CHUNK=16384" --workload c3
  run c3_u4_g2048 "DORA_GPU_PACK_VARIANT=u4nt DORA_GPU_SIGNAL_GRID=2048" --workload c3
  run flat_u8 DORA_X=1 --size 13000068
  run flat_u4 DORA_GPU_PACK_VARIANT=u4nt --size 13000068
  nat n16_u8 DORA_X=1
  nat n16_u4 DORA_GPU_PACK_VARIANT=u4nt
done
