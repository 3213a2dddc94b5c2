#!/bin/bash
# Same-box A/B of two library builds (DORA_GPU_LIB, bench.py's node only): this tree's vs the
# r02 build before stitched boundary units and line-aligned chunks (build/ab_old, built from
# commit af83976), on C3 and on a flat 13 MB pack.  Output: gpurun_out/pack_build_ab.jsonl.
export TMPDIR=/tmp
out=gpurun_out/pack_build_ab.jsonl
mkdir -p gpurun_out
OLD=$PWD/build/ab_old/libdora_gpu.so
run() {
  tag=$1; envv=$2; shift 2
  line=$(timeout -k 10 120 env $envv python bench.py --no-cpu-baseline --no-ladder --steps 1000 "$@") || exit $?
  echo "{\"tag\": \"$tag\", \"bench\": $line}" >> $out
}
for rep in 1 2 3; do
  run c3_new DORA_X=1 --workload c3
  run c3_old DORA_GPU_LIB=$OLD --workload c3
  run c3_new_unit DORA_GPU_LINE_CHUNKS=0 --workload c3
  run flat_new DORA_X=1 --size 13000068
  run flat_old DORA_GPU_LIB=$OLD --size 13000068
done
