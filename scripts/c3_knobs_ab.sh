#!/bin/bash
# C3 (13 MB point clouds, 7-segment AQL packs) under dispatch / pipeline knobs, interleaved.
# Output: gpurun_out/c3_knobs_ab.jsonl (one bench line per run, tagged).
export TMPDIR=/tmp
out=gpurun_out/c3_knobs_ab.jsonl
mkdir -p gpurun_out
run() {
  tag=$1; shift
  line=$(env "$@" timeout -k 10 120 python bench.py --workload c3 --no-cpu-baseline --no-ladder --steps 1000) || exit $?
  echo "{\"tag\": \"$tag\", \"bench\": $line}" >> $out
}
for rep in 1 2; do
  run default DORA_NOTHING=1
  run inflight12 DORA_GPU_MAX_IN_FLIGHT=12
  run inflight6 DORA_GPU_MAX_IN_FLIGHT=6
  run queues2 DORA_GPU_AQL_QUEUES=2
  run queues8 DORA_GPU_AQL_QUEUES=8
  run chunk64k DORA_GPU_PACK_CHUNK=65536
  run chunk16k DORA_GPU_PACK_CHUNK=16384
  run hipstreams DORA_GPU_AQL_MAX_BYTES=0
done
