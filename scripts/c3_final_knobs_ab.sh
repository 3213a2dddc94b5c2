#!/bin/bash
# C3 on the final pack (line-aligned chunks, no release fence): in-flight cap, AQL queue count,
# chunk bytes and signalling grid, interleaved.  Output: gpurun_out/c3_final_knobs_ab.jsonl.
export TMPDIR=/tmp
out=gpurun_out/c3_final_knobs_ab.jsonl
mkdir -p gpurun_out
run() {
  tag=$1; shift
  line=$(timeout -k 10 120 env "$@" python bench.py --workload c3 --no-cpu-baseline --no-ladder --steps 1000) || exit $?
  echo "{\"tag\": \"$tag\", \"bench\": $line}" >> $out
}
for rep in 1 2; do
  run default DORA_X=1
  run if12 DORA_GPU_MAX_IN_FLIGHT=12
  run if16 DORA_GPU_MAX_IN_FLIGHT=16
  run q3 DORA_GPU_AQL_QUEUES=3
  run q6 DORA_GPU_AQL_QUEUES=6
  run c16k DORA_GPU_PACK_CHUNK=16384
  run g512 DORA_GPU_SIGNAL_GRID=512
  run u4 DORA_GPU_PACK_VARIANT=u4nt
done
