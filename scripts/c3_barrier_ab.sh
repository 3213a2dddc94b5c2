#!/bin/bash
# C3 (13 MB point clouds) with the AQL barrier bit (in order per queue over three queues) vs the
# default free overlap on four queues, interleaved.  Output: gpurun_out/c3_barrier_ab.jsonl.
export TMPDIR=/tmp
out=gpurun_out/c3_barrier_ab.jsonl
mkdir -p gpurun_out
run() {
  tag=$1; shift
  line=$(env "$@" timeout -k 10 120 python bench.py --workload c3 --no-cpu-baseline --no-ladder --steps 1000) || exit $?
  echo "{\"tag\": \"$tag\", \"bench\": $line}" >> $out
}
for rep in 1 2 3; do
  run default DORA_NOTHING=1
  run barrier8m DORA_GPU_AQL_BARRIER_BYTES=8388608
  run barrier8m_if12 DORA_GPU_AQL_BARRIER_BYTES=8388608 DORA_GPU_MAX_IN_FLIGHT=12
  run barrier8m_c16k DORA_GPU_AQL_BARRIER_BYTES=8388608 DORA_GPU_PACK_CHUNK=16384
  run if16 DORA_GPU_MAX_IN_FLIGHT=16
done
