#!/bin/bash
# Round-5 probes, seventh set: the AQL queues' packet rings in device memory
# (HSA_ALLOCATE_QUEUE_DEV_MEM=1, the ROCr runtime's placement switch) against the default
# system-memory rings, three interleaved full bench runs each (synchronous sends: 200).
# usage: bash scripts/r05_probe7.sh <out dir under gpurun_out>
set -euo pipefail
out=${1:?out dir}
mkdir -p "$out"
export TMPDIR=/tmp
for r in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --sync-n 200 \
    --lat-n 300 --detail "$out/d_sys_$r.json" > "$out/b_sys_$r.json" 2> "$out/b_sys_$r.err"
  HSA_ALLOCATE_QUEUE_DEV_MEM=1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 \
    --no-cpu-baseline --sync-n 200 --lat-n 300 --detail "$out/d_dev_$r.json" \
    > "$out/b_dev_$r.json" 2> "$out/b_dev_$r.err"
done
echo done
