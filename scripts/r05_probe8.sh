#!/bin/bash
# Round-5 probes, eighth set: the packet rings in device memory (HSA_ALLOCATE_QUEUE_DEV_MEM=1)
# with fenced packet publication — the GPU tests and smoke under it, then three interleaved
# full bench runs against the default system-memory rings (synchronous sends: 200).
# usage: bash scripts/r05_probe8.sh <out dir under gpurun_out>
set -euo pipefail
out=${1:?out dir}
mkdir -p "$out"
export TMPDIR=/tmp
HSA_ALLOCATE_QUEUE_DEV_MEM=1 timeout -k 10 500 python -u -m pytest tests -m gpu -x -q \
  --timeout 120 --timeout-method thread > "$out/gpu_tests_dev.log" 2>&1
HSA_ALLOCATE_QUEUE_DEV_MEM=1 timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" \
  > "$out/smoke_dev.log" 2>&1
for r in 1 2 3; do
  HSA_ALLOCATE_QUEUE_DEV_MEM=1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 \
    --no-cpu-baseline --sync-n 200 --lat-n 300 --detail "$out/d_dev_$r.json" \
    > "$out/b_dev_$r.json" 2> "$out/b_dev_$r.err"
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --sync-n 200 \
    --lat-n 300 --detail "$out/d_sys_$r.json" > "$out/b_sys_$r.json" 2> "$out/b_sys_$r.err"
done
echo done
