#!/bin/bash
# Round-5 probes, ninth set: the packet-ring placement test under both placements, then three
# full bench runs of the current build (fences only for rings in device memory).
# usage: bash scripts/r05_probe9.sh <out dir under gpurun_out>
set -euo pipefail
out=${1:?out dir}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 100 python -u -m pytest tests/test_gpu_fence.py -x -v --timeout 60 \
  --timeout-method thread -s -k packet_rings > "$out/ring_sys.log" 2>&1
HSA_ALLOCATE_QUEUE_DEV_MEM=1 timeout -k 10 100 python -u -m pytest tests/test_gpu_fence.py -x -v \
  --timeout 60 --timeout-method thread -s -k packet_rings > "$out/ring_dev.log" 2>&1
for r in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --sync-n 200 \
    --lat-n 300 --detail "$out/d_sys_$r.json" > "$out/b_sys_$r.json" 2> "$out/b_sys_$r.err"
done
echo done
