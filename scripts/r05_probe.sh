#!/bin/bash
# Round-5 probes on one GPU box (each GPU step under its own limit; the first failure ends it):
#  1. the driver-shape C3 block under a rocprofv3 kernel trace (bench.py --no-ladder: its C3
#     block's 200-cloud steady region and 20-cloud burst), reduced by scripts/c3_region.py;
#  2. the native and the Python node's throughput mode at 64 KB and 1 MiB with the host
#     sub-phase profile (DORA_GPU_TRACE=subphases): where a send's host time goes;
#  3. small messages' latency by stage (scripts/small_lat_probe.py);
#  4. C3 blocks under workgroup caps of the command processor's packs, interleaved.
# usage: bash scripts/r05_probe.sh <out dir under gpurun_out>
set -euo pipefail
out=${1:?out dir}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/c3_trace" -o run -- \
  python bench.py --no-ladder --no-cpu-baseline --steps 20 --warmup 5 \
  > "$out/c3_trace_bench.json" 2> "$out/c3_trace_bench.err"
python scripts/c3_region.py "$out/c3_trace" --line "$out/c3_trace_bench.json" > "$out/c3_region.json"
timeout -k 10 200 python -u scripts/native_tp.py --sizes 65536,1048576 --n 20000 \
  --env DORA_GPU_TRACE=subphases > "$out/native_tp.jsonl" 2> "$out/native_tp.err"
DORA_GPU_TRACE=subphases timeout -k 10 200 python -u scripts/py_tp.py --sizes 65536,1048576 --sources 64 \
  --n 20000 > "$out/py_tp.jsonl" 2> "$out/py_tp.err"
timeout -k 10 120 python -u scripts/small_lat_probe.py --n 500 > "$out/small_lat.jsonl" \
  2> "$out/small_lat.err"
timeout -k 10 200 python -u scripts/c3_burst_probe.py --reps 3 --grids 0,2048,1024,512 \
  > "$out/c3_grid.jsonl" 2> "$out/c3_grid.err"
echo done
