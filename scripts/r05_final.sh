#!/bin/bash
# The round's committed evidence on one GPU box, each GPU step under its own limit (the first
# failure ends the script):
#  1. the GPU tests, smoke and the driver's bench command (scripts/check_round.sh's steps);
#  2. C2 headline: rocprofv3 kernel trace of 200 timed steps (scripts/rocprof_region.py) and the
#     two PMC passes (scripts/pmc_traffic.py);
#  3. C3: the driver-shape block under a kernel trace, reduced by scripts/c3_region.py against
#     the same run's line and the packs' own stamps; the two PMC passes.
# usage: bash scripts/r05_final.sh <out dir under gpurun_out>
set -euo pipefail
out=${1:?out dir}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -s \
  > "$out/gpu_tests.log" 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --detail "$out/bench_detail.json" \
  > "$out/bench.json" 2> "$out/bench.err"
B="python bench.py --no-ladder --no-cpu-baseline"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/c2_trace" -o run -- \
  $B --no-c3 --steps 200 --warmup 20 --detail "$out/c2_trace_detail.json" \
  > "$out/c2_trace_bench.json" 2> "$out/c2_trace_bench.err"
python scripts/rocprof_region.py "$out/c2_trace" --warmup 44 --steps 200 > "$out/c2_region.json"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/c2_fetch" -o run -- \
  $B --no-c3 --steps 50 --warmup 5 --detail "" > "$out/c2_fetch_bench.json" 2> "$out/c2_fetch.err"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/c2_write" -o run -- \
  $B --no-c3 --steps 50 --warmup 5 --detail "" > "$out/c2_write_bench.json" 2> "$out/c2_write.err"
python scripts/pmc_traffic.py "$out/c2_fetch" "$out/c2_write" --kernel dora_aql_pack1_u4 \
  --algorithmic 81920000 --min-kb 30000 > "$out/c2_pmc_traffic.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/c3_trace" -o run -- \
  $B --steps 20 --warmup 5 --detail "$out/c3_trace_detail.json" \
  > "$out/c3_trace_bench.json" 2> "$out/c3_trace_bench.err"
python scripts/c3_region.py "$out/c3_trace" --line "$out/c3_trace_bench.json" \
  --detail "$out/c3_trace_detail.json" > "$out/c3_region.json"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/c3_fetch" -o run -- \
  $B --workload c3 --no-c3 --steps 50 --warmup 5 --detail "" > "$out/c3_fetch_bench.json" \
  2> "$out/c3_fetch.err"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/c3_write" -o run -- \
  $B --workload c3 --no-c3 --steps 50 --warmup 5 --detail "" > "$out/c3_write_bench.json" \
  2> "$out/c3_write.err"
python scripts/pmc_traffic.py "$out/c3_fetch" "$out/c3_write" --kernel dora_aql_pack_u4 \
  --algorithmic 26000136 --min-kb 10000 > "$out/c3_pmc_traffic.json"
echo done
