#!/bin/bash
# The round's committed evidence, on one GPU box: rocprofv3 kernel trace + stats of the C2
# headline and of C3, two PMC passes each (FETCH_SIZE / WRITE_SIZE cannot share one), then the
# driver's own bench command.  Every GPU step has its own time limit; the first failure ends
# the script.   usage: bash scripts/profile_round.sh <out dir under gpurun_out>
set -euo pipefail
out=${1:?out dir}
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p "$out"
B="python bench.py --no-ladder --no-cpu-baseline --no-c3"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/c2_trace" -o run -- \
  $B --steps 200 --warmup 20 > "$out/c2_trace_bench.json" 2> "$out/c2_trace_bench.err"
# the default (synchronous) send: every timed step waits for its own pack (a lone pack)
DORA_BENCH_SYNC_SENDS=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv \
  -d "$out/c2_sync_trace" -o run -- $B --steps 200 --warmup 20 --sync-n 0 \
  > "$out/c2_sync_trace_bench.json" 2> "$out/c2_sync_trace_bench.err"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/c2_fetch" -o run -- \
  $B --steps 50 --warmup 5 > "$out/c2_fetch_bench.json" 2> "$out/c2_fetch.err"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/c2_write" -o run -- \
  $B --steps 50 --warmup 5 > "$out/c2_write_bench.json" 2> "$out/c2_write.err"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/c3_trace" -o run -- \
  $B --workload c3 --steps 200 --warmup 20 > "$out/c3_trace_bench.json" 2> "$out/c3_trace_bench.err"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/c3_fetch" -o run -- \
  $B --workload c3 --steps 50 --warmup 5 > "$out/c3_fetch_bench.json" 2> "$out/c3_fetch.err"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/c3_write" -o run -- \
  $B --workload c3 --steps 50 --warmup 5 > "$out/c3_write_bench.json" 2> "$out/c3_write.err"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > "$out/bench.json" 2> "$out/bench.err"
echo done
