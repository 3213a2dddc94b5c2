#!/bin/bash
# The synchronous send's read-first packs (dora_aql_pack1r_u4) under rocprofv3: a kernel trace +
# stats of 200 synchronous 40.96 MB sends, then FETCH_SIZE and WRITE_SIZE in passes of their
# own.  usage: bash scripts/r06_sync_profile.sh <out dir under gpurun_out>
set -euo pipefail
out=${1:?out dir}
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p "$out"
B="python bench.py --no-ladder --no-cpu-baseline --no-c3 --sync-n 0"
export DORA_BENCH_SYNC_SENDS=1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/sync_trace" -o run -- \
  $B --steps 200 --warmup 20 > "$out/sync_trace_bench.json" 2> "$out/sync_trace_bench.err"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/sync_fetch" -o run -- \
  $B --steps 50 --warmup 5 > "$out/sync_fetch_bench.json" 2> "$out/sync_fetch.err"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/sync_write" -o run -- \
  $B --steps 50 --warmup 5 > "$out/sync_write_bench.json" 2> "$out/sync_write.err"
python scripts/pmc_traffic.py "$out/sync_fetch" "$out/sync_write" --kernel dora_aql_pack1r_u4 \
  --algorithmic 81920000 --min-kb 30000 > "$out/sync_pmc_traffic.json"
cat "$out/sync_pmc_traffic.json"
echo done
