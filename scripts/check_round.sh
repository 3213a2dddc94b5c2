#!/bin/bash
# One GPU box: the GPU tests, smoke and the driver's bench command, each under its own limit;
# the first failure ends the script.   usage: bash scripts/check_round.sh <out dir under gpurun_out> [pytest args]
set -euo pipefail
out=${1:?out dir}
shift
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -s "$@" > "$out/gpu_tests.log" 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --detail "$out/bench_detail.json" > "$out/bench.json" 2> "$out/bench.err"
echo done
