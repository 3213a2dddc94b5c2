#!/bin/bash
# r03 command-processor fill signal: parity tests (single- and multi-segment), C3 and native
# ladder A/Bs.   usage: bash scripts/cp_ab_run.sh <out dir>
set -o pipefail
out=${1:-gpurun_out/cp}
mkdir -p "$out"
export TMPDIR=/tmp
T="python -u -m pytest tests/test_gpu_dataflow.py -x -v -s --timeout 120 --timeout-method thread"
timeout -k 10 300 $T -k "cp_signalled or bench_sink or c3" > "$out/tests.log" 2>&1 || { echo TESTS FAILED; exit 1; }
DORA_GPU_AQL_CP_MULTI=1 timeout -k 10 300 $T -k "cp_signalled or c3 or bench_sink" > "$out/tests_multi.log" 2>&1 || { echo MULTI TESTS FAILED; exit 1; }
timeout -k 10 400 python -u scripts/bench_ab.py --rounds 3 --steps 200 --workloads c3 --cfg base= --cfg cp_multi=DORA_GPU_AQL_CP_MULTI=1 > "$out/c3_ab.jsonl" 2> "$out/c3_ab.err" || { echo C3 AB FAILED; exit 1; }
timeout -k 10 400 python -u scripts/bench_ab.py --rounds 3 --steps 20 --workloads c3 --cfg base= --cfg cp_multi=DORA_GPU_AQL_CP_MULTI=1 > "$out/c3_ab20.jsonl" 2> "$out/c3_ab20.err" || { echo C3 AB FAILED; exit 1; }
timeout -k 10 600 python -u scripts/batch_ab.py --rounds 2 --sizes 1048576,4096000 --n 2000 --cfg base= --cfg cp1m=DORA_GPU_AQL_CP_SIGNAL=1048576:33554432 --cfg if16=DORA_GPU_MAX_IN_FLIGHT=16 > "$out/ab.jsonl" 2> "$out/ab.err" || { echo AB FAILED; exit 1; }
echo ok
