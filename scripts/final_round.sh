#!/bin/bash
# Round-end verification on one GPU box: GPU tests, smoke, the driver's bench command, an N=2
# rehearsal of the multi-GPU flow on the one GPU (DORA_BENCH_GPUS=1), then the rocprof kernel
# trace / PMC passes of scripts/profile_round.sh.  Every GPU step has its own time limit; the
# first failure ends the script.   usage: bash scripts/final_round.sh <out dir under gpurun_out>
set -euo pipefail
out=${1:?out dir}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -s > "$out/gpu_tests.log" 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > "$out/bench.json" 2> "$out/bench.err"
DORA_BENCH_GPUS=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 \
  > "$out/bench_n2.json" 2> "$out/bench_n2.err"
bash scripts/profile_round.sh "$out/prof"
echo done
