#!/bin/bash
# Round-5 rehearsal of the driver's multi-GPU command with two ranks on the one GPU
# (DORA_BENCH_GPUS=1: every rank and cross-GPU stage on GPU 0).
# usage: bash scripts/r05_n2.sh <out dir under gpurun_out>
set -euo pipefail
out=${1:?out dir}
mkdir -p "$out"
export TMPDIR=/tmp
DORA_BENCH_GPUS=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 \
  --detail "$out/bench_n2_detail.json" > "$out/bench_n2.json" 2> "$out/bench_n2.err"
echo done
