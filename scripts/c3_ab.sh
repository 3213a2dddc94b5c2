#!/bin/bash
# Verdict r03 item 2 (C3 burst): the bench's C3 block (200-send steady region + 20-send burst)
# under dispatch variants, interleaved.  usage: bash scripts/c3_ab.sh <out dir> [rounds]
set -euo pipefail
out=${1:?out dir}; rounds=${2:-2}
mkdir -p "$out"
export TMPDIR=/tmp
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python -u scripts/c3_burst_probe.py --reps 2 \
    > "$out/$name.jsonl" 2> "$out/$name.err"
  sed "s/^{/{\"run\": \"$name\", /" "$out/$name.jsonl" >> "$out/summary.jsonl"
}
# variants: `inkernel` (r03's in-kernel-signalled multi-segment packs), `barrier` (13 MB clouds
# run one at a time per queue over three queues, as the headline's >= 32 MiB packs), `depth2`
variants=${C3_AB_VARIANTS:-inkernel}
for r in $(seq 1 "$rounds"); do
  run "r${r}_default"
  for v in $variants; do
    case $v in
      inkernel) run "r${r}_inkernel" DORA_GPU_AQL_CP_MULTI=0 ;;
      barrier) run "r${r}_barrier" DORA_GPU_AQL_BARRIER_BYTES=12000000 ;;
      depth2) run "r${r}_depth2" DORA_GPU_AQL_CP_DEPTH=2 ;;
    esac
  done
done
echo done
