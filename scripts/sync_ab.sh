#!/bin/bash
# Verdict r03 item 1 (lone packs): the synchronous 40.96 MB send and the pipelined headline under
# CP-signal / grid variants, interleaved.  usage: bash scripts/sync_ab.sh <out dir> [rounds]
set -euo pipefail
out=${1:?out dir}; rounds=${2:-2}
mkdir -p "$out"
export TMPDIR=/tmp
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python -u bench.py --steps 200 --warmup 20 --no-ladder --no-c3 \
    --no-cpu-baseline --sync-n 200 --detail "$out/$name.detail.json" > "$out/$name.json" 2> "$out/$name.err"
  python - "$out/$name.detail.json" "$name" >> "$out/summary.jsonl" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); s = d.get("sync_send_headline") or {}
print(json.dumps({"run": sys.argv[2], "headline_frac": d["roofline"]["frac"],
                  "headline_us": d["roofline"]["device_us_per_launch"],
                  "sync": {k: s.get(k) for k in ("us_per_msg", "us_per_send_call", "pack_own_us",
                          "pack_own_us_median", "pack_own_frac", "gap_us_median", "cp_signalled",
                          "send_phase_us")}}))
PY
}
# SYNC_AB_VARIANTS: names from the list below (default: the r04 grid sweep)
variants=${SYNC_AB_VARIANTS:-"g2048_bal g4096_bal g2048 g6144_bal"}
for r in $(seq 1 "$rounds"); do
  run "r${r}_default"
  for v in $variants; do
    case $v in
      g2048_bal) run "r${r}_$v" DORA_GPU_CP_GRID=2048 DORA_GPU_BALANCED_CHUNKS=1 ;;
      g4096_bal) run "r${r}_$v" DORA_GPU_CP_GRID=4096 DORA_GPU_BALANCED_CHUNKS=1 ;;
      g6144_bal) run "r${r}_$v" DORA_GPU_CP_GRID=6144 DORA_GPU_BALANCED_CHUNKS=1 ;;
      g2048) run "r${r}_$v" DORA_GPU_CP_GRID=2048 ;;
      g4096) run "r${r}_$v" DORA_GPU_CP_GRID=4096 ;;
      fenced) run "r${r}_$v" DORA_GPU_AQL_LONE_COHERENT=0 ;;
      hostargs) run "r${r}_$v" DORA_GPU_AQL_LONE_DEV_ARGS=0 ;;
      grid*) run "r${r}_$v" DORA_GPU_CP_GRID=${v#grid} ;;
    esac
  done
done
echo done
