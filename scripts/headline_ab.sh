#!/bin/bash
# The driver's 20-step headline (+ the 20-send synchronous leg) under dispatch variants,
# interleaved.  usage: bash scripts/headline_ab.sh <out dir> [rounds]
set -euo pipefail
out=${1:?out dir}; rounds=${2:-3}
mkdir -p "$out"
export TMPDIR=/tmp
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-ladder --no-c3 \
    --no-cpu-baseline --detail "$out/$name.detail.json" > "$out/$name.json" 2> "$out/$name.err"
  python - "$out/$name.detail.json" "$name" >> "$out/summary.jsonl" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); s = d.get("sync_send_headline") or {}
print(json.dumps({"run": sys.argv[2], "value": d["value"], "frac": d["roofline"]["frac"],
                  "first_receipt_us": d["timed_region"].get("first_msg_receipt_us"),
                  "sync_us": s.get("us_per_msg"), "sync_own": s.get("pack_own_us"),
                  "sync_gap": s.get("gap_us_median"),
                  "sync_calls": [round(b - a, 1) for a, b in zip(s.get("send_calls_us", []),
                                                                 s.get("send_calls_us", [])[1:])]}))
PY
}
for r in $(seq 1 "$rounds"); do
  run "r${r}_default"
  run "r${r}_read_off" DORA_GPU_AQL_READ_SIGNAL=0
  run "r${r}_lone_off" DORA_GPU_AQL_CP_LONE=0
done
echo done
