#!/bin/bash
# Full bench runs with and without the dataflow's NUMA / L3 CPU placement (DORA_GPU_PIN),
# interleaved: the Python 40.96 MB ladder and the C3 burst are token-return bound, so their
# spread follows the host's scheduling.  usage: bash scripts/pin_ab.sh <out dir> [rounds]
set -euo pipefail
out=${1:?out dir}; rounds=${2:-3}
mkdir -p "$out"
export TMPDIR=/tmp
run() {
  local name=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline \
    --detail "$out/$name.detail.json" > "$out/$name.json" 2> "$out/$name.err"
  python - "$out/$name.detail.json" "$name" >> "$out/summary.jsonl" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); t = d["throughput_per_size"]
print(json.dumps({"run": sys.argv[2], "value": d["value"], "frac": d["roofline"]["frac"],
                  "c3": d["c3"]["roofline"]["frac"], "c3_steady": (d["c3"].get("steady") or {}).get("frac"),
                  "py40": t["40960000"]["us_per_msg"], "py4": t["4194304"]["us_per_msg"],
                  "sync": d["sync_send_headline"]["us_per_msg"],
                  "lat4k": d["latency_us"]["4096"]["p50_us"], "drops": d["sink_dropped_by_phase"],
                  "load": d["cpu_share"].get("loadavg_1m"),
                  "affinity_after_init": d.get("affinity_after_init")}))
PY
}
for r in $(seq 1 "$rounds"); do
  run "r${r}_pin"
  run "r${r}_pin_fixed" DORA_GPU_PIN_L3=fixed
  run "r${r}_nopin" DORA_GPU_PIN=0
done
echo done
