#!/bin/bash
# Full driver-command bench runs (`--steps 20 --warmup 5`, no CPU baseline) under environment
# variants, interleaved; one summary line per run in <out dir>/summary.jsonl.
# usage: bash scripts/full_ab.sh <out dir> <rounds> name[:K=V[,K=V...]] ...
#   e.g. bash scripts/full_ab.sh gpurun_out/ab 3 default barrier8m:DORA_GPU_AQL_BARRIER_BYTES=8388608
set -euo pipefail
out=${1:?out dir}; rounds=${2:?rounds}; shift 2
mkdir -p "$out"
export TMPDIR=/tmp
run() {  # name, K=V list
  local name=$1 kv=$2
  local -a envs=()
  if [ -n "$kv" ]; then IFS=, read -r -a envs <<< "$kv"; fi
  env "${envs[@]}" timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline \
    --detail "$out/$name.detail.json" > "$out/$name.json" 2> "$out/$name.err"
  python - "$out/$name.detail.json" "$name" >> "$out/summary.jsonl" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
t, nat = d["throughput_per_size"], d.get("throughput_per_size_native") or {}
us = lambda m, z: (m.get(z) or {}).get("us_per_msg")
print(json.dumps({"run": sys.argv[2], "value": d["value"], "frac": d["roofline"]["frac"],
                  "c3": d["c3"]["roofline"]["frac"], "c3_steady": (d["c3"].get("steady") or {}).get("frac"),
                  "sync": d["sync_send_headline"]["us_per_msg"],
                  "py": {z: us(t, z) for z in ("4096", "1048576", "4194304", "16777216", "40960000")},
                  "native": {z: us(nat, z) for z in ("4096", "1048576", "4096000", "16777216", "40960000")},
                  "lat_p50": {z: d["latency_us"][z]["p50_us"] for z in ("4096", "4194304", "40960000")},
                  "py_device": {z: (t.get(z) or {}).get("device") for z in ("16777216", "40960000")},
                  "drops": {k: v for k, v in d["sink_dropped_by_phase"].items() if v},
                  "load": d["cpu_share"].get("loadavg_1m")}))
PY
}
for r in $(seq 1 "$rounds"); do
  for v in "$@"; do
    run "r${r}_${v%%:*}" "$( [[ $v == *:* ]] && echo "${v#*:}" || true )"
  done
done
echo done
