#!/bin/bash
# Python-node throughput ladder A/B (bench.py's throughput_per_size, 1-16 MB) against the native
# ladder of the same run: queue count and in-flight cap for the bench process.
# Output: gpurun_out/py_ladder_ab.jsonl.  Usage: [VARIANTS='x;K=V'] scripts/py_ladder_ab.sh [rounds]
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/py_ladder_ab.jsonl
: > "$out"
IFS=';' read -ra variants <<< "${VARIANTS:-x;DORA_GPU_AQL_QUEUES=2;DORA_GPU_MAX_IN_FLIGHT=16}"
for r in $(seq 1 "${1:-2}"); do
  for v in "${variants[@]}"; do
    if [ "$v" = x ]; then envs=(); else read -ra envs <<< "$v"; fi
    timeout -k 10 180 env "${envs[@]}" python3 bench.py --steps 100 --warmup 10 --lat-n 0 \
      --no-cpu-baseline > gpurun_out/_pl.json 2> gpurun_out/_pl.err || { echo "bench failed: $v"; exit 1; }
    python3 - "$v" >> "$out" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/_pl.json").read().strip().splitlines()[-1])
sel = ("1048576", "4096000", "4194304", "16777216", "40960000")
print(json.dumps({"variant": sys.argv[1], "value": d["value"],
                  "py_us": {s: d["throughput_per_size"][s]["us_per_msg"] for s in sel},
                  "native_us": {s: v["us_per_msg"] for s, v in
                                (d.get("throughput_per_size_native") or {}).items()}}))
PY
    tail -1 "$out"
  done
done
