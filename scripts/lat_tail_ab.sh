#!/bin/bash
# Latency-tail A/B: the bench's latency ladder (1000 spaced messages per size) under CPU
# placement / spin-budget variants, interleaved, with the busy share of every CPU of the box
# sampled over each run (/proc/stat) so that a tail caused by neighbours on our cores shows.
# Writes gpurun_out/lat_tail_ab.jsonl.  Usage: [VARIANTS='default;K=V K2=V2'] scripts/lat_tail_ab.sh [rounds]
rounds=${1:-1}
out=gpurun_out/lat_tail_ab.jsonl
mkdir -p gpurun_out
: > "$out"
bash scripts/box_diag.sh lat_tail
cat /sys/class/drm/card*/device/numa_node > gpurun_out/gpu_numa.txt 2>/dev/null || true
for r in $(seq 1 "$rounds"); do
  IFS=';' read -ra variants <<< "${VARIANTS:-default;DORA_GPU_PIN_L3=0;DORA_GPU_SPIN_US=3000;DORA_GPU_PIN_L3=0 DORA_GPU_SPIN_US=3000}"
  for v in "${variants[@]}"; do
    python3 scripts/cpu_busy.py snap > gpurun_out/_stat0.json
    if [ "$v" = default ]; then envs=(); else read -ra envs <<< "$v"; fi
    timeout -k 10 180 env "${envs[@]}" python3 bench.py --steps 100 --warmup 10 --tp-n 0 \
      --no-cpu-baseline > gpurun_out/_lat.json 2> gpurun_out/_lat.err || { echo "bench failed: $v"; exit 1; }
    python3 scripts/cpu_busy.py snap > gpurun_out/_stat1.json
    python3 - "$v" "$r" >> "$out" <<'EOF'
import json, sys
sys.path.insert(0, "scripts")
from cpu_busy import busy
line = json.loads(open("gpurun_out/_lat.json").read().strip().splitlines()[-1])
b = busy(json.load(open("gpurun_out/_stat0.json")), json.load(open("gpurun_out/_stat1.json")))
lat = {s: {"p50": v["p50_us"], "p99": v["p99_us"], "max_incl": v.get("p99_incl_pack_us")}
       for s, v in line["latency_us"].items()}
print(json.dumps({"variant": sys.argv[1], "round": int(sys.argv[2]), "value": line["value"],
                  "p99_max_us": max(v["p99"] for v in lat.values()),
                  "p99_median_us": sorted(v["p99"] for v in lat.values())[len(lat) // 2],
                  "latency": lat, "cpu_busy": b}))
EOF
    tail -1 "$out" | cut -c1-200
  done
done
