#!/bin/bash
# Device samples for receivers without a GPU packed into shared memory by the producer: the
# host-edge GPU tests, then the driver's bench command (its d2h_* series).
out=gpurun_out/${1:-r6hp}
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_host_edges.py > $out/test.log 2>&1 || { tail -40 $out/test.log; exit 1; }
grep -E "PASS|FAIL|host-only receiver" $out/test.log | tail -12
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --detail $out/detail.json \
  > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
python - <<PY
import json
d = json.load(open("$out/detail.json"))
print({k: (v.get("p50_us"), v.get("p99_us"), v.get("p50_incl_pack_us")) for k, v in d["latency_us"].items() if k.startswith("d2h")})
print(d.get("host_paths"), d.get("host_path_rates"))
PY
