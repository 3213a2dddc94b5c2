#!/usr/bin/env python3
"""Interleaved A/B of environment knobs on bench.py's latency ladder (1000 messages per size,
1 ms apart; no throughput ladders); one JSON line per run with p50 / p99 per size.

    python scripts/lat_ab.py --rounds 2 --cfg base= --cfg numa=DORA_GPU_PIN=numa
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--cfg", action="append", default=[])
    a = ap.parse_args()
    cfgs = []
    for c in a.cfg or ["base="]:
        name, _, kv = c.partition("=")
        cfgs.append((name, dict(x.split("=", 1) for x in kv.split(",") if x)))
    for r in range(a.rounds):
        for name, env in cfgs:
            cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline", "--tp-n",
                   "0", "--no-c3", "--steps", "20", "--warmup", "5"]
            out = subprocess.run(cmd, capture_output=True, text=True, timeout=300,
                                 env=dict(os.environ, **env))
            line = next((x for x in out.stdout.splitlines() if x.startswith("{")), None)
            if not line:
                print(json.dumps({"round": r, "cfg": name, "error": out.stderr[-400:]}), flush=True)
                continue
            d = json.loads(line)
            lat = d.get("latency_us", {})
            print(json.dumps({"round": r, "cfg": name,
                              "p99_max": max(v["p99_us"] for v in lat.values()),
                              "p99_incl_pack_max": max(v["p99_incl_pack_us"] for v in lat.values()),
                              "p50": {k: v["p50_us"] for k, v in lat.items()},
                              "p99": {k: v["p99_us"] for k, v in lat.items()},
                              "cpu_share": d.get("cpu_share")}), flush=True)


if __name__ == "__main__":
    main()
