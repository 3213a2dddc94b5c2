#!/usr/bin/env python3
"""Interleaved A/B of environment knobs on bench.py's headline (C2, 40.96 MB) and C3 workloads
(no ladders, no CPU baseline); one JSON line per run.

    python scripts/bench_ab.py --rounds 2 --steps 1000 --cfg base= --cfg cap10=DORA_GPU_MAX_IN_FLIGHT=10:8
"""
import argparse
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--workloads", default="c2,c3")
    ap.add_argument("--cfg", action="append", default=[],
                    help="name=K=V[,K=V...] (name= for the defaults)")
    a = ap.parse_args()
    cfgs = []
    for c in a.cfg or ["base="]:
        name, _, kv = c.partition("=")
        env = dict(x.split("=", 1) for x in kv.split(",") if x)
        cfgs.append((name, env))
    for r in range(a.rounds):
        for wl in a.workloads.split(","):
            for name, env in cfgs:
                e = dict(os.environ, **env)
                cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline",
                       "--no-ladder", "--no-c3", "--steps", str(a.steps), "--warmup", "20",
                       "--workload", wl]
                out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=e)
                line = next((x for x in out.stdout.splitlines() if x.startswith("{")), None)
                if not line:
                    print(json.dumps({"round": r, "wl": wl, "cfg": name, "error": out.stderr[-500:]}),
                          flush=True)
                    continue
                d = json.loads(line)
                rf = d.get("roofline", {})
                print(json.dumps({"round": r, "wl": wl, "cfg": name, "value": d.get("value"),
                                  "frac": rf.get("frac"), "dev_us": rf.get("device_us_per_launch"),
                                  "kernels": rf.get("region_kernels"),
                                  "mismatches": d.get("parity", {}).get("mismatches")}), flush=True)


if __name__ == "__main__":
    main()
