#!/usr/bin/env python3
"""A/B of the batch-pack knobs on the native ladder (HBM-resident rotated sources), interleaved
rounds; one JSON line per (round, config, size) on stdout.

    python scripts/batch_ab.py --rounds 2 --sizes 1048576,4096000,16777216
"""
import argparse
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

CONFIGS = {
    "batch_off_if11": {"DORA_GPU_AQL_BATCH": "0"},
    "batch_d2_if11": {},
    "batch_off_if24": {"DORA_GPU_AQL_BATCH": "0", "DORA_GPU_MAX_IN_FLIGHT": "24"},
    "batch_d2_if24": {"DORA_GPU_MAX_IN_FLIGHT": "24"},
    "batch_d1_if24": {"DORA_GPU_MAX_IN_FLIGHT": "24", "DORA_GPU_AQL_DEPTH": "1"},
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--sizes", default="1048576,4096000,16777216")
    ap.add_argument("--n", type=int, default=2000)
    ap.add_argument("--configs", default=",".join(CONFIGS))
    ap.add_argument("--cfg", action="append", default=[],
                    help="name=K=V[,K=V...]: replaces the built-in configs")
    a = ap.parse_args()
    if a.cfg:
        CONFIGS.clear()
        for c in a.cfg:
            name, _, kv = c.partition("=")
            CONFIGS[name] = dict(x.split("=", 1) for x in kv.split(",") if x)
        a.configs = ",".join(CONFIGS)
    import bench
    for r in range(a.rounds):
        for name in a.configs.split(","):
            for size in [int(x) for x in a.sizes.split(",")]:
                env = dict(CONFIGS[name], DORA_BENCH_TP_SOURCES=str(bench.native_sources(size)))
                cmd = [sys.executable, os.path.join(HERE, "native_tp.py"), "--sizes", str(size),
                       "--n", str(a.n if size < (8 << 20) else a.n // 2)]
                for k, v in env.items():
                    cmd += ["--env", f"{k}={v}"]
                out = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
                for line in out.stdout.splitlines():
                    if line.startswith("{"):
                        d = json.loads(line)
                        print(json.dumps({"round": r, "cfg": name, "size": size,
                                          "us_per_msg": d.get("us_per_msg"),
                                          "hbm_frac_2S": round(2 * size / d["us_per_msg"] / 8e6, 4)
                                          if d.get("us_per_msg") else None,
                                          "sink_dropped": d.get("sink_dropped"),
                                          "batched": d.get("aql_batched_msgs"),
                                          "send_phase_us": d.get("send_phase_us")}), flush=True)
                if out.returncode:
                    print(json.dumps({"round": r, "cfg": name, "size": size,
                                      "error": out.stderr[-400:]}), flush=True)


if __name__ == "__main__":
    main()
