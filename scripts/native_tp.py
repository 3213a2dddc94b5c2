#!/usr/bin/env python3
"""Throughput mode of the native benchmark node (dora-gpu-bench-source -> dora-gpu-bench-sink,
both on GPU 0, zero-copy edge) per message size: separates the data plane's own per-send cost
from bench.py's Python node.

    python scripts/native_tp.py --sizes 4096,4096000,16777216,40960000 --n 1000
"""
import argparse
import json
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="4096,65536,1048576,4096000,16777216,40960000")
    ap.add_argument("--n", type=int, default=1000)
    ap.add_argument("--env", action="append", default=[], help="K=V for every node")
    a = ap.parse_args()
    import bench
    from dora_amd.dataflow import Dataflow
    env = dict(kv.split("=", 1) for kv in a.env)
    for size in [int(x) for x in a.sizes.split(",")]:
        tmp = tempfile.mkdtemp(prefix="dora-native-tp-")
        desc = bench.c4_descriptor(2, tmp, "kernel", tp_n=a.n, gpu=lambda g: 0, env=env)
        src = desc["nodes"][0]
        src["env"].update(env)  # c4_descriptor gives `env` to the sinks only
        src["env"].update({"DORA_BENCH_TP_SIZE": str(size), "DORA_BENCH_LAT_SIZES": str(size),
                           "DORA_BENCH_LAT_N": "5", "DORA_BENCH_LAT_GAP_US": "1000"})
        df = Dataflow(desc).start()
        try:
            codes = df.wait(120)
        finally:
            df.stop()
        r = bench._load(os.path.join(tmp, "source.json")) or {}
        sink = bench._load(os.path.join(tmp, "sink1.json")) or {}
        dlog = df.log("_daemon")
        dstat = {}
        for line in dlog.splitlines():
            if '"done"' in line:
                try:
                    dstat = json.loads(line)
                except ValueError:
                    pass
        sub = {}
        for who in ("source", "sink1", "_daemon"):
            for line in (df.log(who) or "").splitlines():
                if line.startswith('{"subphases"'):
                    try:
                        sub[who] = json.loads(line)["subphases"]
                    except ValueError:
                        pass
        print(json.dumps({"size": size, "n": a.n, "GBps": r.get("tp_delivered_GBps"),
                          "us_per_msg": round(size / (r["tp_delivered_GBps"] * 1e3), 3)
                          if r.get("tp_delivered_GBps") else None,
                          "send_phase_us": r.get("send_phase_us"), "ok": r.get("ok"),
                          "aql_batched_msgs": r.get("aql_batched_msgs"),
                          "busy_us_per_msg": {
                              "source": r.get("tp_busy_us_per_msg"),
                              "sink": sink.get("busy_us_per_input"),
                              "sink_fill_wait": sink.get("fill_wait_us_per_input"),
                              "sink_next_event": sink.get("next_event_us"),
                              "sink_free": sink.get("free_us"),
                              "daemon_per_routed": dstat.get("busy_us_per_routed")},
                          "sink_dropped": sink.get("dropped_inputs"),
                          "subphases_ns": sub or None,
                          "exit_codes": codes, "env": env}), flush=True)


if __name__ == "__main__":
    main()
