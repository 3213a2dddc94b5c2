#!/usr/bin/env python3
"""Per-send host stages of the last C3 burst in a DORA_GPU_TRACE directory (the sender's own
trace file): alloc (allocate_data_sample incl. the in-flight wait), launch (plan + AQL dispatch),
launched -> sent (descriptor to the daemon), and the gap to the next send's start, for the last
`--n` sends of the run (the 20-cloud burst of scripts/c3_burst_probe.py).

    DORA_GPU_TRACE=gpurun_out/c3t python scripts/c3_burst_probe.py --reps 1
    python scripts/c3_send_trace.py gpurun_out/c3t --n 20
"""
import argparse
import csv
import glob
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--n", type=int, default=20)
    ap.add_argument("--min-gap-us", type=float, default=0.0)
    a = ap.parse_args()
    ev = {}
    for f in glob.glob(os.path.join(a.trace_dir, "*.trace.csv")):
        for r in csv.DictReader(open(f)):
            ev.setdefault(r["token"], {}).setdefault(int(r["point"]), int(r["t_ns"]))
    sends = sorted((v for v in ev.values() if 1 in v and 3 in v and 5 in v), key=lambda v: v[1])
    last = sends[-a.n:]
    t0 = last[0][1]
    rows = []
    for i, v in enumerate(last):
        nxt = last[i + 1][1] if i + 1 < len(last) else None
        rows.append({"k": i, "t_us": round((v[1] - t0) / 1e3, 2),
                     "alloc_us": round((v[2] - v[1]) / 1e3, 2),
                     "launch_us": round((v[3] - v[2]) / 1e3, 2),
                     "send_us": round((v[5] - v[3]) / 1e3, 2),
                     "to_next_us": round((nxt - v[5]) / 1e3, 2) if nxt else None})
    for r in rows:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
