#!/usr/bin/env python3
"""Per-queue gaps of dora_aql_pack1_u4 dispatches in rocprofv3 kernel traces (scripts/
cp_queue_overlap.sh): next start - previous end on the same queue, in us (negative = overlap)."""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict


def report(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    q = defaultdict(list)
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].startswith("dora_aql_pack1_u4"):
            q[r["Queue_Id"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    gaps, own, n = [], [], 0
    for iv in q.values():
        iv.sort()
        n += len(iv)
        own += [(b - a) / 1e3 for a, b in iv]
        gaps += [(iv[i + 1][0] - iv[i][1]) / 1e3 for i in range(len(iv) - 1)]
    gaps.sort()
    return {"queues": len(q), "packs": n, "own_us_median": round(statistics.median(own), 2),
            "gap_us_p10": round(gaps[len(gaps) // 10], 2), "gap_us_median": round(statistics.median(gaps), 2),
            "gap_us_p90": round(gaps[9 * len(gaps) // 10], 2),
            "overlapping_share": round(sum(g < 0 for g in gaps) / len(gaps), 3)}


if __name__ == "__main__":
    out = {}
    for mode in ("cp", "kernel"):
        out[mode] = report(os.path.join(sys.argv[1], mode))
        tp = os.path.join(sys.argv[1], f"{mode}_tp.json")
        if os.path.exists(tp):
            out[mode]["us_per_msg_under_rocprof"] = json.loads(open(tp).readline())["us_per_delivered_msg"]
    print(json.dumps(out, indent=1))
