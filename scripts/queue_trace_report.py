#!/usr/bin/env python3
"""Per-process, per-queue view of a rocprofv3 kernel trace (`-o %pid%_run`): dispatches, own
duration, start-to-start gap, and how busy the device was with them — the check of the r01
"slow mode" hypothesis (time-sliced hardware queues show as long gaps between dispatches that
were already queued, on every queue at once).

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/nprof -o %pid%_run -- \
        python scripts/native_tp.py --sizes 4194304,40960000 --n 2000
    python scripts/queue_trace_report.py gpurun_out/nprof
"""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict


def union(iv):
    total, end = 0, None
    for a, b in sorted(iv):
        if end is None or a > end:
            total += b - a
            end = b
        elif b > end:
            total += b - end
            end = b
    return total


def main(d):
    out = {}
    for f in sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)):
        rows = list(csv.DictReader(open(f)))
        if not rows:
            continue
        by_kernel_grid = defaultdict(list)
        for r in rows:
            by_kernel_grid[(r["Kernel_Name"], int(r["Grid_Size_X"]))].append(r)
        proc = {}
        for (name, grid), rs in sorted(by_kernel_grid.items(), key=lambda kv: -len(kv[1])):
            if len(rs) < 20:
                continue
            iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rs)
            own = [(b - a) / 1e3 for a, b in iv]
            gaps = [(iv[i + 1][0] - iv[i][0]) / 1e3 for i in range(len(iv) - 1)]
            span = (max(b for _, b in iv) - iv[0][0]) / 1e3
            queues = defaultdict(int)
            for r in rs:
                queues[r["Queue_Id"]] += 1
            proc[f"{name} grid {grid}"] = {
                "dispatches": len(rs), "queues": dict(queues),
                "own_us_p50": round(statistics.median(own), 3),
                "start_gap_us_p50": round(statistics.median(gaps), 3),
                "start_gap_us_p99": round(sorted(gaps)[int(0.99 * (len(gaps) - 1))], 3),
                "max_gap_us": round(max(gaps), 1),
                "span_us": round(span, 1),
                "busy_frac": round(union(iv) / 1e3 / span, 4) if span else None,
                "device_us_per_dispatch": round(span / len(rs), 3)}
        out[os.path.basename(f)] = proc
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
