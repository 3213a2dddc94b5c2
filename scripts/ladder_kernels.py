#!/usr/bin/env python3
"""Per-message-size pack-kernel durations from a rocprofv3 kernel trace of `bench.py`.

bench.py packs, in order: `--warmup` headline messages, then every LADDER size `--lat-n` times
(latency mode), then the timed steps.  This script walks the pack_kernel dispatches of the trace
in that order and reports, per size, the mean/median duration and the HBM roofline fraction of
2*S algorithmic bytes per launch.

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ladder -o run -- python bench.py \
        --no-cpu-baseline --steps 20
    python scripts/ladder_kernels.py gpurun_out/ladder --warmup 20 --lat-n 50
"""
import argparse
import csv
import glob
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

HBM_GBPS = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--lat-n", type=int, default=50)
    a = ap.parse_args()
    from bench import LADDER
    f = glob.glob(os.path.join(a.trace_dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if "pack_kernel" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0 for r in rows]
    i = a.warmup
    for size in LADDER:
        d = durs[i:i + a.lat_n]
        i += a.lat_n
        if not d:
            break
        med = statistics.median(d)
        print(json.dumps({"size": size, "n": len(d), "mean_us": round(statistics.mean(d), 3),
                          "median_us": round(med, 3), "min_us": round(min(d), 3),
                          "GBps_2S": round(2 * size / (med * 1e-6) / 1e9, 1),
                          "frac_of_8TBps": round(2 * size / (med * 1e-6) / 1e9 / HBM_GBPS, 3)}))


if __name__ == "__main__":
    main()
