#!/usr/bin/env python3
"""Pack-kernel timing of bench.py's timed region from a rocprofv3 kernel trace — the
independent check of bench.py's `roofline` (device span of the region / packs).

bench.py --no-ladder packs, in order: a 4 KB cold-start message, `--warmup` messages, 24 refill
messages, then the `--steps` timed ones (pass --warmup W+24).  The timed packs overlap, so besides
each kernel's own mean duration this reports the region's device span (first start -> last end)
per pack and the union of the kernels' intervals per pack.

    rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
        python bench.py --no-ladder --no-cpu-baseline
    python scripts/rocprof_region.py gpurun_out/prof --warmup 20 --steps 200 --size 40960000
"""
import argparse
import csv
import glob
import json
import os
import statistics

HBM_GBPS = 8000.0


def union_ns(iv):
    total, end = 0, None
    for a, b in sorted(iv):
        if end is None or a > end:
            total += b - a
            end = b
        elif b > end:
            total += b - end
            end = b
    return total


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--min-grid", type=int, default=1024 * 256,
                    help="work-items of a headline pack launch (1024 workgroups x 256)")
    ap.add_argument("--size", type=int, default=40960000)
    a = ap.parse_args()
    f = glob.glob(os.path.join(a.trace_dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    # the headline packs: pack kernels (HIP `pack_kernel` or AQL `dora_aql_pack*`) of the
    # headline's grid (the cold-start / small packs of the same kernels have smaller grids)
    rows = [r for r in csv.DictReader(open(f))
            if "pack" in r["Kernel_Name"] and int(r["Grid_Size_X"]) >= a.min_grid]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    region = iv[a.warmup:a.warmup + a.steps]
    own = [(e - s) / 1000.0 for s, e in region]
    span_us = (max(e for _, e in region) - region[0][0]) / 1000.0
    busy_us = union_ns(region) / 1000.0
    per = span_us / len(region)
    out = {"trace": os.path.relpath(f, a.trace_dir), "pack_launches_in_trace": len(iv),
           "region_packs": len(region), "msg_bytes": a.size,
           "own_duration_us": {"mean": round(statistics.mean(own), 3),
                               "median": round(statistics.median(own), 3),
                               "min": round(min(own), 3), "max": round(max(own), 3)},
           "span_us": round(span_us, 1), "device_us_per_launch": round(per, 3),
           "busy_us_per_launch": round(busy_us / len(region), 3),
           "achieved_GBps": round(2.0 * a.size / (per * 1e-6) / 1e9, 1),
           "frac_of_8TBps": round(2.0 * a.size / (per * 1e-6) / 1e9 / HBM_GBPS, 4)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
