#!/usr/bin/env python3
"""HBM traffic per launch of one kernel from two rocprofv3 counter passes (FETCH_SIZE and
WRITE_SIZE cannot share a pass on gfx950), corrected as MI355X_MICROARCH.md prescribes:
FETCH_SIZE counts half the bytes of 16-B-per-lane streaming reads on gfx950 (x2), WRITE_SIZE is
exact for 16-B streaming stores; both are in KiB.

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python bench.py ...
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python bench.py ...
    python scripts/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write --kernel pack_kernel \
        --algorithmic 81920000 --min-kb 30000 > profiles/r01_pack_pmc_traffic.json

`--min-kb` keeps the launches of the bench's headline size (the bench also packs the latency
ladder and warm-up payloads with the same kernel).
"""
import argparse
import csv
import glob
import json
import os
import statistics


def per_dispatch(d, counter, kernel):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    vals = {}
    for f in files:
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter or kernel not in row.get("Kernel_Name", ""):
                continue
            key = (f, row.get("Dispatch_Id") or row.get("Correlation_Id"))
            vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    return list(vals.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--kernel", default="pack_kernel")
    ap.add_argument("--algorithmic", type=float, required=True, help="bytes per launch (2*S)")
    ap.add_argument("--min-kb", type=float, default=0.0)
    ap.add_argument("--note", default="")
    a = ap.parse_args()
    w = [v for v in per_dispatch(a.write_dir, "WRITE_SIZE", a.kernel) if v >= a.min_kb]
    f = per_dispatch(a.fetch_dir, "FETCH_SIZE", a.kernel)
    f = [v for v in f if 2 * v >= a.min_kb]
    fk, wk = statistics.mean(f), statistics.mean(w)
    traffic = (2 * fk + wk) * 1024.0  # rocprofv3 reports KiB
    print(json.dumps({
        "FETCH_SIZE": {"dispatches": len(f), "avg_KB": fk},
        "WRITE_SIZE": {"dispatches": len(w), "avg_KB": wk},
        "traffic_bytes_per_launch": traffic,
        "algorithmic_bytes_per_launch": a.algorithmic,
        "ratio": traffic / a.algorithmic,
        "kernel": a.kernel,
        "note": a.note or "separate --pmc passes; FETCH_SIZE x2 per MI355X_MICROARCH.md",
    }, indent=1))


if __name__ == "__main__":
    main()
