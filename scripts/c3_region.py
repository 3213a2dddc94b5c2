#!/usr/bin/env python3
"""C3 (BASELINE configs[2]) regions of a bench.py run from its rocprofv3 kernel trace — the
independent check of the line's `c3.frac` and `c3.steady_frac` (verdict r04 item 2).

bench.py's C3 block (run_c3_block) dispatches the only multi-segment packs of a C2 run
(`dora_aql_pack_u4`): 2 x 24 warm-up clouds, then the 200-cloud steady region, then the 20-cloud
burst the line reports.  Per region this prints the packs' own durations, the device span (first
start -> last end) per pack — bench.py's figure, from the packs' own stamps — and the union of the
packs' intervals per pack, with the fraction of 8 TB/s each gives for 2 x S bytes per pack.

    rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c3p -o run -- \\
        python bench.py --no-ladder --no-cpu-baseline --steps 20 --warmup 5 > line.json
    python scripts/c3_region.py gpurun_out/c3p --line line.json
"""
import argparse
import csv
import glob
import json
import os
import statistics

HBM_GBPS = 8000.0
C3_SAMPLE = 13125120  # slot bytes of the bench cloud incl. its validity tail
C3_BYTES = 13000068   # the reference sample: algorithmic bytes are 2 x this per pack


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


def region(iv, size):
    own = [(e - s) / 1000.0 for s, e in iv]
    span = (max(e for _, e in iv) - min(s for s, _ in iv)) / 1000.0
    busy = union_ns(iv) / 1000.0
    n = len(iv)
    frac = lambda us: round(2.0 * size / (us * 1e-6) / 1e9 / HBM_GBPS, 4)  # noqa: E731
    return {"packs": n,
            "own_duration_us": {"mean": round(statistics.mean(own), 3),
                                "median": round(statistics.median(own), 3),
                                "max": round(max(own), 3)},
            "span_us": round(span, 2), "span_us_per_pack": round(span / n, 3),
            "union_us_per_pack": round(busy / n, 3),
            "frac_span": frac(span / n), "frac_union": frac(busy / n)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--burst", type=int, default=20)
    ap.add_argument("--steady", type=int, default=200)
    ap.add_argument("--kernel", default="dora_aql_pack_u4")
    ap.add_argument("--size", type=int, default=C3_BYTES)
    ap.add_argument("--line", help="the bench.py stdout line of the same run (its c3 block)")
    ap.add_argument("--detail", help="the bench.py detail file of the same run: its burst's pack "
                    "intervals from the packs' own stamps, compared pack by pack with the trace")
    a = ap.parse_args()
    f = glob.glob(os.path.join(a.trace_dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if r["Kernel_Name"].startswith(a.kernel)]
    # dispatch order: the correlation id grows with every dispatch
    rows.sort(key=lambda r: int(r.get("Correlation_Id") or r["Start_Timestamp"]))
    iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    burst = iv[-a.burst:]
    steady = iv[-a.burst - a.steady:-a.burst]
    out = {"trace": os.path.relpath(f, a.trace_dir), "kernel": a.kernel,
           "launches_in_trace": len(iv), "algorithmic_bytes_per_pack": 2 * a.size,
           "burst": region(burst, a.size), "steady": region(steady, a.size)}
    if a.line:
        line = json.loads(open(a.line).read().strip().splitlines()[-1])
        c3 = line.get("c3") or {}
        out["line"] = {"c3_frac": c3.get("frac"), "c3_steady_frac": c3.get("steady_frac"),
                       "us_per_launch": c3.get("us_per_launch")}
        if c3.get("frac"):
            out["burst_span_vs_line"] = round(out["burst"]["frac_span"] / c3["frac"], 4)
        if c3.get("steady_frac"):
            out["steady_span_vs_line"] = round(out["steady"]["frac_span"] / c3["steady_frac"], 4)
    if a.detail:
        # the packs' own stamps (first workgroup start -> last workgroup end, relative to the
        # burst's first start) against the trace's packet intervals (command-processor start ->
        # end of pipe), both aligned on the burst's first pack
        st = json.load(open(a.detail)).get("c3", {}).get("pack_intervals_us") or []
        if len(st) == len(burst):
            t0 = burst[0][0]
            tr = [((x - t0) / 1000.0, (y - t0) / 1000.0) for x, y in sorted(burst)]
            st = sorted(st)
            d_start = [t[0] - s_[0] for t, s_ in zip(tr, st)]
            d_end = [t[1] - s_[1] for t, s_ in zip(tr, st)]
            out["trace_minus_stamps_us"] = {
                "start_median": round(statistics.median(d_start), 3),
                "end_median": round(statistics.median(d_end), 3),
                "last_end": round(tr[-1][1] - max(e for _, e in st), 3),
                "span_trace": round(max(e for _, e in tr), 3),
                "span_stamps": round(max(e for _, e in st), 3)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
