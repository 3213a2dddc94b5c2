"""Latency outliers from a DORA_GPU_TRACE directory: for every message of the bench's latency
ladder whose sent -> filled time exceeds a threshold, which hop took the time (sender: launch ->
sent; daemon: sent -> routed; receiver: routed -> popped -> filled).  Usage:
    python scripts/lat_outliers.py <trace dir> [threshold_us]"""
import csv
import glob
import statistics
import sys
from collections import defaultdict

HOPS = [("launched", 3, 4), ("fill_ordered->sent", 4, 5), ("sent->routed", 5, 7),
        ("routed->popped", 7, 9), ("popped->filled", 9, 10)]


def main(d, thr):
    ev = defaultdict(dict)
    for f in glob.glob(f"{d}/*.trace.csv"):
        for r in csv.DictReader(open(f)):
            ev[r["token"]].setdefault(int(r["point"]), int(r["t_ns"]))
    full = [v for v in ev.values() if all(p in v for p in (3, 4, 5, 7, 9, 10))]
    tot = sorted((((v[10] - v[5]) / 1e3, v) for v in full), key=lambda x: x[0])
    print(f"{len(full)} complete messages; sent->filled p50 "
          f"{statistics.median(t for t, _ in tot):.1f} us, p99 {tot[int(0.99 * (len(tot) - 1))][0]:.1f}")
    # GPU stamps (points 12/13, s_memrealtime ns) -> host clock: the smallest filled - signal
    # over all messages is the clock offset plus the shortest signal -> observe latency
    g = [v for _, v in tot if 12 in v and 13 in v]
    if g:
        off = min(v[10] - v[13] for v in g)
        for v in g:
            v[12] += off
            v[13] += off
        HOPS[4:] = [("popped->gpu_start", 9, 12), ("gpu_start->signal", 12, 13),
                    ("signal->filled", 13, 10)]
        disp = sorted((v[12] - v[3]) / 1e3 for v in g)
        print(f"launched -> gpu_start (dispatch, + offset error) p50 {statistics.median(disp):.1f}"
              f" p99 {disp[int(0.99 * (len(disp) - 1))]:.1f} us")
    out = [(t, v) for t, v in tot if t > thr]
    blame = defaultdict(int)
    for t, v in out:
        hop = max([h for h in HOPS[2:] if h[1] in v and h[2] in v],
                  key=lambda h: v[h[2]] - v[h[1]])
        blame[hop[0]] += 1
    print(f"{len(out)} above {thr} us; the largest hop of each: {dict(blame)}")
    for t, v in out[-12:]:
        print(f"{t:9.1f} us: " + ", ".join(f"{n} {(v[b] - v[a]) / 1e3:.1f}" for n, a, b in HOPS
                                            if a in v and b in v))


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 50.0)
