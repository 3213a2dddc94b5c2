"""Join DORA_GPU_TRACE csv files by drop token and print median stage-to-stage times (µs)."""
import csv
import glob
import statistics
import sys
from collections import defaultdict

NAMES = {1: "alloc_begin", 2: "alloc_end", 3: "launched", 4: "fill_ordered", 5: "sent",
         6: "token_back", 7: "routed", 8: "token_done", 9: "popped", 10: "filled", 11: "released"}
ORDER = [1, 2, 3, 4, 5, 7, 9, 10, 11, 8, 6]


def main(d):
    ev = defaultdict(dict)
    for f in glob.glob(f"{d}/*.trace.csv"):
        for r in csv.DictReader(open(f)):
            ev[r["token"]].setdefault(int(r["point"]), int(r["t_ns"]))
    # points nobody recorded (e.g. the daemon ran without DORA_GPU_TRACE) drop out of the chain
    seen = [p for p in ORDER if any(p in v for v in ev.values())]
    full = [v for v in ev.values() if all(p in v for p in seen)]
    print(f"{len(ev)} tokens, {len(full)} complete over points {[NAMES[p] for p in seen]}")
    for a, b in zip(seen, seen[1:]):
        xs = [(v[b] - v[a]) / 1000 for v in full]
        if xs:
            print(f"{NAMES[a]:>13} -> {NAMES[b]:<13} p50 {statistics.median(xs):8.2f}  "
                  f"p90 {sorted(xs)[int(0.9 * (len(xs) - 1))]:8.2f}")
    starts = sorted(v[3] for v in full if 3 in v)
    if len(starts) > 2:
        gaps = [(b - a) / 1000 for a, b in zip(starts, starts[1:])]
        print(f"launch-to-launch p50 {statistics.median(gaps):.2f} us")


if __name__ == "__main__":
    main(sys.argv[1])
