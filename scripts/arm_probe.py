#!/usr/bin/env python3
"""Does a dispatch written ahead behind a barrier-AND start sooner than one rung after the gap?

Both modes run no-op dispatches on a queue of their own (dora_gpu_test_arm_probe): mode 0 writes
the packet and rings the doorbell after the gap; mode 1 writes a barrier-AND waiting on a host
signal plus the dispatch before the gap, and stores the signal after it; mode 2 as 1 with the
dispatch's arguments written only after the gap (counted: dispatches that ran on the old ones).  Printed per gap: p50 /
p90 / p99 of release -> completion seen by the host, interleaved rounds.

    python scripts/arm_probe.py --n 400 --gaps-us 20,1000
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=400)
    ap.add_argument("--gaps-us", default="20,1000")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--keep-awake-us", type=float, default=None)
    a = ap.parse_args()
    import torch
    torch.zeros(1, device="cuda")
    from dora_amd._lib import call
    if a.keep_awake_us is not None:
        call("dora_gpu_set_keep_awake", a.keep_awake_us)
    buf = (ctypes.c_uint64 * a.n)()
    for r in range(a.rounds):
        for gap in [int(x) for x in a.gaps_us.split(",")]:
            for mode in (0, 1, 2):
                call("dora_gpu_test_arm_probe", 0, mode, a.n, gap * 1000, buf)
                stale = sum(1 for x in buf if x >> 63)
                v = sorted((x & ((1 << 63) - 1)) / 1e3 for x in buf[10:])
                q = lambda f: round(v[int(f * (len(v) - 1))], 2)
                print(json.dumps({"round": r, "gap_us": gap, "mode": ["doorbell", "armed", "armed_late_args"][mode], "stale_args": stale,
                                  "keep_awake_us": a.keep_awake_us, "p50_us": q(.5),
                                  "p90_us": q(.9), "p99_us": q(.99), "min_us": round(v[0], 2)}),
                      flush=True)


if __name__ == "__main__":
    main()
