#!/usr/bin/env python3
"""A D2H copy of a small sample into pinned host memory, HIP against the HSA copy call
(dora_gpu_test_d2h_copy_probe): p50 / p99 of call -> complete per size, 1 ms apart like the
latency ladder, two interleaved rounds.  The staging of a receiver without a GPU (node.cpp
stage_to_host) pays the HIP figure at every small size.

    python scripts/d2h_copy_probe.py --n 300
"""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=300)
    ap.add_argument("--sizes", default="8,4096,65536,1048576")
    a = ap.parse_args()
    from dora_amd._lib import call
    buf = (ctypes.c_uint64 * a.n)()
    for r in range(2):
        for z in [int(x) for x in a.sizes.split(",")]:
            for mode in (0, 1):
                call("dora_gpu_test_d2h_copy_probe", 0, mode, z, a.n, 1000000, buf)
                v = sorted(x / 1e3 for x in buf[10:])
                q = lambda f: round(v[int(f * (len(v) - 1))], 2)
                print(json.dumps({"round": r, "bytes": z, "mode": ["hip", "hsa"][mode],
                                  "p50_us": q(.5), "p90_us": q(.9), "p99_us": q(.99)}), flush=True)


if __name__ == "__main__":
    main()
