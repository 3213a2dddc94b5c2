#!/usr/bin/env python3
"""Pipelined single-segment AQL packs with the in-kernel fill signal (mode 0) against the
packet's completion signal (1: release fence none, 2: agent), interleaved rounds; one JSON line
per (round, size, mode).  dora_gpu_test_aql_pipeline (csrc/aql.cpp aql_pipeline_bench).

    python scripts/aql_pipeline_probe.py --sizes 4096000,16777216,40960000 --rounds 3
"""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dora_amd import _lib, device  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="4096000,16777216,40960000")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--n", type=int, default=2000)
    ap.add_argument("--modes", default="0,1,2")
    ap.add_argument("--queues", type=int, default=4)
    ap.add_argument("--depth", type=int, default=2)
    a = ap.parse_args()
    device.set_device(0)
    lib = _lib.load()
    for r in range(a.rounds):
        for size in [int(x) for x in a.sizes.split(",")]:
            n = a.n if size < (8 << 20) else a.n // 4
            for mode in [int(x) for x in a.modes.split(",")]:
                us = ctypes.c_double()
                rc = lib.dora_gpu_test_aql_pipeline(0, size, n, mode, a.queues, a.depth,
                                                    ctypes.byref(us))
                if rc:
                    print(json.dumps({"round": r, "size": size, "mode": mode,
                                      "error": lib.dora_gpu_last_error().decode()}), flush=True)
                    return 1
                print(json.dumps({"round": r, "size": size, "mode": mode, "n": n,
                                  "queues": a.queues, "depth": a.depth,
                                  "us_per_msg": round(us.value, 3),
                                  "hbm_frac_2S": round(2 * size / us.value / 8e6, 4)}),
                      flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
