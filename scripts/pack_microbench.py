"""Microbenchmark of the pack kernel vs hipMemcpyAsync D2D (the measured copy peak).

Buffers rotate over > 512 MiB so the 256 MiB Infinity Cache does not inflate HBM numbers.
Prints one JSON line per (variant, size).  Usage: python scripts/pack_microbench.py [--iters N]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dora_amd import device  # noqa: E402
from dora_amd._lib import call  # noqa: E402
from dora_amd.arrow_utils import Plan  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--sizes", default="4096,65536,1048576,4096000,16777216,40960000")
    ap.add_argument("--misalign", type=int, default=0)
    args = ap.parse_args()
    device.set_device(0)
    s = device.Stream()
    e0, e1 = device.Event(), device.Event()
    for size in [int(x) for x in args.sizes.split(",")]:
        nbuf = max(2, min(64, (640 << 20) // (2 * size)))
        srcs = [device.DeviceBuffer(size + 64) for _ in range(nbuf)]
        dsts = [device.DeviceBuffer(size + 64) for _ in range(nbuf)]
        for b in srcs:
            device.fill_splitmix(b.ptr, b.size, 7, s)
        plans = [Plan.of_bytes(b.ptr + args.misalign, size, on_device=True) for b in srcs]
        for variant in ["pack", "memcpy"]:
            for w in range(3):
                k = w % nbuf
                if variant == "pack":
                    plans[k].pack(dsts[k].ptr, size, s)
                else:
                    call("dora_gpu_memcpy_async", dsts[k].ptr, srcs[k].ptr + args.misalign, size,
                         s.handle)
            e0.record(s)
            for it in range(args.iters):
                k = it % nbuf
                if variant == "pack":
                    plans[k].pack(dsts[k].ptr, size, s)
                else:
                    call("dora_gpu_memcpy_async", dsts[k].ptr, srcs[k].ptr + args.misalign, size,
                         s.handle)
            e1.record(s)
            e1.sync()
            ms = e0.elapsed_ms(e1) / args.iters
            gbs = 2 * size / (ms * 1e-3) / 1e9
            print(json.dumps({"variant": variant, "size": size, "misalign": args.misalign,
                              "us_per_launch": round(ms * 1e3, 2), "GBps_2S": round(gbs, 1),
                              "frac_of_8TBps": round(gbs / 8000, 3)}), flush=True)
        for p in plans:
            p.close()
        for b in srcs + dsts:
            b.free()


if __name__ == "__main__":
    main()
