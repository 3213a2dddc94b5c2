"""Microbenchmark of the pack kernel variants vs hipMemcpyAsync D2D (the measured copy peak).

Variants (unroll, non-temporal, chunk bytes) are interleaved in ONE process over several rounds
(cdna_hip_programming.md §5.4 rule 24); kernel time comes from hipExtLaunchKernel start/stop
stamps... here from HIP events around a batch of back-to-back launches (includes launch gaps).
Buffers rotate over > 512 MiB so the 256 MiB Infinity Cache does not inflate HBM numbers.
Prints one JSON line per (variant, size) with the median over rounds.
"""
from __future__ import annotations

import argparse
import itertools
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dora_amd import device  # noqa: E402
from dora_amd._lib import call  # noqa: E402
from dora_amd.arrow_utils import Plan  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--sizes", default="4096000,16777216,40960000")
    ap.add_argument("--misalign", type=int, default=0)
    ap.add_argument("--sweep", action="store_true", help="sweep unroll x nt x chunk")
    ap.add_argument("--signal-sweep", action="store_true",
                    help="packs that signal their fill from the kernel, by workgroups per XCD")
    ap.add_argument("--grids", default="512,1024", help="signal sweep: signalling grids")
    ap.add_argument("--units", default="0,4,8", help="signal sweep: loads in flight per lane")
    ap.add_argument("--chunks", default="0,8192,16384,32768", help="signal sweep: chunk bytes")
    ap.add_argument("--c3", action="store_true",
                    help="C3 shape: 1M-point List<Struct<x,y,z,intensity>> clouds (f32 buffers "
                         "at 4 mod 16) instead of byte buffers; memcpy = one D2D of the sample")
    args = ap.parse_args()
    device.set_device(0)
    s = device.Stream()
    e0, e1 = device.Event(), device.Event()
    if args.sweep:
        variants = [("memcpy", 0, 0, 0)] + [("pack", u, nt, ch) for u, nt, ch in itertools.product(
            [2, 4, 8], [1], [0, 4096, 8192, 16384, 20480, 32768])]
    elif args.signal_sweep:
        # (kind, signalling grid): the pack signals a scratch flag from its workgroup 0;
        # ("pack", 0, 2, 0): the same write-through stores without the signal
        variants = [("memcpy", 0, 0, 0), ("pack", 0, -1, 0), ("pack", 0, 2, 0)] + [
            ("wtgrid", w, 2, 0) for w in [int(x) for x in args.grids.split(",")]] + [
            ("sig", w, u, ch) for w in [int(x) for x in args.grids.split(",")]
            for u in [int(x) for x in args.units.split(",")]
            for ch in [int(x) for x in args.chunks.split(",")]]
    else:
        variants = [("memcpy", 0, 0, 0), ("pack", 0, -1, 0)]
    sizes = [int(x) for x in args.sizes.split(",")]
    if args.c3:
        from dora_amd.device import DeviceArray
        from dora_amd.workloads import point_cloud
        cloud = point_cloud()
        with Plan.of(cloud) as p:
            sizes = [p.size]
    for size in sizes:
        nbuf = max(2, min(64, (640 << 20) // (2 * size)))
        srcs = [device.DeviceBuffer(size + 64) for _ in range(nbuf)]
        dsts = [device.DeviceBuffer(size + 64) for _ in range(nbuf)]
        for b in srcs:
            device.fill_splitmix(b.ptr, b.size, 7, s)
        if args.c3:
            arrays = [DeviceArray.from_pyarrow(cloud) for _ in range(nbuf)]
            plans = [Plan.of(a) for a in arrays]
        else:
            plans = [Plan.of_bytes(b.ptr + args.misalign, size, on_device=True) for b in srcs]
        res = {v: [] for v in variants}
        for _ in range(args.rounds):
            for v in variants:
                kind, u, nt, ch = v
                if kind == "pack":
                    call("dora_gpu_test_pack_tune", u, nt, ch)
                elif kind == "wtgrid":  # write-through stores, no signal, grid capped at u
                    call("dora_gpu_test_pack_tune", 0, 2, ch)
                elif kind == "sig":  # (grid, unroll, chunk)
                    call("dora_gpu_test_pack_tune", nt, -1, ch)
                call("dora_gpu_test_pack_signal_tune", u if kind in ("sig", "wtgrid") else 0,
                     int(kind == "sig"))

                def launch(k):
                    if kind in ("pack", "sig", "wtgrid"):
                        plans[k].pack(dsts[k].ptr, size, s)
                    else:
                        call("dora_gpu_memcpy_async", dsts[k].ptr, srcs[k].ptr + args.misalign,
                             size, s.handle)
                for w in range(3):
                    launch(w % nbuf)
                e0.record(s)
                for it in range(args.iters):
                    launch(it % nbuf)
                e1.record(s)
                e1.sync()
                res[v].append(e0.elapsed_ms(e1) / args.iters)
        call("dora_gpu_test_pack_tune", 0, -1, 0)
        call("dora_gpu_test_pack_signal_tune", 0, 0)
        call("dora_gpu_test_pack_tune", 0, -1, 0)
        for v in variants:
            ms = statistics.median(res[v])
            gbs = 2 * size / (ms * 1e-3) / 1e9
            print(json.dumps({"variant": v[0], "unroll": v[1], "nt": v[2], "chunk": v[3],
                              "size": size, "misalign": "c3" if args.c3 else args.misalign,
                              "us_per_launch": round(ms * 1e3, 2), "min_us": round(min(res[v]) * 1e3, 2),
                              "GBps_2S": round(gbs, 1), "frac_of_8TBps": round(gbs / 8000, 3)}),
                  flush=True)
        for p in plans:
            p.close()
        if args.c3:
            for a in arrays:
                a.close()
        for b in srcs + dsts:
            b.free()


if __name__ == "__main__":
    main()
