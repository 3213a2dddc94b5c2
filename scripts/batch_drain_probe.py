#!/usr/bin/env python3
"""GPU-side rate of batch packs: N async sends held in the AQL backlog (dora_gpu_test_aql_hold),
then released at once — the time from the release to every fill complete is the device's rate
for batches of up to 8 messages.  Sources rotate past the caches.  Run with
DORA_GPU_MAX_IN_FLIGHT >= N.

    DORA_GPU_MAX_IN_FLIGHT=64 python scripts/batch_drain_probe.py --sizes 4096000 --n 64
"""
import argparse
import ctypes
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1048576,4096000,13000068")
    ap.add_argument("--n", type=int, default=16)  # <= the 20-slot cache: no allocations
    ap.add_argument("--reps", type=int, default=12)
    a = ap.parse_args()
    from dora_amd import _lib, device
    from dora_amd.dataflow import daemon_spec, parse_descriptor
    from dora_amd.node import Node
    lib = _lib.load()
    device.set_device(0)
    desc = {"nodes": [
        {"id": "src", "outputs": ["raw"]},
        {"id": "dst", "outputs": [], "inputs": {"raw": {"source": "src/raw", "queue_size": 1000}}},
    ]}
    shm = f"/dora-gpu-drain-{os.getpid()}"
    h = ctypes.c_void_p()
    _lib.call("dora_daemon_create", shm.encode(), daemon_spec(parse_descriptor(desc)).encode(),
              4 << 20, ctypes.byref(h))
    t = threading.Thread(target=lambda: lib.dora_daemon_run(h.value, 600000), daemon=True)
    t.start()
    nodes = {}

    def mk(i):
        nodes[i] = Node(i, dataflow=shm, device=0)
    ts = [threading.Thread(target=mk, args=(i,)) for i in ("src", "dst")]
    [x.start() for x in ts]
    [x.join(60) for x in ts]
    src, dst = nodes["src"], nodes["dst"]
    src.set_async_sends(True)
    batch = True
    for size in [int(x) for x in a.sizes.split(",")]:
        nsrc = max(2, min(64, (1 << 30) // size))
        bufs = [device.DeviceBuffer(size) for _ in range(nsrc)]
        s = device.Stream()
        for b in bufs:
            device.fill_splitmix(b.ptr, size, 7, s)
        s.sync()
        res = []
        for rep in range(a.reps + 1):
            b0 = device.aql_batch_stats(0)
            if batch:
                device.aql_hold(0, True)
            t0 = time.perf_counter()
            for k in range(a.n):
                src.send_output_device_bytes("raw", bufs[(rep * a.n + k) % nsrc].ptr, size)
            t1 = time.perf_counter()
            if batch:
                device.aql_hold(0, False)
            src.sync()
            t2 = time.perf_counter()
            b1 = device.aql_batch_stats(0)
            # drain the receiver so the tokens come back
            got = 0
            while got < a.n:
                ev = dst.next(timeout=10)
                if ev is None:
                    break
                if ev["type"] == "INPUT":
                    got += 1
                    ev["value"].close() if hasattr(ev.get("value"), "close") else None
                    ev["_event"].free()
            if rep:  # the first repetition creates the slots
                t_gpu = (t2 - t1) if batch else (t2 - t0)
                res.append({"us_per_msg": round(t_gpu / a.n * 1e6, 3),
                            "batches": b1["batches"] - b0["batches"],
                            "batched": b1["batched_msgs"] - b0["batched_msgs"],
                            "send_loop_us": round((t1 - t0) * 1e6, 1)})
        us = sorted(r["us_per_msg"] for r in res)
        print(json.dumps({"size": size, "n": a.n, "batch": batch, "us_per_msg_med": us[len(us) // 2],
                          "hbm_frac_2S": round(2 * size / us[len(us) // 2] / 8e6, 4), "reps": res}),
              flush=True)
        for b in bufs:
            b.free()
        s.close()
    src.close()
    dst.close()
    t.join(30)
    lib.dora_daemon_free(h.value)


if __name__ == "__main__":
    main()
