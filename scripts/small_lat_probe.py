#!/usr/bin/env python3
"""Where a small message's latency goes (verdict r04 item 1): device-resident payloads of
8 B..4 KB and host-resident 8 B / 2 KB (inline Vec samples), N messages per size 1 ms apart
from one node to another (in-process daemon, both nodes on GPU 0), with the per-message trace
(DORA_GPU_TRACE, set by this script).  Per size: the median of each host stage (sender's
alloc -> launch -> sent, daemon routing, receiver pop, the wait for the fill flag) and the pack's
own device time from its stamps (s_memrealtime), so
    GPU round trip - kernel = dispatch + completion visibility.

    python scripts/small_lat_probe.py --n 500 > small_lat.json
"""
import argparse
import csv
import glob
import json
import os
import statistics
import sys
import tempfile
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

TRACE_DIR = tempfile.mkdtemp(prefix="dora-small-lat-")
os.environ["DORA_GPU_TRACE"] = TRACE_DIR  # read when the library loads

P = {"alloc_begin": 1, "alloc_end": 2, "launched": 3, "fill_ordered": 4, "sent": 5, "routed": 7,
     "popped": 9, "filled": 10, "released": 11, "gpu_start": 12, "gpu_signal": 13}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=500)
    ap.add_argument("--gap-us", type=int, default=1000)
    a = ap.parse_args()
    import ctypes

    from dora_amd import _lib, device
    from dora_amd.dataflow import daemon_spec, parse_descriptor
    from dora_amd.device import DeviceBuffer
    from dora_amd.node import Node
    lib = _lib.load()
    device.set_device(0)
    desc = {"nodes": [{"id": "src", "outputs": ["x"]},
                      {"id": "dst", "inputs": {"x": {"source": "src/x", "queue_size": 10}}}]}
    shm = f"/dora-gpu-smalllat-{os.getpid()}"
    h = ctypes.c_void_p()
    _lib.call("dora_daemon_create", shm.encode(), daemon_spec(parse_descriptor(desc)).encode(),
              1 << 20, ctypes.byref(h))
    threading.Thread(target=lambda: lib.dora_daemon_run(h.value, 600000), daemon=True).start()
    nodes = {}
    ts = [threading.Thread(target=lambda i=i: nodes.update({i: Node(i, dataflow=shm, device=0)}))
          for i in ("src", "dst")]
    [t.start() for t in ts]
    [t.join(60) for t in ts]
    src, dst = nodes["src"], nodes["dst"]
    buf = DeviceBuffer(4096)
    s = device.Stream()
    device.fill_splitmix(buf.ptr, 4096, 7, s)
    s.sync()
    cases = [("dev", 8), ("dev", 512), ("dev", 2048), ("dev", 4096), ("host", 8), ("host", 2048)]
    host_bytes = bytes(range(256)) * 16
    e2e = {}
    for kind, z in cases:
        lat = []
        for k in range(a.n + 5):
            t0 = time.perf_counter()
            if kind == "dev":
                src.send_output_device_bytes("x", buf.ptr, z, {"k": k})
            else:
                src.send_output("x", host_bytes[:z], {"k": k})
            ev = dst.next(timeout=10)
            lat.append((time.perf_counter() - t0) * 1e6)
            del ev
            time.sleep(a.gap_us / 1e6)
        e2e[(kind, z)] = sorted(lat[5:])
    src.close()
    dst.close()
    lib.dora_daemon_free(h.value)
    # the trace buffer was flushed when the first node went (dora_node_free)
    ev = {}
    for f in glob.glob(os.path.join(TRACE_DIR, "*.trace.csv")):
        for r in csv.DictReader(open(f)):
            ev.setdefault(r["token"], {}).setdefault(int(r["point"]), int(r["t_ns"]))
    msgs = sorted((v for v in ev.values() if P["launched"] in v or P["popped"] in v),
                  key=lambda v: v.get(P["launched"], v.get(P["popped"], 0)))
    out = []
    # device cases have tokens (traced); inline host samples carry none: end-to-end only
    dev_cases = [c for c in cases if c[0] == "dev"]
    per = a.n + 5
    for i, (kind, z) in enumerate(dev_cases):
        grp = msgs[i * per:(i + 1) * per][5:]

        def med(x, y):
            xs = [(v[P[y]] - v[P[x]]) / 1000 for v in grp if P[x] in v and P[y] in v]
            return round(statistics.median(xs), 2) if xs else None
        row = {"source": kind, "bytes": z, "msgs": len(grp),
               "e2e_p50_us": round(statistics.median(e2e[(kind, z)]), 2),
               "stages_p50_us": {"alloc": med("alloc_begin", "alloc_end"),
                                 "launch": med("alloc_end", "launched"),
                                 "launched_to_sent": med("launched", "sent"),
                                 "sent_to_routed": med("sent", "routed"),
                                 "routed_to_popped": med("routed", "popped"),
                                 "popped_to_filled": med("popped", "filled"),
                                 "launched_to_filled": med("launched", "filled"),
                                 "gpu_kernel": med("gpu_start", "gpu_signal")}}
        st = row["stages_p50_us"]
        if st["launched_to_filled"] is not None and st["gpu_kernel"] is not None:
            st["dispatch_and_visibility"] = round(st["launched_to_filled"] - st["gpu_kernel"], 2)
        out.append(row)
    for kind, z in cases:
        if kind == "host":
            out.append({"source": kind, "bytes": z, "msgs": a.n,
                        "e2e_p50_us": round(statistics.median(e2e[(kind, z)]), 2),
                        "e2e_p99_us": round(e2e[(kind, z)][int(0.99 * (a.n - 1))], 2)})
    for r in out:
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
