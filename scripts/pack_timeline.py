#!/usr/bin/env python3
"""Per-pack device timeline of a back-to-back burst from the Python node (this process) to the
native bench sink: every pack's own start -> fill-signal time from the stamps its first
workgroup writes into the fill flag's line, and, per AQL queue (sends rotate over the queues),
the gap from one pack's signal to the next pack's start on the same queue (negative: the two
overlapped).  Sources rotate past the caches.

    python scripts/pack_timeline.py --size 4096000 --n 2000
"""
import argparse
import json
import os
import statistics
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def q(v, p):
    v = sorted(v)
    return round(v[min(len(v) - 1, int(p * len(v)))], 3) if v else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=4096000)
    ap.add_argument("--n", type=int, default=2000)
    ap.add_argument("--sources", type=int, default=64)
    a = ap.parse_args()
    from dora_amd import device
    from dora_amd.dataflow import Dataflow
    from dora_amd.node import Node

    tmp = tempfile.mkdtemp(prefix="dora-timeline-")
    desc = {"nodes": [
        {"id": "node", "path": "dynamic", "outputs": ["throughput"],
         "inputs": {"ack": "sink/ack"}, "_unstable_deploy": {"gpu": 0}},
        {"id": "sink", "path": "dora-gpu-bench-sink", "outputs": ["ack"],
         "inputs": {"throughput": {"source": "node/throughput", "queue_size": 10}},
         "env": {"DORA_BENCH_RESULT": os.path.join(tmp, "sink.json")},
         "_unstable_deploy": {"gpu": 0}},
    ]}
    df = Dataflow(desc).start()
    node = Node("node", dataflow=df.shm, device=0)
    node.set_async_sends(True)  # sources never rewritten: packs overlap
    stream = device.Stream()
    bufs = [device.DeviceBuffer(a.size) for _ in range(a.sources)]
    for b in bufs:
        device.fill_splitmix(b.ptr, a.size, 1, stream)
    stream.sync()
    seq = 0
    for k in range(48):
        node.send_output_device_bytes("throughput", bufs[k % a.sources].ptr, a.size, {"seq": seq})
        seq += 1
    node.send_output("throughput", b"", {"seq": seq, "ack": True})
    node.wait_input("ack", "seq", seq, 60.0)
    seq += 1
    node.region_begin()
    t0 = time.perf_counter()
    for k in range(a.n):
        node.send_output_device_bytes("throughput", bufs[k % a.sources].ptr, a.size, {"seq": seq})
        seq += 1
    node.send_output("throughput", b"", {"seq": seq, "ack": True})
    node.wait_input("ack", "seq", seq, 60.0)
    wall = time.perf_counter() - t0
    node.sync()
    reg = node.region_end()
    iv = node.pack_intervals()[-a.n:]
    nq = 4  # aql.cpp kQueues
    own = [(b - x) * 1e3 for x, b in iv]
    gaps = [(iv[i + nq][0] - iv[i][1]) * 1e3 for i in range(len(iv) - nq)]
    starts = sorted(x for x, _ in iv)
    sgap = [(starts[i + 1] - starts[i]) * 1e3 for i in range(len(starts) - 1)]
    print(json.dumps({
        "size": a.size, "n": a.n, "queues": nq, "sources": a.sources,
        "us_per_msg_wall": round(wall / a.n * 1e6, 3),
        "device_span_us_per_pack": round(reg["span_ms"] * 1e3 / max(reg["packs"], 1), 3),
        "own_us": {"p10": q(own, .1), "p50": q(own, .5), "p90": q(own, .9)},
        "same_queue_gap_us": {"p10": q(gaps, .1), "p50": q(gaps, .5), "p90": q(gaps, .9)},
        "start_gap_us": {"p50": q(sgap, .5), "mean": round(statistics.mean(sgap), 3) if sgap else None},
        "stamped": len(iv)}), flush=True)
    for b in bufs:
        b.free()
    node.close()
    df.wait(30)
    df.stop()


if __name__ == "__main__":
    main()
