#!/usr/bin/env python3
"""In-process A/B of pack shapes on the C3 send path (tuning experiment): one dataflow
(this process's node -> dora-gpu-bench-sink on the same GPU), 1M-point clouds sent back to
back; the pack shape (unroll, chunk bytes) is switched between bursts with dora_gpu_pack_tune
and the variants are interleaved over rounds, so box-to-box noise does not enter the comparison.
Prints one JSON line per variant: median us per cloud over the rounds.

    python scripts/c3_ab.py --rounds 5 --n 300
"""
import argparse
import json
import os
import statistics
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--n", type=int, default=300)
    ap.add_argument("--size", type=int, default=0, help="C2 payload bytes instead of C3 clouds")
    a = ap.parse_args()
    from dora_amd.dataflow import Dataflow
    res = os.path.join(tempfile.mkdtemp(prefix="dora-ab-"), "sink.json")
    desc = {"nodes": [
        {"id": "node", "path": "dynamic", "outputs": ["throughput"], "inputs": {"ack": "sink/ack"}},
        {"id": "sink", "path": "dora-gpu-bench-sink", "outputs": ["ack"],
         "inputs": {"throughput": {"source": "node/throughput", "queue_size": 10}},
         "env": {"DORA_BENCH_RESULT": res}},
    ]}
    df = Dataflow(desc).start()
    from dora_amd import device
    from dora_amd._lib import call
    from dora_amd.device import DeviceArray
    from dora_amd.node import Node
    from dora_amd.workloads import point_cloud
    node = Node("node", dataflow=df.shm, device=0)
    node.set_async_sends(True)  # sources never rewritten: packs overlap
    if a.size:
        s = device.Stream()
        srcs = [device.DeviceBuffer(a.size) for _ in range(max(2, min(16, (640 << 20) // a.size)))]
        for b in srcs:
            device.fill_splitmix(b.ptr, a.size, 7, s)
        s.sync()

        def send(k, meta):
            node.send_output_device_bytes("throughput", srcs[k % len(srcs)].ptr, a.size, meta)
    else:
        cloud = point_cloud()
        srcs = [DeviceArray.from_pyarrow(cloud) for _ in range(24)]

        def send(k, meta):
            node.send_output("throughput", srcs[k % len(srcs)], meta)
    seq = [0]

    def burst(n):
        t0 = time.perf_counter()
        for k in range(n):
            send(k, {"seq": seq[0]})
            seq[0] += 1
        node.send_output("throughput", b"", {"seq": seq[0], "ack": True})
        while True:
            ev = node.next(timeout=30)
            if ev is None:
                raise RuntimeError("no ack")
            if ev["type"] == "INPUT" and ev["id"] == "ack" and ev["metadata"].get("seq") == seq[0]:
                break
        seq[0] += 1
        return (time.perf_counter() - t0) / n * 1e6

    variants = [(0, 0), (4, 8192), (4, 16384), (4, 4096), (8, 32768), (8, 16384), (8, 8192)]
    out = {v: [] for v in variants}
    burst(50)
    for _ in range(a.rounds):
        for v in variants:
            call("dora_gpu_pack_tune", v[0], -1, v[1])
            out[v].append(burst(a.n))
    call("dora_gpu_pack_tune", 0, -1, 0)
    node.close()
    df.wait(60)
    df.stop()
    for v in variants:
        print(json.dumps({"workload": f"C2 {a.size} B" if a.size else "C3 1M-point clouds",
                          "unroll": v[0], "chunk": v[1],
                          "us_per_msg_median": round(statistics.median(out[v]), 3),
                          "us_per_msg_min": round(min(out[v]), 3)}), flush=True)


if __name__ == "__main__":
    main()
