#!/usr/bin/env python3
"""Does the warm thread (aql.cpp warm_main: empty AQL packets while the node sends) delay this
process's other GPU work?  The pattern of tests/test_gpu_dataflow.py
test_device_array_send_waits_for_its_source, timed: a synchronous device send, then a 4 MiB
hipMemcpyAsync on a HIP stream of the same process and its synchronize (timed), 1 ms apart.
Run once per setting of the warm thread's period (dora_gpu_set_keep_awake).

    python scripts/warm_copy_probe.py --n 300 --keep-awake-us 0
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=300)
    ap.add_argument("--bytes", type=int, default=4 << 20)
    ap.add_argument("--keep-awake-us", type=float, default=None)
    a = ap.parse_args()
    from dora_amd import device
    from dora_amd._lib import call
    from dora_amd.dataflow import Dataflow
    from dora_amd.node import Node
    desc = {"nodes": [
        {"id": "node", "path": "dynamic", "outputs": ["latency"], "inputs": {"ack": "sink/ack"}},
        {"id": "sink", "path": "dora-gpu-bench-sink", "outputs": ["ack"],
         "inputs": {"latency": {"source": "node/latency", "queue_size": 10}},
         "env": {"DORA_BENCH_RESULT": os.path.join(os.environ.get("TMPDIR", "/tmp"),
                                                   f"warm-copy-{os.getpid()}.json")}},
    ]}
    if a.keep_awake_us is not None:
        device.set_keep_awake(a.keep_awake_us)
    cpu0 = time.process_time()
    with Dataflow(desc) as df:
        node = Node("node", dataflow=df.shm, device=0)
        src, dst = device.DeviceBuffer(a.bytes), device.DeviceBuffer(a.bytes)
        other = device.Stream()
        copy_us, send_us = [], []
        for k in range(a.n + 20):
            t0 = time.perf_counter()
            node.send_output_device_bytes("latency", src.ptr, 4096, {"seq": k})
            t1 = time.perf_counter()
            call("dora_gpu_memcpy_async", dst.ptr, src.ptr, a.bytes, other.handle)
            other.sync()
            t2 = time.perf_counter()
            if k >= 20:
                send_us.append((t1 - t0) * 1e6)
                copy_us.append((t2 - t1) * 1e6)
            time.sleep(0.001)
        cpu_s = time.process_time() - cpu0
        other.close()
        src.free()
        dst.free()
        node.close()
        df.wait(30)

    def q(xs, f):
        xs = sorted(xs)
        return round(xs[min(len(xs) - 1, int(f * len(xs)))], 2)
    print(json.dumps({"keep_awake_us": a.keep_awake_us, "n": a.n,
                      "process_cpu_s": round(cpu_s, 3),
                      "copy_bytes": a.bytes,
                      "copy_sync_us": {"p50": q(copy_us, 0.5), "p90": q(copy_us, 0.9),
                                       "p99": q(copy_us, 0.99), "max": round(max(copy_us), 2)},
                      "send_us": {"p50": q(send_us, 0.5), "p99": q(send_us, 0.99)},
                      "copy_mean_us": round(statistics.mean(copy_us), 2)}), flush=True)


if __name__ == "__main__":
    main()
