#!/usr/bin/env python3
"""Throughput mode of the Python node (this process, dora_amd.node.Node via the CPython send path)
-> the native bench sink, per size: the Python counterpart of scripts/native_tp.py, with the
sink's and the daemon's host sub-phases when DORA_GPU_TRACE=subphases (this process prints its own to
stderr at exit).

    python scripts/py_tp.py --sizes 1048576,4096000 --n 5000 [--sources 16]
"""
import argparse
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1048576,4096000")
    ap.add_argument("--n", type=int, default=5000)
    ap.add_argument("--sources", type=int, default=16)
    ap.add_argument("--no-params", action="store_true", help="send without parameters")
    ap.add_argument("--align", type=int, default=0,
                    help="allocate each source rounded up to this many bytes (0: exact size)")
    a = ap.parse_args()
    from dora_amd import device
    from dora_amd.dataflow import Dataflow
    from dora_amd.node import Node

    tmp = tempfile.mkdtemp(prefix="dora-py-tp-")
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
    seq = 0
    out = []
    for size in [int(x) for x in a.sizes.split(",")]:
        alloc = -(-size // a.align) * a.align if a.align else size
        bufs = [device.DeviceBuffer(alloc) for _ in range(a.sources)]
        src_mod = sorted({b.ptr % (2 << 20) for b in bufs})
        for b in bufs:
            device.fill_splitmix(b.ptr, size, 1, stream)
        stream.sync()
        for k in range(24):
            node.send_output_device_bytes("throughput", bufs[k % a.sources].ptr, size, {"seq": seq})
            seq += 1
        node.send_output("throughput", b"", {"seq": seq, "ack": True})
        node.wait_input("ack", "seq", seq, 60.0)
        seq += 1
        d0 = node.dataflow_counters("sink")["dropped_inputs"]
        t0 = time.perf_counter()
        if a.no_params:
            for k in range(a.n):
                node.send_output_device_bytes("throughput", bufs[k % a.sources].ptr, size)
        else:
            for k in range(a.n):
                node.send_output_device_bytes("throughput", bufs[k % a.sources].ptr, size,
                                              {"seq": seq})
                seq += 1
        node.send_output("throughput", b"", {"seq": seq, "ack": True})
        node.wait_input("ack", "seq", seq, 60.0)
        seq += 1
        dt = time.perf_counter() - t0
        dropped = node.dataflow_counters("sink")["dropped_inputs"] - d0
        got = a.n - dropped
        out.append({"size": size, "n": a.n, "dropped": dropped,
                    "us_per_delivered_msg": round(dt / got * 1e6, 3),
                    "hbm_frac_2S": round(2 * got * size / dt / 8e12, 4),
                    "src_mod_2MiB": src_mod[:8]})
        for b in bufs:
            b.free()
    node.close()
    df.wait(30)
    df.stop()
    sub = {}
    for who in ("sink", "_daemon"):
        for line in (df.log(who) or "").splitlines():
            if line.startswith('{"subphases"'):
                sub[who] = json.loads(line)["subphases"]
    for r in out:
        print(json.dumps(r), flush=True)
    if sub:
        print(json.dumps({"subphases_ns": sub}), flush=True)


if __name__ == "__main__":
    main()
