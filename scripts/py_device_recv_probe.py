#!/usr/bin/env python3
"""The Python node's receive cost for device inputs on the GPU: this process's Python node sends
`--n` 4 KB device samples (asynchronous) to a Python receiver node (this script again, its own
process), which drains them with Node.next() and reports us per event (each event's DeviceArray
released before the next).

    python scripts/py_device_recv_probe.py --n 2000
"""
import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def receiver():
    from dora_amd.node import Node
    n_want = int(os.environ["PROBE_N"])
    node = Node()
    times, got = [], 0
    t_prev = None
    while got < n_want:
        t0 = time.perf_counter()
        ev = node.next(timeout=30)
        t1 = time.perf_counter()
        if ev is None:
            break
        if ev["type"] != "INPUT":
            continue
        got += 1
        times.append((t1 - t0) * 1e6)
        v = ev.get("value")
        if hasattr(v, "close"):
            v.close()
        del ev
    node.send_output("done", b"", {"got": got})
    times.sort()
    with open(os.environ["PROBE_OUT"], "w") as f:
        json.dump({"n": got, "next_us_p50": round(times[len(times) // 2], 2),
                   "next_us_p10": round(times[len(times) // 10], 2),
                   "next_us_mean": round(sum(times) / len(times), 2)}, f)
    node.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2000)
    a = ap.parse_args()
    from dora_amd import device
    from dora_amd.dataflow import Dataflow
    from dora_amd.node import Node
    out = os.path.join(tempfile.mkdtemp(prefix="dora-pydev-"), "recv.json")
    desc = {"nodes": [
        {"id": "src", "path": "dynamic", "outputs": ["x"], "inputs": {"done": "recv/done"}},
        {"id": "recv", "path": sys.executable, "args": [os.path.abspath(__file__), "--receiver"],
         "inputs": {"x": {"source": "src/x", "queue_size": 100000}}, "outputs": ["done"],
         "env": {"PROBE_N": str(a.n), "PROBE_OUT": out}},
    ]}
    with Dataflow(desc) as df:
        node = Node("src", dataflow=df.shm, device=0)
        buf = device.DeviceBuffer(4096)
        for k in range(a.n):
            node.send_output_device_bytes("x", buf.ptr, 4096, {"seq": k}, asynchronous=True)
            if k % 8 == 7:
                time.sleep(0.0005)  # let slots come back (in-flight cap)
        node.wait_input("done", "got", a.n, 120.0)
        buf.free()
        node.close()
        df.wait(60)
    print(json.dumps(json.load(open(out))))


if __name__ == "__main__":
    if "--receiver" in sys.argv:
        receiver()
    else:
        main()
