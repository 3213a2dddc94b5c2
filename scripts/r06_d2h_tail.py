#!/usr/bin/env python3
"""Where the latency ladder's d2h p99 at 6.2 / 40.96 MB came from (17-34 ms against a 127 /
750 us p50): a device producer and the benchmark sink without a GPU (its own process, as in
bench.py).  The first device sample such a receiver stages ("first_<size>", sent alone) against
the 200 that follow 1 ms apart ("x").  A Python receiver in the producer's process is no
stand-in: its first host value also pays the import of pyarrow.

    python scripts/r06_d2h_tail.py --n 200
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
    ap.add_argument("--n", type=int, default=200)
    ap.add_argument("--sizes", default="6220800,40960000")
    a = ap.parse_args()
    sizes = [int(x) for x in a.sizes.split(",")]
    from dora_amd.launcher import Launcher
    launcher = Launcher()
    from dora_amd import device
    from dora_amd.dataflow import Dataflow
    from dora_amd.device import DeviceBuffer
    from dora_amd.node import Node
    res = os.path.join(tempfile.mkdtemp(prefix="d2h-tail-"), "sink.json")
    outs = ["x"] + [f"first_{z}" for z in sizes]
    desc = {"nodes": [
        {"id": "src", "path": "dynamic", "outputs": outs, "inputs": {"ack": "hs/ack"}},
        {"id": "hs", "path": "dora-gpu-bench-sink", "outputs": ["ack"],
         "inputs": {o: {"source": f"src/{o}", "queue_size": 10} for o in outs},
         "env": {"DORA_BENCH_RESULT": res}, "_unstable_deploy": {"gpu": -1}},
    ]}
    s = device.Stream()
    seq = 0
    with Dataflow(desc, launcher=launcher) as df:
        tx = Node("src", dataflow=df.shm, device=0)
        for z in sizes:
            b = DeviceBuffer(z)
            device.fill_splitmix(b.ptr, z, 7, s)
            s.sync()
            tx.send_output_device_bytes(f"first_{z}", b.ptr, z, {"seq": seq})
            seq += 1
            tx.send_output(f"first_{z}", b"", {"seq": seq, "ack": True})
            tx.wait_input("ack", "seq", seq, 60.0)
            seq += 1
            for k in range(a.n):
                tx.send_output_device_bytes("x", b.ptr, z, {"seq": seq})
                seq += 1
                time.sleep(1e-3)
            tx.send_output("x", b"", {"seq": seq, "ack": True})
            tx.wait_input("ack", "seq", seq, 60.0)
            seq += 1
            b.free()
        tx.close()
        df.wait(60)
    s.close()
    launcher.close()
    for x in json.load(open(res))["series"]:
        if x["size"]:
            print(json.dumps({k: x[k] for k in ("input", "size", "n", "p50_us", "p99_us",
                                                 "mean_us")}), flush=True)


if __name__ == "__main__":
    main()
