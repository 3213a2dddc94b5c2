#!/usr/bin/env python3
"""Device samples to a receiver without a GPU (the native bench sink, DORA_GPU_DEVICE -1): p50 /
p99 per size at 1 ms spacing, for the staging A/B (DESIGN §2 host-only receivers)."""
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    sizes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "8,4096,65536,262144").split(",")]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    from dora_amd import device
    from dora_amd.dataflow import Dataflow
    from dora_amd.launcher import Launcher
    from dora_amd.workloads import payload_seed
    launcher = Launcher()
    res = os.path.join(tempfile.mkdtemp(prefix="dora-d2h-"), "sink.json")
    desc = {"nodes": [
        {"id": "node", "path": "dynamic", "outputs": ["to_host", "warm"],
         "inputs": {"ack": "hostsink/ack"}},
        {"id": "hostsink", "path": "dora-gpu-bench-sink", "outputs": ["ack"],
         "inputs": {"to_host": {"source": "node/to_host", "queue_size": 10},
                    "warm": {"source": "node/warm", "queue_size": 10}},
         "env": {"DORA_BENCH_RESULT": res}, "_unstable_deploy": {"gpu": -1}},
    ]}
    from dora_amd.node import Node
    s = device.Stream()
    with Dataflow(desc, launcher=launcher) as df:
        node = Node("node", dataflow=df.shm, device=0)
        seq = 0
        for z in sizes:
            b = device.DeviceBuffer(z)
            device.fill_splitmix(b.ptr, z, payload_seed(z), s)
            s.sync()
            for _ in range(5):
                node.send_output_device_bytes("warm", b.ptr, z, {"seq": seq})
                seq += 1
                time.sleep(1e-3)
            for _ in range(n):
                node.send_output_device_bytes("to_host", b.ptr, z, {"seq": seq, "t_start": time.time_ns()})
                seq += 1
                time.sleep(1e-3)
            b.free()
        node.send_output("warm", b"", {"seq": seq, "ack": True})
        node.wait_input("ack", "seq", seq, 60)
        node.close()
        df.wait(60)
    launcher.close()
    sink = json.load(open(res))
    out = {"mode": "hip" if os.environ.get("DORA_GPU_STAGE_HIP") == "1" else "aql",
           "sched": sink.get("sched")}
    for x in sink["series"]:
        if x["input"] == "to_host":
            out[str(x["size"])] = [x["p50_us"], x["p99_us"], x["full_p50_us"]]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
