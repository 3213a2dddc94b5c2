#!/usr/bin/env python3
"""The synchronous 40.96 MB send (bench.run_sync_leg: each send returns once its pack has read
the source) under different completion paths, interleaved: the command processor's
end-of-pipe signal with up to 3584 workgroups (the default), or the pack's in-kernel fill
signal (done words polled by workgroup 0) with 1024 / 2048 / 3584 workgroups
(dora_gpu_test_cp_lone, dora_gpu_test_pack_signal_tune).  Python node -> native sink, GPU 0.

    python scripts/sync_probe.py --reps 3 --n 200 --modes cp,k1024,k2048,k3584
"""
import argparse
import json
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--n", type=int, default=200)
    ap.add_argument("--size", type=int, default=40960000)
    ap.add_argument("--modes", default="cp,k1024,k2048,k3584")
    ap.add_argument("--chunks", default="0",
                    help="bytes per workgroup chunk (dora_gpu_test_pack_tune; 0: the default 8 KiB)")
    a = ap.parse_args()
    import bench
    from dora_amd import device
    from dora_amd._lib import call
    from dora_amd.dataflow import Dataflow
    from dora_amd.node import Node
    res = os.path.join(tempfile.mkdtemp(prefix="dora-sync-probe-"), "sink.json")
    desc = {"nodes": [
        {"id": "node", "path": "dynamic", "outputs": ["throughput"], "inputs": {"ack": "sink/ack"}},
        {"id": "sink", "path": "dora-gpu-bench-sink", "outputs": ["ack"],
         "inputs": {"throughput": {"source": "node/throughput", "queue_size": 10}},
         "env": {"DORA_BENCH_RESULT": res}},
    ]}
    S = a.size
    with Dataflow(desc) as df:
        node = Node("node", dataflow=df.shm, device=0)
        stream = device.Stream()
        bufs = [device.DeviceBuffer(S) for _ in range(4)]
        for b in bufs:
            device.fill_splitmix(b.ptr, S, 7, stream)
        stream.sync()

        def send(k, meta):
            node.send_output_device_bytes("throughput", bufs[k % len(bufs)].ptr, S, meta)

        def wait_ack(s, timeout=60.0):
            node.wait_input("ack", "seq", s, timeout)
        seq = 0
        for k in range(24):  # slots of this size
            send(k, {"seq": seq})
            seq += 1
        node.send_output("throughput", b"", {"seq": seq, "ack": True})
        wait_ack(seq)
        seq += 1
        modes = a.modes.split(",")
        chunks = [int(x) for x in a.chunks.split(",")]
        for r in range(a.reps):
            for m, ch in [(m, ch) for m in modes for ch in chunks]:
                call("dora_gpu_test_pack_tune", 0, -1, ch)
                call("dora_gpu_test_cp_lone", 1 if m == "cp" else 0)
                call("dora_gpu_test_pack_signal_tune", 0 if m in ("cp", "k1024") else int(m[1:]), 0)
                out = bench.run_sync_leg(node, send, wait_ack, seq, S, a.n)
                seq = out.pop("seq")
                out.pop("send_calls_us", None)
                print(json.dumps({"rep": r, "mode": m, "chunk": ch, **out}), flush=True)
        call("dora_gpu_test_cp_lone", 1)
        call("dora_gpu_test_pack_signal_tune", 0, 0)
        call("dora_gpu_test_pack_tune", 0, -1, 0)
        for b in bufs:
            b.free()
        stream.close()
        node.close()


if __name__ == "__main__":
    main()
