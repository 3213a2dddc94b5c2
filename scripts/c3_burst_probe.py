#!/usr/bin/env python3
"""The bench's C3 block alone (bench.run_c3_block: warm-up, 200-send steady region, 20-send
burst) `--reps` times in one dataflow, printing per rep the burst's send-call times, pack starts
and fraction of HBM; with DORA_GPU_TRACE=subphases the sender's host sub-phases follow at exit.
Diagnoses the burst's host stall with CP-signalled multi-segment packs.

    python scripts/c3_burst_probe.py --reps 3 [--grids 3584,1024,512]

With --grids, every rep runs once per workgroup cap of the command processor's packs
(dora_gpu_test_cp_grid: C3's clouds are CP-signalled), interleaved; --multi-grids caps only the
multi-segment ones (dora_gpu_test_cp_grid_multi) and --caps sets the sender's in-flight cap
from 8 MiB (dora_gpu_test_in_flight); every combination runs once per rep.
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
    ap.add_argument("--steady", type=int, default=200)
    ap.add_argument("--grids", default="0", help="CP grid caps to interleave (0: the default)")
    ap.add_argument("--multi-grids", default="0", help="multi-segment CP grid caps (0: the default, 640)")
    ap.add_argument("--caps", default="0", help="in-flight caps from 8 MiB (0: the default, 8)")
    ap.add_argument("--mid-queues", default="0",
                    help="queues taking 8-32 MiB packs (0: the default, 4; up to 8 are created)")
    a = ap.parse_args()
    import bench
    from dora_amd import device
    from dora_amd.dataflow import Dataflow
    from dora_amd.node import Node
    res = os.path.join(tempfile.mkdtemp(prefix="dora-c3-burst-"), "sink.json")
    desc = {"nodes": [
        {"id": "node", "path": "dynamic", "outputs": ["throughput"], "inputs": {"ack": "sink/ack"}},
        {"id": "sink", "path": "dora-gpu-bench-sink", "outputs": ["ack"],
         "inputs": {"throughput": {"source": "node/throughput", "queue_size": 10}},
         "env": {"DORA_BENCH_RESULT": res}},
    ]}
    mids = [int(x) for x in a.mid_queues.split(",")]
    from dora_amd._lib import call
    if max(mids) > 4:
        call("dora_gpu_test_mid_queues", max(mids), 0)  # before this process's first AQL use
    with Dataflow(desc) as df:
        node = Node("node", dataflow=df.shm, device=0)
        node.set_async_sends(True)
        stream = device.Stream()
        seq = 0

        def wait_ack(s, timeout=60.0):
            node.wait_input("ack", "seq", s, timeout)

        grids = [int(x) for x in a.grids.split(",")]
        multis = [int(x) for x in a.multi_grids.split(",")]
        caps = [int(x) for x in a.caps.split(",")]
        combos = [(r, g, m, c, q) for r in range(a.reps) for g in grids for m in multis
                  for c in caps for q in mids]
        for r, g, m, c, q in combos:
            call("dora_gpu_test_mid_queues", 0, q if q else 4)
            call("dora_gpu_test_cp_grid", g)
            call("dora_gpu_test_cp_grid_multi", m)
            call("dora_gpu_test_in_flight", 0, c)
            seq, c3 = bench.run_c3_block(node, stream, wait_ack, seq, steady_steps=a.steady)
            print(json.dumps({"rep": r, "cp_grid": g, "multi_grid": m, "big_cap": c, "mid_queues": q,
                              "frac": c3["roofline"]["frac"],
                              "steady_frac": (c3["steady"] or {}).get("frac"),
                              "us_per_cloud": c3["roofline"]["device_us_per_launch"],
                              "send_calls_us": c3["send_calls_us"],
                              "pack_intervals_us": c3["pack_intervals_us"],
                              "cp_signalled": device.aql_cp_signalled(0)}), flush=True)
        call("dora_gpu_test_cp_grid", 0)
        call("dora_gpu_test_cp_grid_multi", 0)
        call("dora_gpu_test_in_flight", 0, 0)
        stream.close()
        node.close()
        df.wait(60)


if __name__ == "__main__":
    main()
