#!/usr/bin/env python3
"""Where a small device message's latency goes (verdict r04 item 1), in bench.py's shape: this
process's Python node sends to the native bench sink (dora-gpu-bench-sink, its own process) on
GPU 0, one synchronous send at a time, the metadata timestamp to the sink's receipt being the
latency the bench line reports.

Cases (one sink series each, told apart by size):
  * empty messages (no sample, no GPU) at 1 ms gaps: the host path alone;
  * device 8 B at 1 ms gaps (the bench's ladder), and device 16 / 24 / 32 B at 200 / 50 / 10 us
    gaps (spun, not slept): how much of the GPU round trip is the GPU waking from idle;
  * device 4096 B at 1 ms.
With the message trace (DORA_GPU_TRACE, every process of the dataflow) each device message is
split into host stages and GPU stages: launched (sender, after the AQL doorbell) -> first
workgroup start -> fill signal (the pack's own s_memrealtime stamps, mapped to the host clock by
the HSA runtime, aql.h aql_gpu_tick_to_realtime_ns) -> the sink observes the fill.

    python scripts/small_lat_probe.py --n 400 > small_lat.jsonl
"""
import argparse
import csv
import glob
import json
import os
import statistics
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

TRACE_DIR = tempfile.mkdtemp(prefix="dora-small-lat-")
os.environ["DORA_GPU_TRACE"] = TRACE_DIR  # read when the library loads, inherited by the dataflow

P = {"alloc_begin": 1, "alloc_end": 2, "launched": 3, "sent": 5, "routed": 7, "popped": 9,
     "filled": 10, "released": 11, "gpu_start": 12, "gpu_signal": 13}
# (label, size, gap_us, spin)
CASES = [("empty", 0, 1000, False), ("dev_gap1000", 8, 1000, False),
         ("dev_gap200", 16, 200, True), ("dev_gap50", 24, 50, True), ("dev_gap10", 32, 10, True),
         ("dev4096_gap1000", 4096, 1000, False)]


def spin(us):
    t = time.perf_counter() + us / 1e6
    while time.perf_counter() < t:
        pass


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=400)
    ap.add_argument("--keep-awake-us", type=float, default=None,
                    help="dora_gpu_set_keep_awake period (0: off; default: the library's)")
    a = ap.parse_args()
    from dora_amd import device
    from dora_amd.dataflow import Dataflow
    from dora_amd.node import Node

    tmp = tempfile.mkdtemp(prefix="dora-small-lat-res-")
    res = os.path.join(tmp, "sink.json")
    desc = {"nodes": [
        {"id": "node", "path": "dynamic", "outputs": ["latency", "throughput"],
         "inputs": {"ack": "sink/ack"}, "_unstable_deploy": {"gpu": 0}},
        {"id": "sink", "path": "dora-gpu-bench-sink", "outputs": ["ack"],
         "inputs": {"latency": {"source": "node/latency", "queue_size": 10},
                    "throughput": {"source": "node/throughput", "queue_size": 10}},
         "env": {"DORA_BENCH_RESULT": res}, "_unstable_deploy": {"gpu": 0}},
    ]}
    if a.keep_awake_us is not None:
        device.set_keep_awake(a.keep_awake_us)
    df = Dataflow(desc).start()
    node = Node("node", dataflow=df.shm, device=0)
    stream = device.Stream()
    buf = device.DeviceBuffer(4096)
    device.fill_splitmix(buf.ptr, 4096, 7, stream)
    stream.sync()
    seq = 0
    for _ in range(4):  # slots and the sink's mapping, untimed
        for _, z, _, _ in CASES:
            if z:
                node.send_output_device_bytes("throughput", buf.ptr, z, {"seq": seq})
                seq += 1
    node.send_output("throughput", b"", {"seq": seq, "ack": True})
    node.wait_input("ack", "seq", seq, 60.0)
    seq += 1
    t_case = {}
    for label, z, gap, spun in CASES:
        t0 = time.time_ns()
        for _ in range(a.n):
            if z:
                node.send_output_device_bytes("latency", buf.ptr, z,
                                              {"seq": seq, "t_start": time.time_ns()})
            else:
                node.send_output("latency", b"", {"seq": seq, "t_start": time.time_ns()})
            seq += 1
            spin(gap) if spun else time.sleep(gap / 1e6)
        t_case[label] = (t0, time.time_ns())
    node.send_output("throughput", b"", {"seq": seq, "ack": True})
    node.wait_input("ack", "seq", seq, 60.0)
    buf.free()
    stream.close()
    node.close()
    df.wait(30)
    df.stop()
    sink = json.load(open(res))
    series = {s["size"]: s for s in sink["series"] if s["input"] == "latency"}
    ev = {}
    for f in glob.glob(os.path.join(TRACE_DIR, "*.trace.csv")):
        for r in csv.DictReader(open(f)):
            ev.setdefault(r["token"], {}).setdefault(int(r["point"]), int(r["t_ns"]))
    for label, z, gap, _ in CASES:
        s = series.get(z, {})
        row = {"case": label,
               "keep_awake_us": a.keep_awake_us, "bytes": z, "gap_us": gap, "n": s.get("n"),
               "latency_p50_us": s.get("p50_us"), "latency_p99_us": s.get("p99_us"),
               "incl_send_p50_us": s.get("full_p50_us")}
        lo, hi = t_case[label]
        grp = [v for v in ev.values() if P["launched"] in v and lo <= v[P["launched"]] <= hi]
        if z and grp:
            def med(x, y):
                xs = [(v[P[y]] - v[P[x]]) / 1000 for v in grp if P[x] in v and P[y] in v]
                return round(statistics.median(xs), 3) if xs else None
            row["traced"] = len(grp)
            row["stages_p50_us"] = {
                "alloc": med("alloc_begin", "alloc_end"),
                "pack_launch": med("alloc_end", "launched"),
                "launched_to_sent": med("launched", "sent"),
                "sent_to_routed": med("sent", "routed"),
                "routed_to_popped": med("routed", "popped"),
                "popped_to_filled": med("popped", "filled"),
                "launched_to_filled": med("launched", "filled"),
                "gpu_dispatch": med("launched", "gpu_start"),
                "gpu_kernel": med("gpu_start", "gpu_signal"),
                "signal_to_observed": med("gpu_signal", "filled")}
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
