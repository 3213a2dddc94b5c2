#!/usr/bin/env python3
"""bench.py — node->node device data plane on MI355X (BASELINE.json metric).

One rank per GPU.  Each rank runs its own local dataflow on its GPU (weak scaling: dataflow
graphs shard by node placement, SURVEY.md §8e — no data-path collective):

    node (this process, `path: dynamic`) --latency/throughput--> sink (dora-gpu-bench-sink)
         ^------------------------------------ ack ---------------------------------'

A step = one message of `--size` bytes (default 40,960,000 B, the top of the C2 ladder) sent
with `send_output_raw` semantics: allocate a device slot (20-entry recycled cache), HIP pack
kernel HBM->HBM from the node's device-resident source, descriptor through the daemon, IPC-mapped
zero-copy delivery at the sink, drop token back.  The timed region is K back-to-back steps
closed by the sink's ack of the last one, bracketed by barrier + device sync.

value = total payload bytes delivered by all ranks / max-over-ranks time (GB/s).
The JSON line also carries the per-size latency ladder (p50/p99, reference semantics: timestamp
after the fill), the pack-kernel roofline (HIP events on the node stream) and the CPU baseline
(C++ restatement of the reference shm path, oracle/build/shm_baseline, rank 0 at N=1).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
LADDER = [4096, 16384, 40960, 65536, 409600, 1 << 20, 4096000, 4 << 20, 16 << 20, 40960000]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--size", type=int, default=40960000)
    ap.add_argument("--workload", choices=["c2", "c3"], default="c2",
                    help="c2: UInt8 payloads (BASELINE configs[1], default); c3: nested "
                         "List<Struct<x,y,z,intensity>> 1M-point clouds (configs[2])")
    ap.add_argument("--lat-n", type=int, default=50, help="latency-mode messages per size")
    ap.add_argument("--lat-gap-us", type=int, default=1000)
    ap.add_argument("--no-ladder", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--sources", type=int, default=0, help="rotating source buffers (0: auto)")
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="skip the per-launch kernel stamps (roofline then unmeasured)")
    return ap.parse_args()


class Ranks:
    """Cross-rank control for the weak-scaled replicas: barrier and max/sum of scalars over a
    gloo (CPU) process group — the data path itself has no collective."""

    def __init__(self, world: int):
        self.dist = None
        if world > 1:
            import torch.distributed as dist
            if not dist.is_initialized():
                dist.init_process_group("gloo")
            self.dist = dist

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def _reduce(self, x: float, op) -> float:
        if self.dist is None:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=op)
        return float(t.item())

    def max(self, x: float) -> float:
        return self._reduce(x, self.dist.ReduceOp.MAX) if self.dist else x

    def sum(self, x: float) -> float:
        return self._reduce(x, self.dist.ReduceOp.SUM) if self.dist else x


def pmc_traffic(msg_bytes: int):
    """HBM bytes per pack launch from the newest committed PMC run for this message size
    (profiles/*pack_pmc_traffic.json, FETCH_SIZE x2 + WRITE_SIZE per MI355X_MICROARCH.md)."""
    import glob
    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pack_pmc_traffic.json"))):
        try:
            d = json.load(open(p))
        except (OSError, ValueError):
            continue
        if d.get("algorithmic_bytes_per_launch") == 2 * msg_bytes:
            best = (os.path.basename(p), d["traffic_bytes_per_launch"])
    return best


def cpu_baseline(rank_cores):
    """Reference shm path restated in C++ (oracle/shm_baseline.cpp), bounded sample."""
    exe = os.path.join(ROOT, "oracle", "build", "shm_baseline")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    cores = ",".join(str(c) for c in rank_cores[:3])
    sizes = "4096,40960,409600,4096000,40960000"
    out = subprocess.run([exe, "--sizes", sizes, "--lat-n", "20", "--lat-gap-us", "10000",
                          "--tp-n", "40", "--cores", cores], capture_output=True, text=True,
                         timeout=300, check=True).stdout
    return json.loads(out)


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    affinity = sorted(os.sched_getaffinity(0))

    # ---- CPU-only work and process spawning first: nothing below touches HIP until Node() ----
    base = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        base = cpu_baseline(affinity)

    from dora_amd.dataflow import Dataflow
    result_path = os.path.join(tempfile.mkdtemp(prefix="dora-bench-"), "sink.json")
    desc = {"nodes": [
        {"id": "node", "path": "dynamic", "outputs": ["latency", "throughput"],
         "inputs": {"ack": "sink/ack"}, "_unstable_deploy": {"gpu": local_rank}},
        {"id": "sink", "path": "dora-gpu-bench-sink", "outputs": ["ack"],
         "inputs": {"latency": {"source": "node/latency", "queue_size": 10},
                    "throughput": {"source": "node/throughput", "queue_size": 10}},
         "env": {"DORA_BENCH_RESULT": result_path}, "_unstable_deploy": {"gpu": local_rank}},
    ]}
    df = Dataflow(desc).start()

    ranks = Ranks(world)
    barrier, max_over_ranks, sum_over_ranks = ranks.barrier, ranks.max, ranks.sum

    from dora_amd import device
    from dora_amd.node import Node
    from dora_amd.verify import to_i64
    from dora_amd.workloads import payload_seed

    node = Node("node", dataflow=df.shm, device=local_rank)
    stream = device.Stream()
    if args.workload == "c2":
        S = args.size
        nsrc = args.sources or max(2, min(16, (640 << 20) // max(S, 1)))
        srcs = []
        for _ in range(nsrc):  # rotate > 512 MiB of sources so the Infinity Cache cannot hold them
            b = device.DeviceBuffer(S)
            device.fill_splitmix(b.ptr, S, payload_seed(S), stream)
            srcs.append(b)
        stream.sync()
        csum = device.csum64(srcs[0].ptr, S, stream)

        def send(k, meta):
            node.send_output_device_bytes("throughput", srcs[k % nsrc].ptr, S, meta)
    else:
        # C3: List<Struct<x,y,z:f32,intensity:u8>> 1M-point clouds resident in HBM; each send is
        # plan (host DFS + validity read-back for the type info) + nested pack kernel
        from dora_amd.arrow_utils import Plan
        from dora_amd.device import DeviceArray
        from dora_amd.workloads import point_cloud
        cloud = point_cloud()
        nsrc = args.sources or 24
        srcs = [DeviceArray.from_pyarrow(cloud) for _ in range(nsrc)]
        with Plan.of(srcs[0]) as p:
            S = p.size
            ref = device.DeviceBuffer(S)
            p.pack(ref.ptr, S, stream)
            stream.sync()
        csum = device.csum64(ref.ptr, S, stream)
        ref.free()

        def send(k, meta):
            node.send_output("throughput", srcs[k % nsrc], meta)

    def wait_ack(seq, timeout=60.0):
        deadline = time.time() + timeout
        while time.time() < deadline:
            ev = node.next(timeout=1.0)
            if ev and ev["type"] == "INPUT" and ev["id"] == "ack" and \
                    ev["metadata"].get("seq") == seq:
                return True
        raise RuntimeError(f"no ack for seq {seq}")

    # ---- warmup (the first messages are verified bit-exact by the sink's csum kernel) ----
    seq = 0
    for k in range(args.warmup):
        meta = {"seq": seq, "t_start": time.time_ns()}
        if k < 3:
            meta.update({"csum": to_i64(csum), "verify": True})
        send(k, meta)
        seq += 1
    node.send_output("throughput", b"", {"seq": seq, "ack": True})
    wait_ack(seq)
    seq += 1

    # ---- latency ladder (reference latency mode: spaced messages, output `latency`) ----
    ladder_bufs = {}
    if not args.no_ladder:
        for size in LADDER:
            b = device.DeviceBuffer(size)
            device.fill_splitmix(b.ptr, size, payload_seed(size), stream)
            ladder_bufs[size] = b
        stream.sync()
        for size in LADDER:
            for _ in range(args.lat_n):
                node.send_output_device_bytes("latency", ladder_bufs[size].ptr, size,
                                              {"seq": seq, "t_start": time.time_ns()})
                seq += 1
                time.sleep(args.lat_gap_us / 1e6)
        node.send_output("throughput", b"", {"seq": seq, "ack": True})
        wait_ack(seq)
        seq += 1
        for b in ladder_bufs.values():
            b.free()

    # ---- timed region: K back-to-back steps, closed by the sink's ack ----
    node.set_profiling(not args.no_kernel_timing)
    barrier()
    device.set_device(local_rank)
    from dora_amd._lib import call
    call("dora_gpu_device_sync")
    t0 = time.perf_counter()
    for k in range(args.steps):
        send(k, {"seq": seq, "t_start": time.time_ns()})
        seq += 1
    node.send_output("throughput", b"", {"seq": seq, "ack": True})
    wait_ack(seq)
    call("dora_gpu_device_sync")
    elapsed = time.perf_counter() - t0
    barrier()
    pack = node.pack_stats()
    stats = node.stats()
    stats["send_phase_us"] = {k: round(v, 2) for k, v in node.send_profile().items()}
    node.close()
    codes = df.wait(120)
    df.stop()
    sink = json.load(open(result_path)) if os.path.exists(result_path) else {"series": []}

    t_max = max_over_ranks(elapsed)
    total_bytes = sum_over_ranks(float(args.steps * S))
    value = total_bytes / t_max / 1e9
    avg_pack_ms = pack["total_ms"] / max(pack["count"], 1)
    achieved = 2.0 * S / (avg_pack_ms * 1e-3) / 1e9 if pack["count"] else 0.0

    if rank != 0:
        return
    traffic = pmc_traffic(S)
    lat = {}
    for s in sink.get("series", []):
        if s["input"] == "latency":
            lat[str(s["size"])] = {"p50_us": s["p50_us"], "p99_us": s["p99_us"],
                                   "p50_incl_pack_us": s["full_p50_us"],
                                   "p99_incl_pack_us": s["full_p99_us"], "n": s["n"]}
    verified = sum(s["verified"] for s in sink.get("series", []))
    mismatches = sum(s["mismatches"] for s in sink.get("series", []))
    if args.workload == "c2":
        metric = f"node->node GB/s ({S:,} B UInt8 samples) + p50/p99 latency per msg size"
        workload = ("C2: examples/benchmark node->sink edge, device-resident UInt8 samples, "
                    "1 node + 1 sink per GPU")
        data = "synthetic (splitmix64 payloads, seed 0xD05A + size)"
    else:
        metric = "node->node GB/s (List<Struct<x,y,z:f32,intensity:u8>> 1M points) + latency"
        workload = ("C3: nested Arrow packing, 1M-point clouds in 16 lists with validity "
                    "bitmaps, node->sink edge per GPU")
        data = "synthetic (seeded point clouds, dora_amd.workloads.point_cloud)"
    line = {
        "metric": metric,
        "value": round(value, 3), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(t_max / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": data,
        "config": {"workload": workload,
                   "msg_bytes": S, "parallelism": f"dp{world} (one dataflow per GPU)",
                   "sources_rotated": nsrc},
        "latency_us": lat,
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                     "traffic": traffic[1] if traffic else None,
                     "traffic_source": traffic[0] if traffic else None, "kernel": "pack_kernel",
                     "avg_kernel_us": round(avg_pack_ms * 1e3, 3),
                     "kernel_stamps": pack["count"],
                     "timing": "hipExtLaunchKernel start/stop stamps on the node stream, every "
                               "8th pack of the timed region (DORA_GPU_TIMING_SAMPLE)",
                     "algorithmic_bytes_per_launch": 2 * S},
        "parity": {"verified_msgs": verified, "mismatches": mismatches},
        "sink_us": {"next_event": sink.get("next_event_us"), "free": sink.get("free_us")},
        "node_stats": stats, "exit_codes": codes,
    }
    if base is not None:
        tp = [s for s in base["series"] if s["mode"] == "throughput" and s["size"] == 40960000]
        line["cpu_baseline"] = {
            "value": tp[0]["GBps"] if tp else None, "unit": "GB/s", "cores": 3, "kind": "port",
            "sample": "reference shm path restated in C++ (sender/daemon/sink pinned to 3 cores,"
                      " TCP control, F8 daemon copy): 20 latency + 40 throughput msgs per size "
                      "in {4096, 40960, 409600, 4096000, 40960000}",
            "latency_us": {str(s["size"]): {"p50_us": s["p50_us"], "p99_us": s["p99_us"]}
                           for s in base["series"] if s["mode"] == "latency"},
            "wall_s": base["wall_s"], "nproc": base["nproc"], "cores_used": base["cores"]}
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
